#!/bin/bash
# round 3: fused bottleneck with the W-DMA / A-load issue order pinned: tests, model, bench
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > $O/r03z_bneck_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only > $O/r03z_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_contracts.py -x -q --timeout 300 --timeout-method thread > $O/r03z_model.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03z_bench.json 2> $O/r03z_bench.err || exit 4
