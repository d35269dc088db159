#!/bin/bash
# round 3: fused bottleneck with the balanced phase-1 wave map: op tests, micro-bench, model, bench
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > $O/r03s_bneck_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only > $O/r03s_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only --proj >> $O/r03s_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only --mid 128 >> $O/r03s_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > $O/r03s_model.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03s_bench.json 2> $O/r03s_bench.err || exit 4
