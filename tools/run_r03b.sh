#!/bin/bash
# round 3: LDS-DMA upconv -- op tests, then the upconv micro-bench and the per-layer profile
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "upconv or planes or smallco" > $O/r03b_ops.log 2>&1 || exit 1
timeout -k 10 200 python tools/upconv_bench.py --fused-only --batch 64 > $O/r03b_upconv_bench.txt 2>&1 || exit 2
PRPE_UPCONV_DMA=0 timeout -k 10 200 python tools/upconv_bench.py --fused-only --batch 64 > $O/r03b_upconv_bench_fused.txt 2>&1 || exit 3
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 300 > $O/r03b_layer_profile.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03b_bench.json 2> $O/r03b_bench.err || exit 5
