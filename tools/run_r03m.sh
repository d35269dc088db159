#!/bin/bash
# round 3: double-buffered W3 parts in the layer2 fused block: op tests + micro-bench + bench
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > $O/r03m_bneck_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --mid 128 --fused-only > $O/r03m_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03m_bench.json 2> $O/r03m_bench.err || exit 3
