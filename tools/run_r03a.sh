#!/bin/bash
# round 3, first GPU pass: halo-kernel op tests first (fast failure), the whole -m gpu suite,
# the per-layer profile and the benches. Every GPU step has its own time limit; stop at the
# first failure.
set -o pipefail
O=gpurun_out
mkdir -p $O
#timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "halo or wave or psa or dual or f16" > $O/r03a_halo_ops.log 2>&1 || exit 1
#timeout -k 10 840 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/r03a_gpu_tests.log 2>&1 || exit 2
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 200 > $O/r03a_layer_profile.txt 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/r03a_bench.json 2> $O/r03a_bench.err || exit 4
timeout -k 10 200 python bench.py --config yolo_raw --steps 10 --warmup 2 > $O/r03a_bench_yolo_raw.json 2> $O/r03a_bench_yolo_raw.err || exit 5
