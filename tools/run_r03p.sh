#!/bin/bash
# round 3: stem + pool on 40-column strips (11 waves): tests, A/B vs the unfused pair, profile
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stem.py -x -q --timeout 200 --timeout-method thread > $O/r03p_stem_tests.log 2>&1 || exit 1
for D in 1 0; do
  PRPE_STEM_POOL=$D timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03p_bench_sp$D.json 2> $O/r03p_bench_sp$D.err || exit 4
done
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 20 > $O/r03p_layer_profile.txt 2>&1 || exit 5
