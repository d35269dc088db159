#!/bin/bash
# round 3: fused stem + max-pool -- op tests (bit identity vs the unfused pair), model parity,
# bench A/B, per-layer profile
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stem.py -x -v -s --timeout 200 --timeout-method thread > $O/r03n_stem_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_contracts.py -x -q --timeout 300 --timeout-method thread > $O/r03n_model.log 2>&1 || exit 3
for D in 1 0; do
  PRPE_STEM_POOL=$D timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03n_bench_sp$D.json 2> $O/r03n_bench_sp$D.err || exit 4
done
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 300 > $O/r03n_layer_profile.txt 2>&1 || exit 5
