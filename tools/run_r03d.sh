#!/bin/bash
# round 3: fused bottleneck -- op tests, model tests, per-layer profile, bench
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u tools/bneck_diag.py > $O/r03d_diag.txt 2>&1 || exit 5
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -v -s --timeout 120 --timeout-method thread > $O/r03d_bneck.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_contracts.py -x -q --timeout 300 --timeout-method thread > $O/r03d_model.log 2>&1 || exit 2
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 300 > $O/r03d_layer_profile.txt 2>&1 || exit 3
for D in 1 0; do
  PRPE_BNECK_FUSE=$D timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03d_bench_f$D.json 2> $O/r03d_bench_f$D.err || exit 4
done
