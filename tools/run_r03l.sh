#!/bin/bash
# round 3: fused identity bottleneck generalised to layer2 (mid 128, 160-KB workgroup): op
# tests, micro-bench, model parity + A/B
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bneck.py -x -v -s --timeout 120 --timeout-method thread > $O/r03l_bneck_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --mid 128 > $O/r03l_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only >> $O/r03l_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only --proj >> $O/r03l_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_contracts.py -x -q --timeout 300 --timeout-method thread > $O/r03l_model.log 2>&1 || exit 3
for D in 1 0; do
  PRPE_BNECK_L2=$D timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03l_bench_l2$D.json 2> $O/r03l_bench_l2$D.err || exit 4
done
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 60 > $O/r03l_layer_profile.txt 2>&1 || exit 5
