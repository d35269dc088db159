#!/bin/bash
# round 3: after fencing every wait_barrier with sched_barrier (no LDS read hoisted above an
# s_barrier): determinism + batch independence, fused bottleneck speed, full GPU suite, bench
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/batch_indep_diag.py --batch 256 --frame 127 --concurrent 0 > $O/r03j_diag.txt 2>&1 || exit 1
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 > $O/r03j_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r03j_gpu_tests.log 2>&1 || exit 3
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/r03j_bench.json 2> $O/r03j_bench.err || exit 4
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 300 > $O/r03j_layer_profile.txt 2>&1 || exit 5
