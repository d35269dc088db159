#!/bin/bash
# round 3 (final): full GPU suite + smoke + bench line on the committed tree
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r03t_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r03t_smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py > $O/r03t_bench_default.json 2> $O/r03t_bench_default.err || exit 3
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/r03t_bench.json 2> $O/r03t_bench.err || exit 4
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 300 > $O/r03t_layer_profile.txt 2>&1 || exit 5
