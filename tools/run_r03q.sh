#!/bin/bash
# round 3: attention K rows at a 160-B pitch (tests, micro-bench, LDS counters) and the
# BASELINE config-2 / config-3 bench lines on the current tree
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "attention" > $O/r03q_attn_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/attn_bench.py > $O/r03q_attn_bench.txt 2>&1 || exit 2
timeout -k 10 240 rocprofv3 -i tools/pmc_attn.txt --kernel-trace -d $O/r03q_pmc -o pmc -- python3 tools/attn_bench.py --iters 2 > $O/r03q_pmc.log 2>&1 || exit 3
python tools/pmc_summary.py $O/r03q_pmc --kernel vit_attention --min-us 50 > $O/r03q_pmc_attn.txt
rm -rf $O/r03q_pmc
timeout -k 10 300 python bench.py --config vitpose --steps 20 --warmup 3 > $O/r03q_bench_vitpose.json 2> $O/r03q_bench_vitpose.err || exit 4
timeout -k 10 300 python bench.py --config yolo_face --steps 20 --warmup 3 > $O/r03q_bench_yolo_face.json 2> $O/r03q_bench_yolo_face.err || exit 5
