#!/bin/bash
# round 3: fused bottleneck with the 4-stage W ring and A two K-steps ahead (tests, micro-bench, counters)
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -v -s --timeout 120 --timeout-method thread > $O/r03g_bneck_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 > $O/r03g_bneck_bench.txt 2>&1 || exit 2
CB="tools/conv_bench.py --only vit_adapter.7 --prec 0 --korders 1 --batch 256 --planes --act gelu --taps 27"
ARGS="tools/bneck_bench.py --batch 64 --iters 2 --fused-only"
timeout -k 10 240 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d $O/r03g_pmc -o pmc -- python3 $ARGS > $O/r03g_pmc.log 2>&1 || exit 4
python tools/pmc_summary.py $O/r03g_pmc --kernel bneck --min-us 300 > $O/r03g_pmc_bneck.txt
rm -rf $O/r03g_pmc
