#!/bin/bash
# round 3: fused bottleneck micro-bench + its counters
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -v -s --timeout 120 --timeout-method thread > $O/r03e_bneck_tests.log 2>&1 || exit 9
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 > $O/r03e_bneck_bench.txt 2>&1 || exit 1
ARGS="tools/bneck_bench.py --batch 64 --iters 2 --fused-only"
timeout -k 10 240 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d $O/r03e_pmc -o pmc -- python3 $ARGS > $O/r03e_pmc.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/r03e_pmc_w -o pmc -- python3 $ARGS > $O/r03e_pmc_w.log 2>&1 || exit 3
python tools/pmc_summary.py $O/r03e_pmc --kernel bneck --min-us 300 > $O/r03e_pmc_bneck.txt
python tools/pmc_summary.py $O/r03e_pmc_w --kernel bneck --min-us 300 >> $O/r03e_pmc_bneck.txt
rm -rf $O/r03e_pmc $O/r03e_pmc_w
