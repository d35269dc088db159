#!/bin/bash
# round 3: transposed fused bottleneck (tests + micro-bench + counters) and the 16x16 taps tile
# of the dominant launch (time + HBM traffic)
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -v -s --timeout 120 --timeout-method thread > $O/r03f_bneck_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 > $O/r03f_bneck_bench.txt 2>&1 || exit 2
CB="tools/conv_bench.py --only vit_adapter.7 --prec 0 --korders 1 --batch 256 --planes --act gelu --taps 27"
timeout -k 10 300 python $CB --tiles 0,32,0,32 --iters 5 > $O/r03f_cb_taps16.txt 2>&1 || exit 3
ARGS="tools/bneck_bench.py --batch 64 --iters 2 --fused-only"
timeout -k 10 240 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d $O/r03f_pmc -o pmc -- python3 $ARGS > $O/r03f_pmc.log 2>&1 || exit 4
python tools/pmc_summary.py $O/r03f_pmc --kernel bneck --min-us 300 > $O/r03f_pmc_bneck.txt
rm -rf $O/r03f_pmc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d $O/r03f_tr_$C -o pmc -- python3 $CB --tiles 32 --iters 2 > $O/r03f_tr_$C.log 2>&1 || exit 5
done
python tools/pmc_summary.py $O/r03f_tr_FETCH_SIZE --kernel conv_halo --min-us 5000 > $O/r03f_traffic_taps16.txt
python tools/pmc_summary.py $O/r03f_tr_WRITE_SIZE --kernel conv_halo --min-us 5000 >> $O/r03f_traffic_taps16.txt
rm -rf $O/r03f_tr_FETCH_SIZE $O/r03f_tr_WRITE_SIZE
