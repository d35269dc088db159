#!/bin/bash
# round 3: PMC counters of the fused trunk launches (bottleneck family, stem + max-pool) inside
# a sequential bs=64 forward, and their HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
ARGS="tools/layer_profile.py --batch 64 --top 5"
timeout -k 10 300 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d $O/r03u_pmc -o pmc -- python3 $ARGS > $O/r03u_pmc.log 2>&1 || exit 1
python tools/pmc_summary.py $O/r03u_pmc --kernel bneck_kernel --min-us 300 > $O/r03u_pmc_fused.txt
python tools/pmc_summary.py $O/r03u_pmc --kernel stem_pool --min-us 300 >> $O/r03u_pmc_fused.txt
rm -rf $O/r03u_pmc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $O/r03u_tr_$C -o pmc -- python3 $ARGS > $O/r03u_tr_$C.log 2>&1 || exit 2
  python tools/pmc_summary.py $O/r03u_tr_$C --kernel bneck_kernel --min-us 300 > $O/r03u_traffic_$C.txt
  python tools/pmc_summary.py $O/r03u_tr_$C --kernel stem_pool --min-us 300 >> $O/r03u_traffic_$C.txt
  rm -rf $O/r03u_tr_$C
done
