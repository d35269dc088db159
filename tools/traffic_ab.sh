#!/bin/bash
# GPU box: HBM-side traffic and time of the dominant launch (vit_pose.adapter.7, conv_halo,
# bs = 256) for several builds of libprpe.so (tools/abl/libprpe_<V>.so; HEAD = shipped): per
# build, tools/conv_bench.py's time, then one rocprofv3 pass each of FETCH_SIZE and TCC_HIT/MISS
# (separate --pmc runs, kernel trace only). Output gpurun_out/TAG_traffic_ab.txt.
#   bash tools/traffic_ab.sh TAG "HEAD halont"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out; mkdir -p $O
TAG=$1; VARS=$2
L=person-recognition-for-pose-estimation_amd/prpe/libprpe.so
cp $L /tmp/libprpe_orig.so || exit 9
CB=(tools/conv_bench.py --only vit_adapter.7 --prec 0 --tiles 0 --korders 1 --batch 256 --planes --act gelu --taps 27)
rc=0
for k in $VARS; do
  if [ $k = HEAD ]; then cp /tmp/libprpe_orig.so $L || exit 9; else cp tools/abl/libprpe_$k.so $L || exit 9; fi
  echo "== lib $k"
  timeout -k 10 200 python3 "${CB[@]}" --iters 5 2>&1 | grep -v amdgpu.ids || { rc=1; break; }
  for C in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    D=$O/${TAG}_${k}_pmc
    rm -rf $D
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $D -o pmc -- python3 "${CB[@]}" --iters 2 > $D.log 2>&1 || { rc=2; break 2; }
    python3 tools/pmc_summary.py $D --kernel conv_halo --min-us 5000 | grep -v "^#"
    rm -rf $D
  done
done > $O/${TAG}_traffic_ab.txt 2>&1
cp /tmp/libprpe_orig.so $L
cat $O/${TAG}_traffic_ab.txt
exit $rc
