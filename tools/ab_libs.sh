#!/bin/bash
# GPU box: run one measurement command against several builds of libprpe.so in turn (A/B of a
# kernel change; the variants are tools/abl/libprpe_<V>.so from tools/rev_variant_build.py or
# the ablation builders, linked with the shipped build_info.o). HEAD = the shipped library.
#   bash tools/ab_libs.sh TAG "bnprev HEAD" python3 tools/bneck_bench.py --batch 256 --fused-only
# Output: gpurun_out/TAG_ab.txt. Each run is time-limited; the shipped library is restored.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out; mkdir -p $O
TAG=$1; VARS=$2; shift 2
L=person-recognition-for-pose-estimation_amd/prpe/libprpe.so
cp $L /tmp/libprpe_orig.so || exit 9
rc=0
for k in $VARS; do
  if [ $k = HEAD ]; then cp /tmp/libprpe_orig.so $L || exit 9; else cp tools/abl/libprpe_$k.so $L || exit 9; fi
  echo "== lib $k: $*"
  timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids
  rc=$?
  [ $rc -ne 0 ] && break
done > $O/${TAG}_ab.txt 2>&1
cp /tmp/libprpe_orig.so $L
cat $O/${TAG}_ab.txt
exit $rc
