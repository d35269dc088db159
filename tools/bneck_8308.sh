#!/bin/bash
# GPU box: test_gpu_bneck.py on each 8308d2f variant (tools/bneck_8308_variants.py), the shipped
# library last. Measurement only; results in gpurun_out/TAG_8308.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out; mkdir -p $O
TAG=${1:-r05}; VARS=${2:-"A B C D"}
L=person-recognition-for-pose-estimation_amd/prpe/libprpe.so
cp $L /tmp/libprpe_orig.so || exit 9
for k in $VARS HEAD; do
  if [ $k = HEAD ]; then cp /tmp/libprpe_orig.so $L || exit 9; else cp tools/abl/libprpe_8308$k.so $L || exit 9; fi
  echo "== variant $k"
  timeout -k 10 300 python3 -m pytest tests/test_gpu_bneck.py -m gpu -q --tb=line -p no:cacheprovider --timeout 120 \
    --timeout-method thread 2>&1 | grep -v amdgpu | tail -25
  rc=$?
  [ $rc -ge 124 ] && break
done > $O/${TAG}_8308.txt 2>&1
cp /tmp/libprpe_orig.so $L
cat $O/${TAG}_8308.txt
