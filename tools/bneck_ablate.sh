#!/bin/bash
# Phase-cost ablation of the fused bottleneck (GPU box; measurement only, results are WRONG by
# design): tools/abl/libprpe_ablK.so are builds of conv_bneck.hip with -DPRPE_BNECK_ABLATE=K from
# a scratch copy whose phase-K MFMAs are compiled out (1: phase 2, 2: phase 1, 3: phase 3,
# 4: all three); each replaces the box copy's libprpe.so in turn (same source hash) for
# tools/bneck_bench.py --fused-only. Baseline first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out; mkdir -p $O
L=person-recognition-for-pose-estimation_amd/prpe/libprpe.so
cp $L /tmp/libprpe_orig.so || exit 9
for k in 0 1 2 3 4; do
  [ $k -gt 0 ] && { cp tools/abl/libprpe_abl$k.so $L || exit 9; }
  for mid in 64 128; do
    echo "== ablate $k mid $mid"
    timeout -k 10 120 python3 tools/bneck_bench.py --batch 256 --iters 10 --fused-only --mid $mid || exit 8
  done
done > $O/r04_bneck_ablate.txt 2>&1
rc=$?
cp /tmp/libprpe_orig.so $L
cat $O/r04_bneck_ablate.txt | grep -v amdgpu
exit $rc
