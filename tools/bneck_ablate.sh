#!/bin/bash
# Phase-cost ablation of the fused bottleneck (GPU box; measurement only, results are WRONG by
# design): tools/abl/libprpe_ablK.so are builds of conv_bneck.hip with parts compiled out
# (tools/bneck_ablate_build.py, run in the container: 1 phase-2 MFMAs, 2 phase-1 MFMAs, 3 phase-3
# MFMAs, 4 all MFMAs, 5 all MFMAs + the W1/W2/W3 LDS-DMA, 6 the W LDS-DMA only, 7 all MFMAs +
# the phase-1 x loads); each replaces the box copy's libprpe.so in turn (same source hash) for
# tools/bneck_bench.py --fused-only. Baseline (0) first.
#   bash tools/bneck_ablate.sh TAG "0 4 5 6 7"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out; mkdir -p $O
TAG=${1:-r05}; VARS=${2:-"0 1 2 3 4 5 6 7"}
L=person-recognition-for-pose-estimation_amd/prpe/libprpe.so
cp $L /tmp/libprpe_orig.so || exit 9
for k in $VARS; do
  if [ $k -gt 0 ]; then cp tools/abl/libprpe_abl$k.so $L || exit 9; else cp /tmp/libprpe_orig.so $L || exit 9; fi
  for mid in 64 128; do
    echo "== ablate $k mid $mid"
    timeout -k 10 120 python3 tools/bneck_bench.py --batch 256 --iters 10 --fused-only --mid $mid || exit 8
  done
  echo "== ablate $k proj"
  timeout -k 10 120 python3 tools/bneck_bench.py --batch 256 --iters 10 --fused-only --proj || exit 8
done > $O/${TAG}_bneck_ablate.txt 2>&1
rc=$?
cp /tmp/libprpe_orig.so $L
grep -v amdgpu $O/${TAG}_bneck_ablate.txt
exit $rc
