#!/bin/bash
# GPU-box script: upconv fused-kernel ablation (no z loads / no stores) on the adapters' shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for a in ${ABLS:-0 4 8 12}; do
  echo "== PRPE_UPCONV_ABL=$a"
  PRPE_UPCONV_ABL=$a timeout -k 10 200 python tools/upconv_bench.py --batch 64 --iters 5 --fused-only > gpurun_out/upabl_$a.txt 2>&1 || { tail -20 gpurun_out/upabl_$a.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/upabl_$a.txt
done
