#!/bin/bash
# GPU-box script: fused upconv block order (PRPE_UPCONV_XCD) x row run (PRPE_UPCONV_R) sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/upsweep.txt
: > $out
for x in ${XCDS:-0 1}; do
  for r in ${RS:-256 64 32 16}; do
    echo "== XCD=$x R=$r" >> $out
    PRPE_UPCONV_XCD=$x PRPE_UPCONV_R=$r timeout -k 10 200 python tools/upconv_bench.py --batch 64 --iters 5 --fused-only > gpurun_out/upsweep_1.txt 2>&1 || { tail -20 gpurun_out/upsweep_1.txt; exit 1; }
    grep -v "amdgpu.ids\|copy\|head" gpurun_out/upsweep_1.txt >> $out
  done
done
cat $out
