#!/bin/bash
# GPU-box script: PMC passes (tools/pmc_upconv.txt) of the fused upconv kernel per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in ${ABLS:-8 12}; do
  rm -rf gpurun_out/uppmc_$a
  PRPE_UPCONV_ABL=$a timeout -k 10 300 rocprofv3 -i tools/pmc_upconv.txt --kernel-trace -d gpurun_out/uppmc_$a -o pmc -- python3 tools/upconv_bench.py --batch 64 --iters 1 --fused-only > gpurun_out/uppmc_$a.log 2>&1 || { tail -30 gpurun_out/uppmc_$a.log; exit 1; }
  echo "== ABL $a"
  python tools/pmc_summary.py gpurun_out/uppmc_$a --kernel "upconv" --min-us 200 | tee gpurun_out/uppmc_$a.txt
  find gpurun_out/uppmc_$a -name "*.db" -delete
done
