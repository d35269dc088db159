#!/bin/bash
# GPU-box script: HBM traffic of the bench's dominant kernel (vit_pose.adapter.7, 3x3 256->128 at
# 256x192, bs=256, precision 0, auto tile) from PMC counters, one pass per counter
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass), kernel-trace only. The
# input is in the planes format, as the model feeds this conv (upconv writes it).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-traffic}
export TMPDIR=/tmp
ARGS="tools/conv_bench.py --only vit_adapter.7 --prec 0 --tiles 0 --korders 1 --batch 256 --iters 2 --planes"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${TAG}_$C -o pmc -- python3 $ARGS > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG}_$C.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_${TAG}_FETCH_SIZE --kernel conv_wave --min-us 1000
python tools/pmc_summary.py gpurun_out/pmc_${TAG}_WRITE_SIZE --kernel conv_wave --min-us 1000
