#!/bin/bash
# GPU-box script: per-layer ViT GEMM times in the model with the GEMM kernel on / off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-vitab}
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 400 > gpurun_out/${TAG}_on.txt 2>&1 || { tail -30 gpurun_out/${TAG}_on.txt; exit 1; }
PRPE_CONV_GEMM=0 timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 400 > gpurun_out/${TAG}_off.txt 2>&1 || { tail -30 gpurun_out/${TAG}_off.txt; exit 1; }
for f in on off; do echo "== $f"; grep "layer\.[05]:\|adapter.7 \|adapter.0 \|taps\|by comp\|total" gpurun_out/${TAG}_$f.txt; done
