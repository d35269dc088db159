#!/bin/bash
# GPU-box script: ablations of the planes-input wave tile (diagnostic; outputs wrong by design)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-abl}
timeout -k 10 300 python -u tools/conv_bench.py --batch 64 --planes --prec 0 --korders 1 --act gelu --only "vit_adapter.7" --iters 10 --tiles 28,41,42,43,44,47,28 > gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
timeout -k 10 300 python -u tools/conv_bench.py --batch 256 --planes --prec 0 --korders 0 --act none --only "vit fc2" --iters 10 --tiles 28,41,42,43,44,47,28 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_cb.txt
