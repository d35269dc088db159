#!/bin/bash
# GPU-box script: A via LDS-DMA full lines (conv_glds tiles 10-12) vs A fragment-loads (wave tile 28)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-glds}
for S in "vit_adapter.7" "yolo_adapter.10" "ada_adapter.7" "vit fc1" "yolo_adapter.7"; do
  timeout -k 10 200 python -u tools/conv_bench.py --batch 64 --prec 0 --korders 1 --act gelu --only "$S" --tiles 28,10,11,12 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/${TAG}_cb.txt
