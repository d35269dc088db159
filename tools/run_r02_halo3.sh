#!/bin/bash
# GPU-box script: haloed-tile kernel, 64-row-per-wave tile (36) vs the 32-row tile (31): tests, micro-bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-halo3}
TILES=${TILES:-31,36,32,37}
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "halo" -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
: > gpurun_out/${TAG}_cb.txt
for S in "vit_adapter.7" "yolo_adapter.10" "ada_adapter.7"; do
  timeout -k 10 200 python -u tools/conv_bench.py --batch 64 --planes --prec 0 --korders 1 --act gelu --only "$S" --iters 10 --tiles $TILES >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
done
for S in "trunk l1 3x3"; do
  timeout -k 10 200 python -u tools/conv_bench.py --batch 256 --prec 3 --korders 1 --act relu --only "$S" --iters 10 --tiles $TILES >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/${TAG}_cb.txt
