#!/bin/bash
# GPU-box script: 256x256 GEMM kernel tests (synchronous launches first), micro-bench vs the wave tile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-gemm}
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k gemm -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u tools/conv_bench.py --batch 256 --prec 0 --korders 0 --act gelu --only "vit fc1" --iters 10 --tiles 28,40,41,42 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
timeout -k 10 200 python -u tools/conv_bench.py --batch 256 --prec 0 --korders 0 --act none --only "vit qkv" --iters 10 --tiles 28,40,41,42 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
timeout -k 10 200 python -u tools/conv_bench.py --batch 256 --planes --prec 0 --korders 0 --act none --only "vit fc2" --iters 10 --tiles 28,40,41,42 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
timeout -k 10 200 python -u tools/conv_bench.py --batch 256 --prec 0 --korders 0 --act none --only "vit proj" --iters 10 --tiles 28,40,41,42 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
timeout -k 10 200 python -u tools/conv_bench.py --batch 64 --planes --prec 0 --korders 0 --act silu --only "yolo_adapter.7" --iters 10 --tiles 28,40,41,42 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_cb.txt
