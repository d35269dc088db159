#!/bin/bash
# GPU-box script: GPU tests, then wave-kernel tile sweeps on the adapter 3x3 (planes input) and
# the ViT GEMMs, then the sequential-forward kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-sweep}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u tools/conv_bench.py --batch 64 --planes --prec 0 --korders 1 --act gelu --only "vit_adapter.7" --tiles 21,23,24,25,26,27,28,29 > gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
timeout -k 10 300 python -u tools/conv_bench.py --batch 256 --prec 0 --korders 0 --act gelu --only "vit fc1" --tiles 21,23,24,25,26,27,28,29 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
timeout -k 10 300 python -u tools/conv_bench.py --batch 256 --prec 0 --korders 0 --act none --only "vit qkv" --tiles 21,23,24,25,26,27,28,29 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
timeout -k 10 300 python -u tools/conv_bench.py --batch 256 --planes --prec 0 --korders 0 --act none --only "vit fc2" --tiles 21,23,24,25,26,27,28,29 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_cb.txt
bash tools/run_r02_trace.sh ${TAG}_trace | head -16
