#!/bin/bash
# GPU-box script: conv parity tests, then the conv micro-bench at bs=64 (auto tile)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-cc}; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ops_$TAG.log 2>&1 || { tail -40 gpurun_out/ops_$TAG.log; exit 1; }
tail -2 gpurun_out/ops_$TAG.log
timeout -k 10 300 python -u tools/conv_bench.py --batch 64 --iters 5 "$@" > gpurun_out/cb_$TAG.log 2>&1 || { tail -30 gpurun_out/cb_$TAG.log; exit 1; }
cat gpurun_out/cb_$TAG.log
