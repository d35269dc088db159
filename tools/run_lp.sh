#!/bin/bash
# GPU-box script: op parity tests, then the full per-layer profile (bs=256)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-lp}; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ops_$TAG.log 2>&1 || { tail -40 gpurun_out/ops_$TAG.log; exit 1; }
tail -1 gpurun_out/ops_$TAG.log
timeout -k 10 300 python tools/layer_profile.py --batch 256 "$@" > gpurun_out/layer_profile_$TAG.txt 2>&1 || { tail -30 gpurun_out/layer_profile_$TAG.txt; exit 1; }
head -3 gpurun_out/layer_profile_$TAG.txt; tail -1 gpurun_out/layer_profile_$TAG.txt
