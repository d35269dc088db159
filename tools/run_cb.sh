#!/bin/bash
# GPU-box script: conv micro-bench only (no tests); args go to tools/conv_bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-cb}; shift
timeout -k 10 300 python -u tools/conv_bench.py "$@" > gpurun_out/cb_$TAG.log 2>&1 || { tail -30 gpurun_out/cb_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cb_$TAG.log | sed -E 's/ +alg.*exec/ exec/'
