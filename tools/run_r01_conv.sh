#!/bin/bash
# GPU-box script: conv tests + conv micro-bench (tile / K-order sweep)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -x -q > gpurun_out/ops_tests.log 2>&1 || { tail -40 gpurun_out/ops_tests.log; exit 1; }
tail -3 gpurun_out/ops_tests.log
timeout -k 10 400 python tools/conv_bench.py --batch 32 --prec 0,2 --tiles 1,2,5,6 > gpurun_out/conv_bench.log 2>&1
rc=$?; cat gpurun_out/conv_bench.log; exit $rc
