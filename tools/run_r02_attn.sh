#!/bin/bash
# GPU-box script: attention tests, then the attention micro-bench per kernel variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-attn}
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k attention -x -q --timeout 100 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for V in 1 64; do
  PRPE_ATTN=$V timeout -k 10 120 python -u tools/attn_bench.py --batch 256 --iters 20 >> gpurun_out/${TAG}_bench.txt 2>&1 || { tail -20 gpurun_out/${TAG}_bench.txt; exit 1; }
done
grep "PRPE\|head-major" gpurun_out/${TAG}_bench.txt
