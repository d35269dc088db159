#!/bin/bash
# GPU-box script: upconv op tests then the upconv micro-bench, A/B of an env setting
#   bash tools/run_upbench.sh TAG "VAR=a" "VAR=b"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-up}; A=${2:-X=0}; B=${3:-X=1}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "upconv or smallco" > gpurun_out/uptests_$TAG.log 2>&1 || { tail -40 gpurun_out/uptests_$TAG.log; exit 1; }
tail -1 gpurun_out/uptests_$TAG.log
for V in "$A" "$B"; do
  echo "== $V"
  env $V timeout -k 10 200 python tools/upconv_bench.py --batch 64 --iters 3 > gpurun_out/upbench_$TAG.txt 2>&1 || { tail -20 gpurun_out/upbench_$TAG.txt; exit 1; }
  grep fused gpurun_out/upbench_$TAG.txt
done
