#!/bin/bash
# GPU-box script: bench A/B over several env settings, interleaved twice
#   bash tools/run_ab_multi.sh TAG "VAR=a" "VAR=b" ["VAR=c" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
for i in 1 2; do
  for V in "$@"; do
    env $V timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err || { tail -20 gpurun_out/ab_${TAG}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/ab_${TAG}.json "$V"
  done
done
