#!/bin/bash
# GPU-box script: A/B of an environment setting on the full bench, interleaved A B A B
#   bash tools/run_ab_env.sh TAG "VAR=a" "VAR=b"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; A=$2; B=$3
for i in 1 2; do
  for V in "$A" "$B"; do
    env $V timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err || { tail -20 gpurun_out/ab_${TAG}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" gpurun_out/ab_${TAG}_$i.json "$V"
  done
done
