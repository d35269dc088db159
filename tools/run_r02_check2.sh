#!/bin/bash
# GPU-box script: full GPU suite, per-layer profile, one bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-check}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputests.log
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 400 > gpurun_out/${TAG}_lp.txt 2>&1 || { tail -30 gpurun_out/${TAG}_lp.txt; exit 1; }
grep "layer\.[05]:fc1\|adapter.1[036]\|input_layer\|by comp\|total" gpurun_out/${TAG}_lp.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
