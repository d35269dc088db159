#!/bin/bash
# GPU-box script: GPU tests, per-layer profile, bench line (new kernels on / off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-model}
OFF=${2:-PRPE_CONV_GEMM}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputests.log
timeout -k 10 300 python tools/layer_profile.py --batch 256 > gpurun_out/${TAG}_layer_profile.txt 2>&1 || { tail -30 gpurun_out/${TAG}_layer_profile.txt; exit 1; }
head -14 gpurun_out/${TAG}_layer_profile.txt; tail -1 gpurun_out/${TAG}_layer_profile.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('on', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
env $OFF=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_off.json 2> gpurun_out/${TAG}_bench_off.err || { tail -20 gpurun_out/${TAG}_bench_off.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_off.json'));print('off', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
