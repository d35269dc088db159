#!/bin/bash
# GPU-box script: conv op tests, planes-input conv micro-bench, per-layer profile, bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-apl}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_ops.log 2>&1 || { tail -40 gpurun_out/${TAG}_ops.log; exit 1; }
tail -1 gpurun_out/${TAG}_ops.log
timeout -k 10 200 python -u tools/conv_bench.py --batch 64 --planes --prec 0 --korders 1 --act gelu --only adapter > gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
cat gpurun_out/${TAG}_cb.txt
timeout -k 10 300 python tools/layer_profile.py --batch 256 > gpurun_out/${TAG}_layer_profile.txt 2>&1 || { tail -30 gpurun_out/${TAG}_layer_profile.txt; exit 1; }
head -12 gpurun_out/${TAG}_layer_profile.txt; tail -1 gpurun_out/${TAG}_layer_profile.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
