#!/bin/bash
# GPU-box script: new-op tests (sync), full GPU suite, per-layer A/B, bench on/off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-model2}
OFF=${2:-PRPE_CONV_GEMM}
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "${KSEL:-planes or attention or gemm or halo or upconv or smallco or activation or splitk}" -x -q --timeout 100 --timeout-method thread > gpurun_out/${TAG}_newtests.log 2>&1 || { tail -40 gpurun_out/${TAG}_newtests.log; exit 1; }
tail -1 gpurun_out/${TAG}_newtests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputests.log
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 400 > gpurun_out/${TAG}_on.txt 2>&1 || { tail -30 gpurun_out/${TAG}_on.txt; exit 1; }
env $OFF=${OFFVAL:-0} timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 400 > gpurun_out/${TAG}_off.txt 2>&1 || { tail -30 gpurun_out/${TAG}_off.txt; exit 1; }
for f in on off; do echo "== $f"; grep "layer\.[05]:\|adapter\.7\|adapter\.10\|by comp\|total" gpurun_out/${TAG}_$f.txt; done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('on', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
env $OFF=${OFFVAL:-0} timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_off.json 2> gpurun_out/${TAG}_bench_off.err || { tail -20 gpurun_out/${TAG}_bench_off.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_off.json'));print('off', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
