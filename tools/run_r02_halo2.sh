#!/bin/bash
# GPU-box script: halo tests, 64-channel tiles bench, layer profile, bench line (halo on / off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-halo2}
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k halo -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for S in "ada_adapter.10" "trunk l1 3x3" "ada body.0"; do
  timeout -k 10 200 python -u tools/conv_bench.py --batch 64 --planes --prec 0 --korders 1 --act gelu --only "$S" --iters 10 --tiles 28,31,34,35 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
done
timeout -k 10 200 python -u tools/conv_bench.py --batch 256 --prec 3 --korders 1 --act relu --only "trunk l1 3x3" --iters 10 --tiles 25,31,34,35 >> gpurun_out/${TAG}_cb.txt 2>&1 || { tail -30 gpurun_out/${TAG}_cb.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_cb.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputests.log
timeout -k 10 300 python tools/layer_profile.py --batch 256 > gpurun_out/${TAG}_layer_profile.txt 2>&1 || { tail -30 gpurun_out/${TAG}_layer_profile.txt; exit 1; }
head -14 gpurun_out/${TAG}_layer_profile.txt; tail -1 gpurun_out/${TAG}_layer_profile.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('halo on', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
PRPE_CONV_HALO=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_off.json 2> gpurun_out/${TAG}_bench_off.err || { tail -20 gpurun_out/${TAG}_bench_off.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_off.json'));print('halo off', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
