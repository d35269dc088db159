#!/bin/bash
# GPU-box script: full GPU tests, per-layer profile, bench line, rocprofv3 kernel summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 40 > gpurun_out/layer_profile_$TAG.txt 2>&1 || { tail -30 gpurun_out/layer_profile_$TAG.txt; exit 1; }
head -60 gpurun_out/layer_profile_$TAG.txt
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o prof -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
  DB=$(python -c "import glob,sys;print(sorted(glob.glob(sys.argv[1]+'/**/*.db',recursive=True))[0])" gpurun_out/prof_$TAG)
  python tools/prof_summary.py $DB --passes 7 --dominant '%conv_wave_kernelILi4ELi2ELi8ELi2ELi2ELb0ELb0ELb0E%' --grid 25165824 > gpurun_out/prof_summary_$TAG.txt 2>&1; cat gpurun_out/prof_summary_$TAG.txt
fi
