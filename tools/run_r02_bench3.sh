#!/bin/bash
# GPU-box script: full GPU test suite log, then the bench line of each BASELINE config with its CPU baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputests_full.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests_full.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputests_full.log
for C in full yolo_face vitpose; do
  timeout -k 10 400 python -u bench.py --config $C > gpurun_out/${TAG}_bench_$C.json 2> gpurun_out/${TAG}_bench_$C.err || { tail -20 gpurun_out/${TAG}_bench_$C.err; exit 1; }
  cat gpurun_out/${TAG}_bench_$C.json
done
