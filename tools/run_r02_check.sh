#!/bin/bash
# GPU-box script (round 2): the new NMS global path alone (synchronous launches, so a fault
# names its launch), then the -m gpu suite, then one bench line per BASELINE config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02}
HIP_LAUNCH_BLOCKING=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_postproc.py -m gpu -x -v -k global --timeout 100 --timeout-method thread > gpurun_out/${TAG}_nms_global.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_nms_global.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for C in full yolo_face vitpose; do
  timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_$C.json 2> gpurun_out/${TAG}_bench_$C.err || { tail -20 gpurun_out/${TAG}_bench_$C.err; exit 1; }
  cat gpurun_out/${TAG}_bench_$C.json
done
