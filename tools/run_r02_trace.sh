#!/bin/bash
# GPU-box script: kernel trace of sequential bs=256 forward passes -> per-kernel summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-trace}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG} -o ${TAG} -- python3 tools/seq_forward.py --batch 256 --passes 2 > gpurun_out/${TAG}.log 2>&1 || { tail -30 gpurun_out/${TAG}.log; exit 1; }
grep "ms/pass" gpurun_out/${TAG}.log
DB=$(find gpurun_out/${TAG} -name "*.db" | head -1)
python3 tools/prof_summary.py "$DB" --passes 3 > gpurun_out/${TAG}_summary.txt
head -45 gpurun_out/${TAG}_summary.txt
