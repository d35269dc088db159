#!/bin/bash
# GPU-box script: upconv micro-bench (times) then its PMC passes (kernel-trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-up}
timeout -k 10 200 python tools/upconv_bench.py --batch 64 --iters 3 > gpurun_out/upbench_$TAG.txt 2>&1 || { tail -20 gpurun_out/upbench_$TAG.txt; exit 1; }
cat gpurun_out/upbench_$TAG.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -i tools/pmc_upconv.txt --kernel-trace -d gpurun_out/pmc_$TAG -o pmc -- python3 tools/upconv_bench.py --batch 64 --iters 1 > gpurun_out/pmc_$TAG.log 2>&1 || { tail -30 gpurun_out/pmc_$TAG.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_$TAG --kernel "upconv" --min-us 200
