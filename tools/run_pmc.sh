#!/bin/bash
# GPU-box script: PMC passes (kernel-trace only, no runtime/sys traces) over one conv_bench shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d gpurun_out/pmc_$TAG -o pmc -- python3 tools/conv_bench.py "$@" > gpurun_out/pmc_$TAG.log 2>&1 || { tail -30 gpurun_out/pmc_$TAG.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_$TAG --kernel "${KFILTER:-conv_}" --min-us 200
