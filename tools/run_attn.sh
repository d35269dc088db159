#!/bin/bash
# GPU-box script: attention tests, micro-bench, PMC pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-at}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "attention" > gpurun_out/attn_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/attn_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/attn_tests_$TAG.log
timeout -k 10 100 python tools/attn_bench.py
if [ "${PMC:-1}" = "1" ]; then
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 -i tools/pmc_attn.txt --kernel-trace -d gpurun_out/pmc_$TAG -o pmc -- python3 tools/attn_bench.py --iters 1 > gpurun_out/pmc_$TAG.log 2>&1 || { tail -30 gpurun_out/pmc_$TAG.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_$TAG --kernel "vit_attention" --min-us 50
fi
