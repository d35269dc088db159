#!/bin/bash
# GPU-box script: small-Co tap rewrite -- its op test, model parity tests, then A/B on the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "smallco or upconv" tests/test_gpu_model.py > gpurun_out/smallco_tests.log 2>&1 || { tail -40 gpurun_out/smallco_tests.log; exit 1; }
tail -2 gpurun_out/smallco_tests.log
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 12 > gpurun_out/lp_smallco.txt 2>&1 || { tail -30 gpurun_out/lp_smallco.txt; exit 1; }
head -16 gpurun_out/lp_smallco.txt
bash tools/run_ab_env.sh smallco PRPE_SMALLCO_TAPS=0 PRPE_SMALLCO_TAPS=1
