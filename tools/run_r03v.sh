#!/bin/bash
# round 3: stem ring swizzle -- bit identity tests, LDS counters, A/B in the profile
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stem.py -x -q --timeout 200 --timeout-method thread > $O/r03v_stem_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 12 > $O/r03v_layer_profile.txt 2>&1 || exit 2
timeout -k 10 300 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d $O/r03v_pmc -o pmc -- python3 tools/layer_profile.py --batch 64 --top 5 > $O/r03v_pmc.log 2>&1 || exit 3
python tools/pmc_summary.py $O/r03v_pmc --kernel stem_pool --min-us 300 > $O/r03v_pmc_stem.txt
rm -rf $O/r03v_pmc
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > $O/r03v_model.log 2>&1 || exit 4
