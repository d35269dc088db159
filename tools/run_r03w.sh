#!/bin/bash
# round 3: conflict-free halo / row swizzles (conv_halo, conv_bneck): op tests, LDS counters of
# the dominant conv, model tests, bench
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bneck.py -x -q --timeout 200 --timeout-method thread > $O/r03w_ops.log 2>&1 || exit 1
CB="tools/conv_bench.py --only vit_adapter.7 --prec 0 --korders 1 --planes --act gelu --taps 27"
timeout -k 10 240 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d $O/r03w_pmc -o pmc -- python3 $CB --batch 64 --tiles 0 --iters 2 > $O/r03w_pmc.log 2>&1 || exit 2
python tools/pmc_summary.py $O/r03w_pmc --kernel conv_halo --min-us 1000 > $O/r03w_pmc_va7.txt
rm -rf $O/r03w_pmc
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_contracts.py -x -q --timeout 300 --timeout-method thread > $O/r03w_model.log 2>&1 || exit 3
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03w_bench.json 2> $O/r03w_bench.err || exit 4
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 12 > $O/r03w_layer_profile.txt 2>&1 || exit 5
