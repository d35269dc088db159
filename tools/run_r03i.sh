#!/bin/bash
# round 3: locate the bs=256 vs bs=2 frame-independence mismatch (fused layer1 bottleneck);
# conv_gemm with the conflict-free A swizzle: op tests, ViT GEMM micro-bench, LDS counters
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -v -s --timeout 120 --timeout-method thread > $O/r03i_bneck_tests.log 2>&1
timeout -k 10 400 python -u tools/batch_indep_diag.py --batch 256 --frame 127 --concurrent 0 > $O/r03i_diag_seq2.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "gemm or bit_exact" --timeout 120 --timeout-method thread > $O/r03i_ops_gemm.log 2>&1 || exit 2
CB="timeout -k 10 200 python -u tools/conv_bench.py --batch 256 --prec 0 --korders 0 --iters 10 --tiles 40"
$CB --act gelu --only "vit fc1" > $O/r03i_cb_gemm.txt 2>&1 || exit 3
$CB --act none --only "vit qkv" >> $O/r03i_cb_gemm.txt 2>&1 || exit 3
$CB --planes --act none --only "vit fc2" >> $O/r03i_cb_gemm.txt 2>&1 || exit 3
$CB --act none --only "vit proj" >> $O/r03i_cb_gemm.txt 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d $O/r03i_pmc -o pmc -- python3 tools/conv_bench.py --batch 256 --prec 0 --korders 0 --iters 2 --tiles 40 --planes --act none --only "vit fc2" > $O/r03i_pmc.log 2>&1 || exit 4
python tools/pmc_summary.py $O/r03i_pmc --kernel conv_gemm --min-us 100 > $O/r03i_pmc_fc2.txt
rm -rf $O/r03i_pmc
