#!/bin/bash
# round 3: LDS-DMA upconv -- op tests, then the upconv micro-bench and the per-layer profile
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "upconv or planes or smallco" > $O/r03b_ops.log 2>&1 || exit 1
timeout -k 10 200 python tools/upconv_bench.py --fused-only --batch 64 > $O/r03b_upconv_bench.txt 2>&1 || exit 2
PRPE_UPCONV_DMA=0 timeout -k 10 200 python tools/upconv_bench.py --fused-only --batch 64 > $O/r03b_upconv_bench_fused.txt 2>&1 || exit 3
timeout -k 10 300 python tools/layer_profile.py --batch 256 --top 300 > $O/r03b_layer_profile.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03b_bench.json 2> $O/r03b_bench.err || exit 5
# HBM traffic of the bench's dominant launch after the round-3 halo rewrite (two PMC passes)
ARGS="tools/conv_bench.py --only vit_adapter.7 --prec 0 --tiles 0 --korders 1 --batch 256 --iters 2 --planes --act gelu --taps 27"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d $O/r03b_tr_$C -o pmc -- python3 $ARGS > $O/r03b_tr_$C.log 2>&1 || exit 6
done
python tools/traffic_json.py $O/r03b_tr_FETCH_SIZE $O/r03b_tr_WRITE_SIZE --kernel conv_halo --min-us 5000 \
  --layer vit_pose.adapter.7 --batch 256 --precision 0 --algorithmic 14245036032 --sources conv_halo.hip,conv.h,common.h \
  --shape "3x3 256->128 @256x192, planes input, GELU, epilogue tap GEMM to 27 ch" --out $O/r03_pmc_traffic_full.json \
  --command tools/run_r03b.sh || exit 7
rm -rf $O/r03b_tr_FETCH_SIZE $O/r03b_tr_WRITE_SIZE
timeout -k 10 240 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d $O/r03b_pmc_va7 -o pmc -- python3 $ARGS > $O/r03b_pmc_va7.log 2>&1 || exit 8
python tools/pmc_summary.py $O/r03b_pmc_va7 --kernel conv_halo --min-us 5000 > $O/r03b_pmc_vitadapter7.txt
rm -rf $O/r03b_pmc_va7
