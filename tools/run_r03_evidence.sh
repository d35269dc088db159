#!/bin/bash
# GPU-box script (round 3 evidence on the committed kernel sources): HBM traffic of the bench's
# dominant launch (two PMC passes -> profiles/r03_pmc_traffic_full.json), PMC counters of the
# dominant conv, ViT fc2 and attention, and the rocprofv3 kernel trace of the bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
TAG=${1:-r03ev}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > $O/${TAG}_bneck_tests.log 2>&1 || exit 1
ARGS="tools/conv_bench.py --only vit_adapter.7 --prec 0 --tiles 0 --korders 1 --batch 256 --iters 2 --planes --act gelu --taps 27"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d $O/${TAG}_tr_$C -o pmc -- python3 $ARGS > $O/${TAG}_tr_$C.log 2>&1 || exit 2
done
# algorithmic bytes: planes input 256 x 256 x 192 x 256 x 4 B + the epilogue tap GEMM's fp32
# output (27 ch; the 128-ch map stays in LDS) + weight planes
python tools/traffic_json.py $O/${TAG}_tr_FETCH_SIZE $O/${TAG}_tr_WRITE_SIZE --kernel conv_halo --min-us 5000 \
  --layer vit_pose.adapter.7 --batch 256 --precision 0 --algorithmic 14245036032 --sources conv_halo.hip,conv.h,common.h \
  --shape "3x3 256->128 @256x192, planes input, GELU, epilogue tap GEMM to 27 ch" --out $O/r03_pmc_traffic_full.json \
  --command "tools/run_r03_evidence.sh" || exit 3
rm -rf $O/${TAG}_tr_FETCH_SIZE $O/${TAG}_tr_WRITE_SIZE
cp $O/r03_pmc_traffic_full.json profiles/    # (box copy) so this call's bench lines carry it
run() {  # name counters kernel-filter min-us -- args
  local N=$1 CF=$2 K=$3 MIN=$4; shift 4
  timeout -k 10 240 rocprofv3 -i $CF --kernel-trace -d $O/${TAG}_$N -o pmc -- python3 "$@" > $O/${TAG}_$N.log 2>&1 || exit 4
  python tools/pmc_summary.py $O/${TAG}_$N --kernel "$K" --min-us $MIN > $O/${TAG}_pmc_$N.txt
  rm -rf $O/${TAG}_$N
}
run vitadapter7 tools/pmc_conv.txt conv_halo 1000 tools/conv_bench.py --only vit_adapter.7 --prec 0 --tiles 0 --korders 1 --batch 64 --iters 2 --planes --act gelu --taps 27
run fc2 tools/pmc_conv.txt conv_gemm 100 tools/conv_bench.py --only "vit fc2" --prec 0 --tiles 40 --korders 0 --batch 256 --iters 2 --planes --act none
run attn tools/pmc_attn.txt vit_attention 50 tools/attn_bench.py --iters 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_bench -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit 5
DB=$(find $O/${TAG}_bench -name "*.db" | head -1)
python3 tools/prof_summary.py "$DB" --passes 1 --dominant "%conv_halo%" > $O/${TAG}_kernel_trace.txt
rm -rf $O/${TAG}_bench
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/${TAG}_bench_final.json 2> $O/${TAG}_bench_final.err || exit 6
