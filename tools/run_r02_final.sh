#!/bin/bash
# GPU-box script (round 2 evidence): PMC counters of the dominant conv (halo kernel, ViT adapter
# 3x3), the ViT GEMMs and attention; HBM traffic of the bench's dominant launch; rocprofv3 kernel
# trace of the default bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-final}
export TMPDIR=/tmp
run() {  # name counters kernel-filter min-us -- args
  local N=$1 CF=$2 K=$3 MIN=$4; shift 4
  timeout -k 10 240 rocprofv3 -i $CF --kernel-trace -d gpurun_out/${TAG}_$N -o pmc -- python3 "$@" > gpurun_out/${TAG}_$N.log 2>&1 || { tail -30 gpurun_out/${TAG}_$N.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/${TAG}_$N --kernel "$K" --min-us $MIN > gpurun_out/${TAG}_$N.txt
  rm -rf gpurun_out/${TAG}_$N        # the DBs stay on the box (the merge back is capped at 64 MiB)
  cat gpurun_out/${TAG}_$N.txt
}
run vitadapter7 tools/pmc_conv.txt conv_halo 1000 tools/conv_bench.py --only vit_adapter.7 --prec 0 --tiles 0 --korders 1 --batch 64 --iters 2 --planes --act gelu --taps 27
run fc2 tools/pmc_conv.txt conv_gemm 100 tools/conv_bench.py --only "vit fc2" --prec 0 --tiles 40 --korders 0 --batch 256 --iters 2 --planes --act none
run attn tools/pmc_attn.txt vit_attention 50 tools/attn_bench.py --iters 2
ARGS="tools/conv_bench.py --only vit_adapter.7 --prec 0 --tiles 0 --korders 1 --batch 256 --iters 2 --planes --act gelu --taps 27"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_tr_$C -o pmc -- python3 $ARGS > gpurun_out/${TAG}_tr_$C.log 2>&1 || { tail -20 gpurun_out/${TAG}_tr_$C.log; exit 1; }
done
# algorithmic bytes: planes input 256 x 256 x 192 x 256 x 4 B + the epilogue tap GEMM's fp32
# output (27 ch; the 128-ch map stays in LDS) + weight planes (3x3 x 256 x 128 x 2 x 2 B)
python tools/traffic_json.py gpurun_out/${TAG}_tr_FETCH_SIZE gpurun_out/${TAG}_tr_WRITE_SIZE --kernel conv_halo --min-us 5000 \
  --layer vit_pose.adapter.7 --batch 256 --precision 0 --algorithmic 14245036032 --sources conv_halo.hip,conv.h,common.h \
  --shape "3x3 256->128 @256x192, planes input, GELU, epilogue tap GEMM to 27 ch" --out gpurun_out/r02_pmc_traffic_full.json
rm -rf gpurun_out/${TAG}_tr_FETCH_SIZE gpurun_out/${TAG}_tr_WRITE_SIZE
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_bench -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
DB=$(find gpurun_out/${TAG}_bench -name "*.db" | head -1)
python3 tools/prof_summary.py "$DB" --passes 1 --dominant "%conv_halo%" > gpurun_out/${TAG}_kernel_trace.txt
rm -rf gpurun_out/${TAG}_bench
head -30 gpurun_out/${TAG}_kernel_trace.txt; tail -3 gpurun_out/${TAG}_kernel_trace.txt
