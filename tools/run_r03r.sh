#!/bin/bash
# GPU-box script: HBM traffic (two PMC passes, FETCH_SIZE / WRITE_SIZE, kernel trace only) of the
# dominant launches of BASELINE configs 2 (face-YOLO adapter.10 with its epilogue chain, measured
# inside the config's own bench run) and 3 (ViT fc1, the GEMM kernel at the in-model shape), then
# the config benches with those records.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/yf_$C -o pmc -- python3 bench.py --config yolo_face --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/yf_$C.log 2>&1 || { tail -20 gpurun_out/yf_$C.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/vp_$C -o pmc -- python3 tools/conv_bench.py --only "vit fc1" --prec 0 --tiles 0 --korders 0 --batch 256 --iters 3 --planes --act gelu > gpurun_out/vp_$C.log 2>&1 || { tail -20 gpurun_out/vp_$C.log; exit 1; }
done
# algorithmic bytes -- yolo_face.adapter.10 at bs 64: planes input 64*160*160*256*4 + the chain's
# 27-channel fp32 output 64*160*160*27*4 + weight planes 9*256*128*2*2 (+ w2 / w3, < 0.1 MB)
python tools/traffic_json.py gpurun_out/yf_FETCH_SIZE gpurun_out/yf_WRITE_SIZE --kernel "conv_halo_kernel<4, 8, 16, 8, false, true, 2" --min-us 1000 \
  --layer yolo_face.adapter.10 --batch 64 --precision 0 --algorithmic 1855848448 --sources conv_halo.hip,conv.h,common.h \
  --shape "3x3 256->128 @160x160, planes input, SiLU, epilogue chain 1x1 128->64 + SiLU -> 27 taps" --out gpurun_out/r03_pmc_traffic_yolo_face.json --command tools/run_r03r.sh
# vit fc1 at 256 crops: planes input 49152*768*4 + planes output 49152*3072*4 + weight planes 3072*768*2*2
python tools/traffic_json.py gpurun_out/vp_FETCH_SIZE gpurun_out/vp_WRITE_SIZE --kernel conv_gemm_kernel --min-us 300 \
  --layer "vit_pose.vit_pose.backbone.encoder.layer.0:fc1" --batch 256 --precision 0 --algorithmic 764411904 --sources conv_gemm.hip,conv.h,common.h \
  --shape "1x1 768->3072 over 49152 tokens, planes input and output, GELU" --out gpurun_out/r03_pmc_traffic_vitpose.json --command tools/run_r03r.sh
rm -rf gpurun_out/yf_FETCH_SIZE gpurun_out/yf_WRITE_SIZE gpurun_out/vp_FETCH_SIZE gpurun_out/vp_WRITE_SIZE
cat gpurun_out/r03_pmc_traffic_yolo_face.json gpurun_out/r03_pmc_traffic_vitpose.json

cp gpurun_out/r03_pmc_traffic_yolo_face.json gpurun_out/r03_pmc_traffic_vitpose.json profiles/   # (box copy) for the lines below
timeout -k 10 300 python bench.py --config vitpose --steps 20 --warmup 3 > gpurun_out/r03r_bench_vitpose.json 2> gpurun_out/r03r_bench_vitpose.err || exit 4
timeout -k 10 300 python bench.py --config yolo_face --steps 20 --warmup 3 > gpurun_out/r03r_bench_yolo_face.json 2> gpurun_out/r03r_bench_yolo_face.err || exit 5
timeout -k 10 300 python bench.py --config yolo_raw --steps 20 --warmup 3 > gpurun_out/r03r_bench_yolo_raw.json 2> gpurun_out/r03r_bench_yolo_raw.err || exit 6
