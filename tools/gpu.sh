#!/bin/bash
# GPU-box driver for every measurement this repo commits under profiles/ (round 4 on; the round 1-3
# one-off run_r0*.sh scripts are in git history, commit 9d55af4). Each step runs under its own
# time limit; chain steps with && so a failure ends the call.
#
#   bash tools/gpu.sh tests [pytest -k expr]     -m gpu parity suite (one process)
#   bash tools/gpu.sh smoke
#   bash tools/gpu.sh bench TAG [bench.py args]  one bench line -> gpurun_out/TAG_bench.json
#   bash tools/gpu.sh lp TAG [layer_profile args] per-conv profile -> gpurun_out/TAG_layer_profile.txt
#   bash tools/gpu.sh trace TAG                  rocprofv3 --kernel-trace --stats of the bench command
#   bash tools/gpu.sh pmc TAG COUNTERS KERNEL MIN_US -- python-args...   counter passes (-i file)
#   bash tools/gpu.sh traffic TAG KERNEL MIN_US ALG_BYTES LAYER BATCH PREC SOURCES SHAPE -- python-args...
#                                                FETCH_SIZE / WRITE_SIZE passes -> gpurun_out/TAG_traffic.json
#   bash tools/gpu.sh py TAG SECONDS -- python-args...   any tool script -> gpurun_out/TAG.txt
#   bash tools/gpu.sh evidence rNN               traffic records of the four configs, kernel trace, bench lines
#                                                (= evidence_pmc rNN, then evidence_bench rNN)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cmd=$1; shift
case "$cmd" in
  tests)
    K=()
    [ -n "$1" ] && K=(-k "$1")
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" \
      > $O/gpu_tests.log 2>&1
    rc=$?; tail -3 $O/gpu_tests.log; exit $rc ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
    rc=$?; tail -2 $O/smoke.log; exit $rc ;;
  bench)
    TAG=$1; shift
    timeout -k 10 400 python bench.py "$@" > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err
    rc=$?; cat $O/${TAG}_bench.json; exit $rc ;;
  lp)
    TAG=$1; shift
    timeout -k 10 300 python tools/layer_profile.py --batch 256 "$@" > $O/${TAG}_layer_profile.txt 2>&1
    rc=$?; head -2 $O/${TAG}_layer_profile.txt; tail -1 $O/${TAG}_layer_profile.txt; exit $rc ;;
  trace)
    TAG=$1; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_tr -o bench -- python3 bench.py --steps 5 --warmup 2 \
      --no-cpu-baseline "$@" > $O/${TAG}_trace_bench.json 2> $O/${TAG}_trace_bench.err || exit 5
    DB=$(find $O/${TAG}_tr -name "*.db" | head -1)
    python3 tools/prof_summary.py "$DB" --passes 1 --dominant "%conv_halo%" > $O/${TAG}_kernel_trace.txt
    rc=$?
    STATS=$(find $O/${TAG}_tr -name "*kernel_stats.csv" | head -1)
    [ -n "$STATS" ] && cp "$STATS" $O/${TAG}_kernel_stats.csv
    rm -rf $O/${TAG}_tr; head -30 $O/${TAG}_kernel_trace.txt; exit $rc ;;
  pmc)
    TAG=$1 CF=$2 KF=$3 MIN=$4; shift 4; [ "$1" = "--" ] && shift
    timeout -k 10 240 rocprofv3 -i "$CF" --kernel-trace -d $O/${TAG}_pmcraw -o pmc -- python3 "$@" > $O/${TAG}_pmc.log 2>&1 || exit 4
    python3 tools/pmc_summary.py $O/${TAG}_pmcraw --kernel "$KF" --min-us "$MIN" > $O/${TAG}_pmc.txt
    rc=$?; rm -rf $O/${TAG}_pmcraw; cat $O/${TAG}_pmc.txt; exit $rc ;;
  traffic)
    TAG=$1 KF=$2 MIN=$3 ALG=$4 LAYER=$5 BATCH=$6 PREC=$7 SRCS=$8 SHAPE=$9; shift 9; [ "$1" = "--" ] && shift
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $O/${TAG}_$C -o pmc -- python3 "$@" > $O/${TAG}_$C.log 2>&1 || exit 3
    done
    python3 tools/traffic_json.py $O/${TAG}_FETCH_SIZE $O/${TAG}_WRITE_SIZE --kernel "$KF" --min-us "$MIN" --layer "$LAYER" \
      --batch "$BATCH" --precision "$PREC" --algorithmic "$ALG" --sources "$SRCS" --shape "$SHAPE" \
      --out $O/${TAG}_traffic.json --command "tools/gpu.sh traffic $TAG"
    rc=$?; rm -rf $O/${TAG}_FETCH_SIZE $O/${TAG}_WRITE_SIZE; cat $O/${TAG}_traffic.json; exit $rc ;;
  evidence)
    # end-of-round record on the committed sources: PMC traffic of every bench config's dominant
    # launch (profiles/rNN_pmc_traffic_<config>.json, read by bench.py while the sources match),
    # the kernel trace of the bench command, and the four bench lines with CPU baselines
    # (evidence_pmc + evidence_bench: the same in two calls, each within one gpurun limit)
    R=$1; [ -n "$R" ] || { echo "evidence needs the round tag (e.g. r04)"; exit 9; }
    bash tools/gpu.sh evidence_pmc $R && bash tools/gpu.sh evidence_bench $R; exit $? ;;
  evidence_pmc)
    R=$1; [ -n "$R" ] || { echo "evidence needs the round tag (e.g. r04)"; exit 9; }
    bash tools/gpu.sh traffic ${R}_full conv_halo 5000 14245036032 vit_pose.adapter.7 256 0 conv_halo.hip,conv.h,common.h \
      "3x3 256->128 @256x192, planes input, GELU, epilogue tap GEMM to 27 ch" -- tools/conv_bench.py --only vit_adapter.7 \
      --prec 0 --tiles 0 --korders 1 --batch 256 --iters 2 --planes --act gelu --taps 27 || exit 11
    bash tools/gpu.sh traffic ${R}_yolo_face "conv_halo_kernel<4, 8, 16, 8, false, true, 2" 1000 1855848448 yolo_face.adapter.10 64 0 \
      conv_halo.hip,conv.h,common.h "3x3 256->128 @160x160, planes input, SiLU, epilogue chain 1x1 128->64 + SiLU -> 27 taps" \
      -- bench.py --config yolo_face --steps 2 --warmup 1 --no-cpu-baseline || exit 12
    bash tools/gpu.sh traffic ${R}_vitpose conv_gemm_kernel 300 764411904 "vit_pose.vit_pose.backbone.encoder.layer.0:fc1" 256 0 \
      conv_gemm.hip,conv.h,common.h "1x1 768->3072 over 49152 tokens, planes input and output, GELU" \
      -- tools/conv_bench.py --only "vit fc1" --prec 0 --tiles 0 --korders 0 --batch 256 --iters 3 --planes --y-planes \
      --act gelu || exit 13
    # yolo_raw: p1.0 (3x3/2 3->16 on the raw NCHW frames; algorithmic = 64 frames in + the 16-ch map out)
    bash tools/gpu.sh traffic ${R}_yolo_raw "conv_igemm_kernel<128, 16" 300 734004928 yolo_face.yolo.net.p1.0 64 2 \
      conv_igemm.hip,conv.h,common.h "3x3/2 3->16 @640x640, NCHW frames read in place" \
      -- bench.py --config yolo_raw --steps 2 --warmup 1 --no-cpu-baseline || exit 14
    for C in full yolo_face vitpose yolo_raw; do
      mv $O/${R}_${C}_traffic.json $O/${R}_pmc_traffic_${C}.json && cp $O/${R}_pmc_traffic_${C}.json profiles/ || exit 15
    done
    bash tools/gpu.sh trace ${R}_final || exit 16 ;;
  evidence_bench)
    R=$1; [ -n "$R" ] || { echo "evidence needs the round tag (e.g. r04)"; exit 9; }
    for C in full yolo_face vitpose yolo_raw; do
      timeout -k 10 400 python bench.py --config $C --steps 20 --warmup 3 > $O/${R}_bench_${C}.json 2> $O/${R}_bench_${C}.err || exit 17
      tail -c 300 $O/${R}_bench_${C}.json
    done ;;
  py)
    TAG=$1 SEC=$2; shift 2; [ "$1" = "--" ] && shift
    timeout -k 10 "$SEC" python3 -u "$@" > $O/${TAG}.txt 2>&1
    rc=$?; tail -25 $O/${TAG}.txt; exit $rc ;;
  *) echo "unknown step $cmd"; exit 9 ;;
esac
