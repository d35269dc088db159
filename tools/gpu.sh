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
  py)
    TAG=$1 SEC=$2; shift 2; [ "$1" = "--" ] && shift
    timeout -k 10 "$SEC" python3 -u "$@" > $O/${TAG}.txt 2>&1
    rc=$?; tail -25 $O/${TAG}.txt; exit $rc ;;
  *) echo "unknown step $cmd"; exit 9 ;;
esac
