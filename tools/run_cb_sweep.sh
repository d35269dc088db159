#!/bin/bash
# GPU-box script: conv_bench tile sweeps for the memory-/latency-bound conv shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-cb}
O=gpurun_out/cb_$TAG.txt
: > $O
timeout -k 10 120 python tools/conv_bench.py --batch 64 --only "yolo_adapter.7" --prec 0 --tiles 0,21,22,23,24,25,26,27 --planes >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 120 python tools/conv_bench.py --batch 64 --only "yolo_adapter.13" --prec 0 --tiles 0,1,2,3,5,6,10,11,12,21,22,23,24,25,26,27 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 120 python tools/conv_bench.py --batch 64 --only "ada_adapter.10" --prec 0 --korders 1 --tiles 0,1,2,5,6,10,11,12,21,22,23,24,25,26,27 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 120 python tools/conv_bench.py --batch 64 --only "ada body.0" --prec 0 --korders 1 --tiles 0,1,2,5,6,10,11,12,21,22,23,24,25,26,27 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 120 python tools/conv_bench.py --batch 256 --only "conv3 1x1" --prec 3 --amax --tiles 0,21,22,23,24,25,26 >> $O 2>&1 || { tail -20 $O; exit 1; }
grep -v "n/a" $O
