#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/t41.txt
timeout -k 10 200 python tools/conv_bench.py --only "yolo_adapter.7" --prec 0 --tiles 40,41,40,41 --korders 0 --batch 256 --iters 5 --planes --act silu >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 200 python tools/conv_bench.py --only "trunk l1 conv3" --prec 3 --tiles 0,40,41,0,40,41 --korders 0 --batch 256 --iters 5 --act relu >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 200 python tools/conv_bench.py --only "trunk l2 conv3" --prec 3 --tiles 0,40,41,0,40,41 --korders 0 --batch 256 --iters 5 --act relu >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 200 python tools/conv_bench.py --only "trunk l1 1x1 64->256" --prec 3 --tiles 0,40,41,0,40,41 --korders 0 --batch 256 --iters 5 --act relu >> $O 2>&1 || { tail -20 $O; exit 1; }
grep -v amdgpu $O
