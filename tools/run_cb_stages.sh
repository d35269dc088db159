#!/bin/bash
# GPU-box script: wave-kernel tiles incl. the 2-stage ring variants on the big precision-0 shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/cb_stages.txt
: > $O
timeout -k 10 150 python tools/conv_bench.py --batch 64 --only "vit_adapter.7" --prec 0 --korders 1 --tiles 26,28,29,24 --planes --iters 3 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 150 python tools/conv_bench.py --batch 64 --only "yolo_adapter.7" --prec 0 --tiles 26,28,29,24 --planes --iters 3 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 150 python tools/conv_bench.py --batch 256 --only "vit fc" --prec 0 --tiles 26,28,29,24 --iters 3 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 150 python tools/conv_bench.py --batch 64 --only "ada_adapter.7" --prec 0 --korders 1 --tiles 26,28,29,24 --iters 3 >> $O 2>&1 || { tail -20 $O; exit 1; }
grep -v "n/a\|amdgpu.ids" $O
