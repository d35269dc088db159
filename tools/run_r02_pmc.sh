#!/bin/bash
# GPU-box script: PMC counter passes (kernel-trace only; one rocprofv3 run per counter line of
# the input file) over (1) the dominant 3x3 adapter conv, (2) the ViT fc1 GEMM, (3) the ViT
# attention kernel; summaries under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-pmc}
export TMPDIR=/tmp
run() {  # name filter kernel-filter min-us -- args
  local N=$1 K=$2 MIN=$3; shift 3
  timeout -k 10 240 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d gpurun_out/${TAG}_$N -o pmc -- python3 "$@" > gpurun_out/${TAG}_$N.log 2>&1 || { tail -30 gpurun_out/${TAG}_$N.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/${TAG}_$N --kernel "$K" --min-us $MIN > gpurun_out/${TAG}_$N.txt
  cat gpurun_out/${TAG}_$N.txt
}
run vitadapter7 conv_wave 1000 tools/conv_bench.py --only vit_adapter.7 --prec 0 --tiles 0 --korders 1 --batch 64 --iters 2 --planes --act gelu
run fc1 conv_wave 100 tools/conv_bench.py --only "vit fc1" --prec 0 --tiles 0 --korders 0 --batch 256 --iters 2 --act gelu
timeout -k 10 240 rocprofv3 -i tools/pmc_attn.txt --kernel-trace -d gpurun_out/${TAG}_attn -o pmc -- python3 tools/attn_bench.py --iters 2 > gpurun_out/${TAG}_attn.log 2>&1 || { tail -30 gpurun_out/${TAG}_attn.log; exit 1; }
python tools/pmc_summary.py gpurun_out/${TAG}_attn --kernel vit_attention --min-us 50 > gpurun_out/${TAG}_attn.txt
cat gpurun_out/${TAG}_attn.txt
