#!/bin/bash
# GPU-box script: PMC counters (tools/pmc_conv.txt passes) of the trunk's latency-bound launches
# in isolation -- the stem conv and the layer1.0 conv3 + downsample dual GEMM (bs 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in stem dual; do
  timeout -k 10 240 rocprofv3 -i tools/pmc_conv.txt --kernel-trace -d gpurun_out/tp_$W -o pmc -- python3 tools/trunk_kernels.py $W --batch 64 > gpurun_out/tp_$W.log 2>&1 || { tail -30 gpurun_out/tp_$W.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/tp_$W --kernel conv_wave_kernel --min-us 200 > gpurun_out/tp_$W.txt
  rm -rf gpurun_out/tp_$W
  echo "== $W"; cat gpurun_out/tp_$W.txt
done
