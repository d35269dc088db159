#!/bin/bash
# same-box A/B of the LDS-DMA upconv in the model (bench, concurrent heads), alternating arms
set -o pipefail
O=gpurun_out
for i in 1 2; do
  for D in 1 0; do
    PRPE_UPCONV_DMA=$D timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03c_bench_dma${D}_$i.json 2> $O/r03c_bench_dma${D}_$i.err || exit 1
  done
done
for f in $O/r03c_bench_dma*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
