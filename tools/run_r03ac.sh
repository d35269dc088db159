#!/bin/bash
# round 3: the SHIPPED bottleneck kernel with its launch bound read as waves per SIMD (WPC * NW / 4),
# applied by sed and built
# ON THE BOX (the committed tree keeps the shipped kernel): tests, micro-bench, model, bench
set -o pipefail
O=gpurun_out
mkdir -p $O
for a in "" "--proj" "--mid 128"; do timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only $a >> $O/r03ac_bneck_bench_shipped.txt 2>&1 || exit 8; done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03ac_bench_shipped.json 2> $O/r03ac_bench_shipped.err || exit 8
sed -i 's/__launch_bounds__(NW \* 64, (BShape<MIDT, PROJ>::WPC))/__launch_bounds__(NW * 64, (BShape<MIDT, PROJ>::WPC * NW \/ 4))/' person-recognition-for-pose-estimation_amd/csrc/conv_bneck.hip
grep -c 'WPC \* NW / 4' person-recognition-for-pose-estimation_amd/csrc/conv_bneck.hip || exit 7
timeout -k 10 600 python person-recognition-for-pose-estimation_amd/build.py --jobs 16 > $O/r03ac_build.log 2>&1 || exit 9
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > $O/r03ac_bneck_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only > $O/r03ac_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only --proj >> $O/r03ac_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 200 python tools/bneck_bench.py --batch 256 --iters 10 --fused-only --mid 128 >> $O/r03ac_bneck_bench.txt 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_contracts.py -x -q --timeout 300 --timeout-method thread > $O/r03ac_model.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/r03ac_bench.json 2> $O/r03ac_bench.err || exit 4
