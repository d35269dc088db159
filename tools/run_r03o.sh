#!/bin/bash
# round 3 (late): full GPU suite + smoke on the current tree, bench kernel trace, bench line
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r03o_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r03o_smoke.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r03o_bench -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/r03o_trace_bench.json 2> $O/r03o_trace_bench.err || exit 3
DB=$(find $O/r03o_bench -name "*.db" | head -1)
python3 tools/prof_summary.py "$DB" --passes 1 --dominant "%conv_halo%" > $O/r03o_kernel_trace.txt
rm -rf $O/r03o_bench
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/r03o_bench.json 2> $O/r03o_bench.err || exit 4
