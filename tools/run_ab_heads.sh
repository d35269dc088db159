#!/bin/bash
# GPU-box script: bench with concurrent vs sequential heads (same box, back to back)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_conc_$TAG.json 2> gpurun_out/bench_conc_$TAG.err || { tail -20 gpurun_out/bench_conc_$TAG.err; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --sequential-heads > gpurun_out/bench_seq_$TAG.json 2> gpurun_out/bench_seq_$TAG.err || { tail -20 gpurun_out/bench_seq_$TAG.err; exit 1; }
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d['roofline'] or {}
    print(f, d['value'], d['ms_per_step'], r.get('avg_launch_ms'))
" gpurun_out/bench_conc_$TAG.json gpurun_out/bench_seq_$TAG.json
