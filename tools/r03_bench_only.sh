#!/bin/bash
# default bench line, then its kernel trace under rocprofv3 (per-call sum)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/bench}
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo "bench failed"; tail -20 $OUT/bench_n1.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/bench_n1.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic'), d['train_step']['ms_per_step'], d['rmat26']['value'], d['rmat26']['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 25 --warmup 5 --no-traffic --no-rmat-leg --no-cpu-baseline --no-train-leg > "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.err" || { echo "rocprof bench failed"; exit 1; }
cd "$GRAFT_REPO_ROOT"
T=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python tools/kernel_per_call.py "$T" 30 gspmm $OUT/bench_under_rocprof.json > $OUT/kernel_per_call.json && python -c "
import json; d=json.load(open('$OUT/kernel_per_call.json')); print('trace', d['kernel_ms_per_call'], 'bench', d.get('bench_kernel_ms'))"
