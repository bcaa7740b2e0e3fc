#!/bin/bash
# round-3 measurement after the source-blocked schedule: -m gpu suite, the
# default bench line (PMC traffic, rmat26 and train legs), the kernel trace of
# the headline and its per-call sum beside the bench's own kernel_ms
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03m2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo "bench failed"; tail -20 $OUT/bench_n1.err; exit 1; }
echo "bench ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 25 --warmup 5 --no-traffic --no-rmat-leg --no-cpu-baseline --no-train-leg > "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.err" || { echo "rocprof bench failed"; exit 1; }
echo "rocprof ok"
cd "$GRAFT_REPO_ROOT"
T=$(ls $OUT/prof/*kernel_trace.csv 2>/dev/null | head -1 || true)
[ -z "$T" ] && T=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python tools/kernel_per_call.py "$T" 30 gspmm $OUT/bench_under_rocprof.json > $OUT/kernel_per_call.json && python -c "
import json; d=json.load(open('$OUT/kernel_per_call.json')); print('trace', d['kernel_ms_per_call'], 'bench', d.get('bench_kernel_ms'))"
