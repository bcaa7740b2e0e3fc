#!/bin/bash
# round-3 measurement with 6 MiB source blocks: -m gpu suite, default bench
# line, its kernel trace + per-call sum, emulated N=2/4/8 ranks, GAT bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/r03m3}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo "bench failed"; tail -20 $OUT/bench_n1.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/bench_n1.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic'), r.get('l2_miss_traffic_frac'), d['train_step']['ms_per_step'])"
for W in 2 4 8; do
  timeout -k 10 300 python bench.py --emulate-world $W --steps 10 --warmup 3 --no-traffic > $OUT/emu_$W.json 2> $OUT/emu_$W.err || { echo "emu $W failed"; tail $OUT/emu_$W.err; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/emu_$W.json').read().strip().splitlines()[-1]); print('emu', $W, d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python tools/gat_bench.py > $OUT/gat_bench.json 2> $OUT/gat_bench.err || { echo "gat bench failed"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/gat_bench.json'))
for r in d[:1]: print('gat', {k: r[k]['kernel_ms'] for k in r if isinstance(r[k], dict) and 'kernel_ms' in r[k]}, r['fwd_bwd_wall_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 25 --warmup 5 --no-traffic --no-rmat-leg --no-cpu-baseline --no-train-leg > "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.err" || { echo "rocprof bench failed"; exit 1; }
cd "$GRAFT_REPO_ROOT"
T=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python tools/kernel_per_call.py "$T" 30 gspmm $OUT/bench_under_rocprof.json > $OUT/kernel_per_call.json && python -c "
import json; d=json.load(open('$OUT/kernel_per_call.json')); print('trace', d['kernel_ms_per_call'], 'bench', d.get('bench_kernel_ms'))"
