#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03gp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/gat_bench.py" --fwd-bwd-only --iters 5 > "$GRAFT_REPO_ROOT/$OUT/fb.json" 2> "$GRAFT_REPO_ROOT/$OUT/fb.err" || { echo "rocprof failed"; tail "$GRAFT_REPO_ROOT/$OUT/fb.err"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r03gp/prof/*kernel_stats.csv')[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r['Name'][:100], r['Calls'], round(float(r['AverageNs'])/1e6, 3), r['Percentage'])
PY
