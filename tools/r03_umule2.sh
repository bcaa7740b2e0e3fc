#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03u
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_blocked.py tests/test_gat_fused.py tests/test_edge_order.py > $OUT/tests2.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests2.log; exit 1; }
tail -1 $OUT/tests2.log
timeout -k 10 300 python tools/blocked_ranges_ab.py > $OUT/ab2.json 2> $OUT/ab2.err || { echo "ab failed"; tail $OUT/ab2.err; exit 1; }
python -c "
import json
for r in json.load(open('$OUT/ab2.json'))['cases']: print(r)"
timeout -k 10 300 python tools/gat_bench.py > $OUT/gat.json 2> $OUT/gat.err || { echo "gat failed"; tail $OUT/gat.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/gat.json'))
for r in d[:1]: print('gat', {k: r[k]['kernel_ms'] for k in r if isinstance(r[k], dict) and 'kernel_ms' in r[k]}, r['fwd_bwd_wall_ms'])"
