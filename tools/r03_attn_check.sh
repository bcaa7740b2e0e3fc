#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_blocked.py tests/test_edge_order.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python tools/reducer_bench.py > $OUT/reducers.json 2> $OUT/reducers.err || { echo "reducer bench failed"; tail $OUT/reducers.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/reducers.json').read())
for r in (d if isinstance(d, list) else d.get('results', [])):
    print({k: r[k] for k in r if k in ('msg','reduce','edge_order','kernel_ms','frac')})" || true
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --graph-scale 0.05 --rmat-scale 18 --steps 3 --warmup 1 > $OUT/gloo2.json 2> $OUT/gloo2.err || { echo "gloo2 failed"; tail $OUT/gloo2.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/gloo2.json').read().strip().splitlines()[-1]); print('gloo2', d['n_gpus'], d['value'], d['ms_per_step'])"
