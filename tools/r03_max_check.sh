#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03mx
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_blocked.py tests/test_max_reducer.py tests/test_message_passing.py tests/test_gpu_kernels.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python tools/reducer_bench.py > $OUT/reducers.json 2> $OUT/reducers.err || { echo "reducer bench failed"; tail $OUT/reducers.err; exit 1; }
python -c "
import json
for r in json.load(open('$OUT/reducers.json'))['cases'][:6]: print({k: r[k] for k in r if k in ('msg','reduce','edge_order','kernel_ms','launches','frac')})"
