#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03it
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_blocked.py tests/test_golden_reddit_rows.py tests/test_gpu_kernels.py tests/test_gat_fused.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python tools/blocked_ranges_ab.py > $OUT/ab.json 2> $OUT/ab.err || { echo "ab failed"; tail $OUT/ab.err; exit 1; }
python -c "
import json
for r in json.load(open('$OUT/ab.json'))['cases']: print(r)"
