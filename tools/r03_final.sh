#!/bin/bash
# round-end validation: the -m gpu suite, smoke(), the default bench line and
# its rocprofv3 kernel statistics
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/final}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
OUT=$OUT bash tools/r03_bench_only.sh
