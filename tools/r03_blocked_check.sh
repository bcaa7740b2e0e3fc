#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03b
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_blocked.py tests/test_gpu_kernels.py tests/test_accumulate.py tests/test_message_passing.py tests/test_golden_reddit_rows.py tests/test_mean_add.py tests/test_examples.py > gpurun_out/r03b/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03b/tests.log; exit 1; }
tail -1 gpurun_out/r03b/tests.log
timeout -k 10 400 python bench.py --no-traffic --no-rmat-leg > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err || { echo "bench failed"; tail gpurun_out/r03b/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r03b/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['achieved'], d.get('train_step',{}).get('ms_per_step'))"
