#!/bin/bash
# r05 call 7: headline time by round, cold, then after a GPU test run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 200 python -u tools/r05/clock_probe.py 20 > $O/probe_cold.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gat_fused.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/probe_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/r05/clock_probe.py 20 > $O/probe_after.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-train-leg --no-cpu-baseline --no-model-legs > $O/hl_after.json 2> $O/hl_after.err || exit $?
python -c "import json; d=json.loads(open('$O/hl_after.json').read().strip().splitlines()[-1]); print('hl_after', d['ms_per_step'])"
head -3 $O/probe_cold.log; tail -2 $O/probe_cold.log; head -3 $O/probe_after.log; tail -2 $O/probe_after.log
