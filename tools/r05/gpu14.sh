#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_blocked.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_blocked.log 2>&1
rc=$?; tail -3 $O/pytest_blocked.log; exit $rc
