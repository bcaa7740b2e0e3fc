#!/bin/bash
# the whole -m gpu suite, as the driver runs it at round end
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r03.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_r03.log
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_r03.log | head
exit $rc
