#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rmat26.py -x -v -s -m gpu --timeout 400 --timeout-method thread -k graphsage > gpurun_out/rmat_test.log 2>&1
rc=$?
grep -o "{'graph': 'rmat-26'.*" gpurun_out/rmat_test.log
tail -2 gpurun_out/rmat_test.log
exit $rc
