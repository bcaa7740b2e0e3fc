#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_accumulate.py > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
timeout -k 10 400 python tools/gather_mode_ab.py > gpurun_out/gather_mode_ab.json 2> gpurun_out/gather_mode_ab.err
echo "ab rc=$?"
cat gpurun_out/gather_mode_ab.json
