#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests/test_gat_fused.py tests/test_nn.py tests/test_examples.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_logits.log 2>&1
rc=$?; tail -3 $O/pytest_logits.log; exit $rc
