#!/bin/bash
# r05 call 13: typed-block g-SpMM with 8 output slices per wave
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_typed_block.py tests/test_examples.py tests/test_distmult.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_typed.log 2>&1
rc=$?; tail -2 $O/pytest_typed.log; [ $rc -eq 0 ] || exit $rc
for w in 1 2 4 1 2 4; do
  timeout -k 10 200 python tools/rgcn_step.py --steps 20 --kernels --typed-width $w > $O/rgcn_w$w.json 2> /dev/null || exit $?
  python -c "
import json; d=json.loads(open('$O/rgcn_w$w.json').read())
k=d['kernels']; print('width $w step', round(d['step_ms'],3), 'fwd', round(k['forward']['ms'],4), 'dH', round(k['dH_ms'],4), 'dW', round(k['dW_ms'],4))"
done
