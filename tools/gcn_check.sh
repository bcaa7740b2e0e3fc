#!/bin/bash
# The GCN example's tests on the device and its bench leg twice (GraphSAGE
# beside it): gpu_check-style, stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_examples.py tests/test_nn.py tests/test_node_linear.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gcn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gcn_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-train-leg \
    --no-one-launch-leg --no-cpu-baseline --model-legs ${LEGS:-gcn_reddit,sage} > gpurun_out/gcn_leg_$i.json 2> gpurun_out/gcn_leg_$i.err
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/gcn_leg_$i.err; exit $rc; }
  python tools/bench_summary.py gpurun_out/gcn_leg_$i.json | grep -E "gcn|sage"
done
