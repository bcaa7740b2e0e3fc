#!/bin/bash
# mean_add / blocked-plan tests on the device and the GraphSAGE leg twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export DGLHIP_TEST_BLOCKED_MEAN_ADD=1 DGLHIP_BLOCKED_MEAN_ADD=${DGLHIP_BLOCKED_MEAN_ADD:-1}
timeout -k 10 600 python -u -m pytest tests/test_mean_add.py tests/test_blocked.py tests/test_capi_plan.py tests/test_gpu_kernels.py tests/test_node_linear.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sage_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sage_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-train-leg \
    --no-one-launch-leg --no-cpu-baseline --model-legs sage,gcn_reddit > gpurun_out/sage_leg_$i.json 2> gpurun_out/sage_leg_$i.err
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/sage_leg_$i.err; exit $rc; }
  python tools/bench_summary.py gpurun_out/sage_leg_$i.json | grep -E "gcn|sage"
done
