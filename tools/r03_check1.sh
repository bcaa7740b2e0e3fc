#!/bin/bash
# round-3 GPU check: new tests, the bench launcher with 2 gloo ranks, counter list
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
(cd /tmp && TMPDIR=/tmp timeout -k 10 120 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters_list.txt" 2>&1) || echo "counter list failed"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_grad_handoff.py tests/test_inc_known_answers.py > gpurun_out/r03_tests1.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03_tests1.log; exit 1; }
tail -3 gpurun_out/r03_tests1.log
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --graph-scale 0.05 --rmat-scale 18 --steps 3 --warmup 1 > gpurun_out/bench_gpus2_gloo.json 2> gpurun_out/bench_gpus2_gloo.log
echo "bench rc=$?"
