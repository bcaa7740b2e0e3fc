#!/bin/bash
# round-3 GPU check 2: fused GAT tests, kernel bench, Pubmed epochs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gat_fused.py tests/test_nn.py tests/test_edge_order.py tests/test_row_split_policy.py tests/test_abi.py > gpurun_out/r03_gat_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r03_gat_tests.log; exit 1; }
tail -2 gpurun_out/r03_gat_tests.log
$T 300 python tools/gat_bench.py > gpurun_out/gat_bench.json 2> gpurun_out/gat_bench.err || { echo "gat bench failed"; tail gpurun_out/gat_bench.err; exit 1; }
for mode in "" "--unfused" "--hip-graph" "--unfused --hip-graph"; do
  echo "pubmed $mode: $($T 200 python examples/gat/train.py --dataset pubmed --gpu 0 --epochs 60 $mode 2>&1 | tail -1)"
done
