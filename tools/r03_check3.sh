#!/bin/bash
# round-3 GPU check 3: fused GAT (LDS-shared attention) tests and kernel bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gat_fused.py tests/test_nn.py tests/test_node_loss.py tests/test_node_linear.py tests/test_row_split_policy.py > gpurun_out/r03_check3_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r03_check3_tests.log; exit 1; }
tail -2 gpurun_out/r03_check3_tests.log
$T 300 python tools/gat_bench.py > gpurun_out/gat_bench2.json 2> gpurun_out/gat_bench2.err || { echo "gat bench failed"; tail gpurun_out/gat_bench2.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/gat_bench2.json'))
for r in d: print(r['graph'], r['heads'], r['head_dim'], {k: r[k]['kernel_ms'] for k in r if isinstance(r[k], dict) and 'kernel_ms' in r[k]}, r['fwd_bwd_wall_ms'])"
