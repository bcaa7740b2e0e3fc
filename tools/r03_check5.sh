#!/bin/bash
# round-3 GPU check 5: fused GAT backward (attention-gradient epilogue)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gatprof2
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gat_fused.py tests/test_nn.py tests/test_edge_order.py tests/test_sddmm_walk.py tests/test_message_passing.py > gpurun_out/r03_check5_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r03_check5_tests.log; exit 1; }
tail -2 gpurun_out/r03_check5_tests.log
$T 300 python tools/gat_bench.py > gpurun_out/gat_bench3.json 2> gpurun_out/gat_bench3.err || { echo "gat bench failed"; tail gpurun_out/gat_bench3.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/gat_bench3.json'))
for r in d: print(r['graph'], r['heads'], r['head_dim'], {k: r[k]['kernel_ms'] for k in r if isinstance(r[k], dict) and 'kernel_ms' in r[k]}, r['fwd_bwd_wall_ms'])"
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/gatprof2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/gat_bench.py" --fwd-bwd-only --iters 5 > "$GRAFT_REPO_ROOT/gpurun_out/gatprof2/out.txt" 2>&1
echo "prof rc=$?"
