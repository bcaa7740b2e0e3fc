#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03g
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gat_fused.py tests/test_edge_order.py tests/test_sddmm_walk.py > gpurun_out/r03g/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03g/tests.log; exit 1; }
tail -1 gpurun_out/r03g/tests.log
timeout -k 10 300 python tools/gat_bench.py > gpurun_out/r03g/gat_bench.json 2> gpurun_out/r03g/gat_bench.err || { echo "gat bench failed"; tail gpurun_out/r03g/gat_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r03g/gat_bench.json'))
for r in d: print(r['graph'], r['head_dim'], {k: r[k]['kernel_ms'] for k in r if isinstance(r[k], dict) and 'kernel_ms' in r[k]}, r['fwd_bwd_wall_ms'])"
