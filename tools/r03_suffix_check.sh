#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_blocked.py tests/test_gat_fused.py tests/test_examples.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python examples/gcn/gcn_spmv.py --dataset reddit --gpu 0 --n-hidden 128 --n-epochs 20 > $OUT/gcn.log 2>&1 || { echo "gcn failed"; tail $OUT/gcn.log; exit 1; }
tail -1 $OUT/gcn.log
DGLHIP_BLOCKED=off timeout -k 10 300 python examples/gcn/gcn_spmv.py --dataset reddit --gpu 0 --n-hidden 128 --n-epochs 20 > $OUT/gcn_off.log 2>&1 || { echo "gcn off failed"; tail $OUT/gcn_off.log; exit 1; }
tail -1 $OUT/gcn_off.log
