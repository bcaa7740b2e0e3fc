#!/bin/bash
# r05 call 2: the native launch plan behind every g-SpMM: the whole GPU suite,
# smoke, the quick bench line, and the packed er/dz A/B of the GAT backward.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
# (gat pack A/B done in the first run of this script)

timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py --no-traffic --no-rmat-leg > $O/benchquick.json 2> $O/benchquick.err || exit $?
cat $O/benchquick.json
echo done
