#!/bin/bash
# r05 call 19 (final): the whole GPU suite, smoke, the default bench line
# (every leg, PMC traffic) and the rocprofv3 kernel-trace summary of the
# headline command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
s=$(date +%s)
timeout -k 10 600 python bench.py > $O/bench_full.json 2> $O/bench_full.err || exit $?
echo "bench wall $(( $(date +%s) - s )) s"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/benchprof -o run --output-format csv -- python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-model-legs --no-train-leg --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || exit $?
echo done
