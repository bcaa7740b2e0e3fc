#!/bin/bash
# r05 call 9: the default bench line (every leg, PMC traffic), then the
# rocprofv3 kernel-trace summary of the headline command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
s=$(date +%s)
timeout -k 10 900 python bench.py > $O/bench_full.json 2> $O/bench_full.err || exit $?
echo "bench wall $(( $(date +%s) - s )) s"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/benchprof -o run --output-format csv -- python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-model-legs --no-train-leg --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || exit $?
echo done
