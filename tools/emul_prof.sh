#!/bin/bash
# Kernel trace of the emulated rank-0 step (bench.py --emulate-world W
# --pipeline-chunks C), its timed steps' kernels alone (tools/window_stats.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/emulprof -o run --output-format csv \
  -- python bench.py --emulate-world ${W:-8} --pipeline-chunks ${C:-4} --steps 10 --warmup 3 --no-traffic \
  > gpurun_out/emulprof.json 2> gpurun_out/emulprof.log
rc=$?; tail -1 gpurun_out/emulprof.log; [ $rc -eq 0 ] || exit $rc
python tools/window_stats.py gpurun_out/emulprof/run_kernel_trace.csv --window 0 \
  --out gpurun_out/emulprof/timed_kernel_stats.csv
