#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
PROBE_SAVEALL=1 PROBE_SCHEDULE_FIRST=1 timeout -k 10 200 python -u tools/r05/clock_probe.py 12 > $O/probe_gc.log 2>&1 || exit $?
grep -v amdgpu $O/probe_gc.log
