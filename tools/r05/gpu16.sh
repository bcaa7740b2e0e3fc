#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/r05/host_costs.py > gpurun_out/r05/host_costs.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/r05/host_costs.txt
