#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/r05/rgcn_host_profile.py > gpurun_out/r05/rgcn_host_profile.txt 2>&1 || exit $?
head -45 gpurun_out/r05/rgcn_host_profile.txt
