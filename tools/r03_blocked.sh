#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python tools/blocked_study.py > gpurun_out/blocked_study.json 2> gpurun_out/blocked_study.err
echo "rc=$?"
cat gpurun_out/blocked_study.json | head -8
tail -3 gpurun_out/blocked_study.err
