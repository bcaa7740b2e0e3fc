#!/bin/bash
# round-3 GPU check 4: kernel breakdown of the fused GAT forward + backward
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gatprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/gatprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/gat_bench.py" --fwd-bwd-only --iters 5 > "$GRAFT_REPO_ROOT/gpurun_out/gatprof/out.txt" 2>&1
echo "rc=$?"
ls "$GRAFT_REPO_ROOT/gpurun_out/gatprof"
