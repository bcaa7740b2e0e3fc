#!/bin/bash
# four gloo ranks on one GPU through bench.py's own launcher (every leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03d
timeout -k 10 600 python bench.py --gpus 4 --dist-backend gloo --graph-scale 0.05 --rmat-scale 20 --steps 3 --warmup 1 > gpurun_out/r03d/gpus4_gloo.json 2> gpurun_out/r03d/gpus4.err || { echo "gpus4 failed"; tail -20 gpurun_out/r03d/gpus4.err; exit 1; }
echo gpus4 ok
