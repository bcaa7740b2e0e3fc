#!/bin/bash
# the bench's multi-rank path on one GPU: a world-1 RCCL group, then two gloo
# ranks started by bench.py's own launcher
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03d
timeout -k 10 300 python bench.py --dist-rehearsal --graph-scale 0.5 --rmat-scale 24 --steps 10 --warmup 3 > gpurun_out/r03d/rehearsal_world1_rccl.json 2> gpurun_out/r03d/rehearsal.err || { echo "rehearsal failed"; tail -20 gpurun_out/r03d/rehearsal.err; exit 1; }
echo rehearsal ok
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --graph-scale 0.25 --rmat-scale 22 --steps 5 --warmup 2 > gpurun_out/r03d/gpus2_gloo.json 2> gpurun_out/r03d/gpus2.err || { echo "gpus2 failed"; tail -20 gpurun_out/r03d/gpus2.err; exit 1; }
echo gpus2 ok
