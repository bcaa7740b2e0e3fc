#!/bin/bash
# Blocked-schedule gate sweep on emulated ranks of the weak-scaled graph:
# minimum slots per row and block x block bytes, N = 1 (headline), 2, 4, 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03bs
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > gpurun_out/r03bs/$tag.json 2> gpurun_out/r03bs/$tag.err || { echo "$tag failed"; tail gpurun_out/r03bs/$tag.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r03bs/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), flush=True)"
}
for W in 4 8 2; do
  for S in 12 16 24; do
    for BB in 7864320 15728640; do
      run w${W}_s${S}_b${BB} DGLHIP_BLOCK_MIN_SLOTS=$S DGLHIP_BLOCK_BYTES=$BB timeout -k 10 200 python bench.py --emulate-world $W --steps 10 --warmup 3 --no-traffic
    done
  done
done
for S in 12 16 24; do
  run w1_s${S} DGLHIP_BLOCK_MIN_SLOTS=$S timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-traffic --no-rmat-leg --no-train-leg --no-cpu-baseline
done
