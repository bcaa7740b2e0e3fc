#!/bin/bash
# block-bytes sweep of the source-blocked schedule: headline (N=1) and emulated ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03bb
for BB in 4194304 4718592 5242880 5767168 6291456 7864320; do
  DGLHIP_BLOCK_BYTES=$BB timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-traffic --no-rmat-leg --no-train-leg --no-cpu-baseline > gpurun_out/r03bb/w1_$BB.json 2> gpurun_out/r03bb/w1_$BB.err || { echo "w1 $BB failed"; tail gpurun_out/r03bb/w1_$BB.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r03bb/w1_$BB.json').read().strip().splitlines()[-1]); print('w1', $BB, round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), flush=True)"
done
for W in 2 4; do
  for BB in 4718592 5242880 7864320; do
    DGLHIP_BLOCK_BYTES=$BB timeout -k 10 200 python bench.py --emulate-world $W --steps 10 --warmup 3 --no-traffic > gpurun_out/r03bb/w${W}_$BB.json 2> gpurun_out/r03bb/w${W}_$BB.err || { echo "w$W $BB failed"; tail gpurun_out/r03bb/w${W}_$BB.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r03bb/w${W}_$BB.json').read().strip().splitlines()[-1]); print('w$W', $BB, round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), flush=True)"
  done
done
