#!/bin/bash
# emulated rank compute vs pipeline chunk count under the blocked schedule
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03c
for W in 4 8; do
  for C in 1 2 4 8; do
    timeout -k 10 200 python bench.py --emulate-world $W --pipeline-chunks $C --steps 10 --warmup 3 --no-traffic > gpurun_out/r03c/w${W}_c$C.json 2> gpurun_out/r03c/w${W}_c$C.err || { echo "w$W c$C failed"; tail gpurun_out/r03c/w${W}_c$C.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r03c/w${W}_c$C.json').read().strip().splitlines()[-1]); r=d['roofline']; print('w$W c$C', round(d['ms_per_step'],3), round(r['kernel_ms'],3), r.get('launches_per_call'), flush=True)"
  done
done
