#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03ef
mkdir -p $OUT
for W in 2 4 8; do
  timeout -k 10 300 python bench.py --emulate-world $W --steps 10 --warmup 3 --no-traffic > $OUT/emu_$W.json 2> $OUT/emu_$W.err || { echo "emu $W failed"; tail $OUT/emu_$W.err; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/emu_$W.json').read().strip().splitlines()[-1]); r=d['roofline']; print('emu', $W, round(d['ms_per_step'],3), round(r['kernel_ms'],3), r.get('launches_per_call'), round(r['frac'],3))"
done
timeout -k 10 600 python bench.py --no-traffic --no-rmat-leg > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
