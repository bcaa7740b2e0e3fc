#!/bin/bash
# swept schedule: rounds of resident waves as separate launches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/sweep2}
mkdir -p $OUT
for L in 0 5120 2560; do
  DGLHIP_SWEEP_LAUNCH_WAVES=$L timeout -k 10 300 python -u tools/sweep_study.py --rows 4 8 --slices-mib 1 2 4 256 --iters 5 > $OUT/sweep_L$L.json 2> $OUT/sweep_L$L.err || { echo "sweep study $L failed"; tail -20 $OUT/sweep_L$L.err; exit 1; }
  echo "L=$L"; grep -v '"variants"' $OUT/sweep_L$L.json | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items() if k not in ('launches', 'heavy', 'algorithmic_TBs')})"
done
