#!/bin/bash
# round-3 (session 2): the source-swept schedule vs one launch / blocked on the
# Reddit-shaped graph, then emulated N=2/8 ranks with it on and off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/sweep1}
mkdir -p $OUT
timeout -k 10 400 python -u tools/sweep_study.py ${SWEEP_ARGS} > $OUT/sweep_study.json 2> $OUT/sweep_study.err || { echo "sweep study failed"; tail -20 $OUT/sweep_study.err; exit 1; }
grep -v '"variants"' $OUT/sweep_study.json
for W in 2 8; do
  for S in off on; do
    DGLHIP_SWEEP=$S timeout -k 10 300 python bench.py --emulate-world $W --steps 10 --warmup 3 --no-traffic --no-rmat-leg --no-cpu-baseline --no-train-leg > $OUT/emu_${W}_$S.json 2> $OUT/emu_${W}_$S.err || { echo "emu $W $S failed"; tail $OUT/emu_${W}_$S.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/emu_${W}_$S.json').read().strip().splitlines()[-1]); print('emu', $W, '$S', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
