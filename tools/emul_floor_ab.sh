#!/bin/bash
# Emulated rank 0 (bench.py --emulate-world W --pipeline-chunks 4) with the
# accumulating sweep's floors at their defaults and lowered (every halo chunk
# and the own segment on the sweep), per W; one line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/emul_floor
for W in ${WORLDS:-2 4 8}; do
  for mode in default low; do
    if [ $mode = low ]; then
      export DGLHIP_SWEEP_ACCUM_TABLE_MIN=33554432 DGLHIP_SWEEP_ACCUM_MIN_SLOTS=32
    else
      unset DGLHIP_SWEEP_ACCUM_TABLE_MIN DGLHIP_SWEEP_ACCUM_MIN_SLOTS
    fi
    out=gpurun_out/emul_floor/w${W}_$mode.json
    timeout -k 10 300 python bench.py --emulate-world $W --pipeline-chunks 4 --steps 10 \
      --warmup 3 --no-traffic > $out 2> ${out%.json}.err || exit $?
    python -c "import json; d=json.load(open('$out')); print('W=$W $mode', round(d['ms_per_step'], 3), round(d['roofline']['kernel_ms'], 3))"
  done
done
