#!/bin/bash
# Emulated rank 0 at W ranks (bench.py --emulate-world W --pipeline-chunks 4)
# per source-sweep block size (DGLHIP_SWEEP_BLOCK_BYTES, MiB list in MIBS);
# one line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/emul_block
W=${W:-8}
for mib in ${MIBS:-6 3 4 2 6}; do
  export DGLHIP_SWEEP_BLOCK_BYTES=$((mib * 1048576))
  out=gpurun_out/emul_block/w${W}_${mib}mib.json
  timeout -k 10 300 python bench.py --emulate-world $W --pipeline-chunks 4 --steps 10 \
    --warmup 3 --no-traffic > $out 2> ${out%.json}.err || exit $?
  python -c "import json; d=json.load(open('$out')); print('W=$W ${mib}MiB', round(d['ms_per_step'], 3), round(d['roofline']['kernel_ms'], 3))"
done
