#!/bin/bash
# Emulated rank 0 of the weak-scaled Reddit-shaped graph (bench.py --emulate-world N,
# pipelined halo in 4 chunks) under the blocked schedule's slot rule / stretch cap
# (DGLHIP_BLOCK_MIN_SLOTS, DGLHIP_BLOCK_MAX_STRETCH): ms per step and kernel ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/emul_sweep
for w in ${EMUL_WORLDS:-2 4 8}; do
  for cfg in ${CFGS:-12:3 8:3 8:6 6:6}; do
    ms=${cfg%%:*}; st=${cfg##*:}
    tag=w${w}_s${ms}_x${st}
    DGLHIP_BLOCK_MIN_SLOTS=$ms DGLHIP_BLOCK_MAX_STRETCH=$st timeout -k 10 300 \
      python bench.py --workload reddit --emulate-world $w --pipeline-chunks 4 --steps 10 --warmup 3 \
      --no-traffic > gpurun_out/emul_sweep/$tag.json 2> gpurun_out/emul_sweep/$tag.err
    rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/emul_sweep/$tag.err; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/emul_sweep/$tag.json')); print('$tag', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['roofline'].get('launches_per_call'))"
  done
done
