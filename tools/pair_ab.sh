#!/bin/bash
# Paired-slot gathers (DGLHIP_PAIR_SLOTS 0 / 1) on the GCN leg's F = 41
# aggregation and the headline F = 128 step, one bench process per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pair_ab
for P in ${PAIRS:-0 1 0}; do
  out=gpurun_out/pair_ab/p$P.json
  DGLHIP_PAIR_SLOTS=$P timeout -k 10 400 python bench.py --no-traffic --no-rmat-leg \
    --no-sage-rmat-leg --no-train-leg --no-one-launch-leg --no-cpu-baseline \
    --model-legs gcn_reddit > $out 2> ${out%.json}.err || exit $?
  python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); g=d['gcn_reddit']; print('pair $P headline', round(d['ms_per_step'],3), 'gcn', round(g['ms_per_epoch'],3), g['aggregation_ms'])"
done
