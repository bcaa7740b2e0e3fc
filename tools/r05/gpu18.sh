#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 400 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-train-leg --no-cpu-baseline --no-one-launch-leg > $O/bench_gat.json 2> $O/bench_gat.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_gat.json').read().strip().splitlines()[-1])
g=d['gat']; print('gat', g['ms_per_step'], 'fwd', g['roofline']['kernel_ms'], 'fwd recomputed', g['forward_ms_logits_recomputed'], 'frac', g['roofline']['frac'], 'bwd frac', g.get('roofline_backward',{}).get('frac'))
print('pubmed', d['gat_pubmed']['ms_per_epoch_hip_graph'], 'rgcn', d['rgcn']['ms_per_step'], 'headline', d['ms_per_step'])"
