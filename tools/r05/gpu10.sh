#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 600 python bench.py --no-traffic --no-model-legs --no-train-leg --no-cpu-baseline > $O/bench_rmat.json 2> $O/bench_rmat.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_rmat.json').read().strip().splitlines()[-1])
s=d['sage_rmat26']; print('sage_rmat', s['ms_per_epoch'], s['kernel_ms'], s['alloc_retries'], s['peak_hbm_gb'])
print('rmat', d['rmat26']['ms_per_step'])"
