#!/bin/bash
# r05 call 5: the headline line at the default warm-up and at a long one
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
F="--no-traffic --no-rmat-leg --no-sage-rmat-leg --no-model-legs --no-train-leg --no-cpu-baseline"
timeout -k 10 300 python bench.py $F > $O/hl_default.json 2> $O/hl_default.err || exit $?
timeout -k 10 300 python bench.py $F --warmup 100 > $O/hl_w100.json 2> $O/hl_w100.err || exit $?
timeout -k 10 300 python bench.py $F --steps 200 > $O/hl_s200.json 2> $O/hl_s200.err || exit $?
for f in hl_default hl_w100 hl_s200; do python -c "import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['roofline']['kernel_ms'])"; done
