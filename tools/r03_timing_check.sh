#!/bin/bash
# per-call kernel timing: default bench line, a 2-rank gloo line on one GPU,
# and the timing test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/timing}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k per_call_timing --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "test failed"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo "bench failed"; tail -20 $OUT/bench_n1.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/bench_n1.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['train_step']['ms_per_step'], d['train_step'].get('kernel_ms_rank0'), d['rmat26']['value'], d['rmat26']['ms_per_step'], d['rmat26']['roofline']['kernel_ms'])"
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --graph-scale 0.25 --rmat-scale 22 --steps 5 --warmup 2 > $OUT/gpus2_gloo.json 2> $OUT/gpus2.err || { echo "gpus2 failed"; tail -20 $OUT/gpus2.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/gpus2_gloo.json').read().strip().splitlines()[-1]); r=d['roofline']; print('gpus2', d['n_gpus'], d['value'], d['ms_per_step'], r['kernel_ms'], [p['kernel_ms'] for p in r['per_rank']])"
