#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03sd
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_sddmm_walk.py tests/test_edge_order.py tests/test_gpu_kernels.py tests/test_blocked.py tests/test_gat_fused.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python tools/reducer_bench.py > $OUT/reducers.json 2> $OUT/reducers.err || { echo "reducer bench failed"; tail $OUT/reducers.err; exit 1; }
python -c "
import json
for r in json.load(open('$OUT/reducers.json'))['cases']: print({k: r[k] for k in r if k in ('msg','reduce','variant','edge_order','kernel_ms','frac')})"
timeout -k 10 300 python tools/gat_bench.py > $OUT/gat_bench.json 2> $OUT/gat_bench.err || { echo "gat bench failed"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/gat_bench.json'))
for r in d[:1]: print('gat', {k: (r[k]['kernel_ms'], r[k].get('frac')) for k in r if isinstance(r[k], dict) and 'kernel_ms' in r[k]}, r['fwd_bwd_wall_ms'])"
timeout -k 10 300 python bench.py --emulate-world 2 --steps 10 --warmup 3 --no-traffic > $OUT/emu_2.json 2> $OUT/emu_2.err || { echo "emu failed"; tail $OUT/emu_2.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/emu_2.json').read().strip().splitlines()[-1]); r=d['roofline']; print('emu2', d['ms_per_step'], r['kernel_ms'], r['peak'], r['frac'], r.get('launches_per_call'))"
