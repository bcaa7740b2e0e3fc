#!/bin/bash
# r05 call 1: GAT backward 5-wave A/B, its L2 / EA split, headline at 3 MiB slices.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
set -o pipefail
timeout -k 10 240 python -u tools/gat_bwd_variants.py --variants 0 4 --rounds 3 --out $O/gat_bwd_w5.json > $O/gat_bwd_w5.log 2>&1 || exit $?
tail -3 $O/gat_bwd_w5.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/gsa -o run --output-format csv \
  -- python tools/gat_bwd_split.py run --out $O/gat_plan.json > $O/gsa.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/gsb -o run --output-format csv \
  -- python tools/gat_bwd_split.py run --out $O/gat_plan.json > $O/gsb.log 2>&1 || exit $?
python tools/gat_bwd_split.py parse $O/gat_plan.json $O/gsa/run_counter_collection.csv $O/gsb/run_counter_collection.csv --out $O/gat_bwd_l2_split.json > /dev/null || exit $?
( export DGLHIP_BLOCK_BYTES=3145728
  timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/l2b3 -o run \
    --output-format csv -- python tools/l2_split.py run --out $O/l2_plan3.json > $O/l2b3.log 2>&1 ) || exit $?
python tools/l2_split.py parse $O/l2_plan3.json $O/l2b3/run_counter_collection.csv --out $O/l2_split_ea_3mib.json > /dev/null || exit $?
timeout -k 10 240 python tools/block_bytes_percall.py --mib 3 4 6 --rounds 3 > $O/block_bytes_3_4_6.json 2> $O/block_bytes.err || exit $?
cat $O/block_bytes_3_4_6.json | tail -5
echo done
