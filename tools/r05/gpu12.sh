#!/bin/bash
# r05 call 12: GAT backward g store through 16-B write-through stores (variant 3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 400 python -u tools/gat_bwd_variants.py --variants 0 3 2 --rounds 3 --out $O/gat_bwd_sc1.json > $O/gat_bwd_sc1.log 2>&1 || exit $?
tail -2 $O/gat_bwd_sc1.log
