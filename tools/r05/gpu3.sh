#!/bin/bash
# r05 call 3: where the model legs' non-engine time goes (kernel traces of the
# R-GCN step and the GAT-Pubmed HIP-graph epoch, grouped), and the GAT
# backward's source-block size re-swept with the packed er/dz table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/rgcnprof -o run \
  --output-format csv -- python tools/rgcn_step.py --steps 20 > $O/rgcnprof.log 2>&1 || exit $?
tail -2 $O/rgcnprof.log
python tools/trace_groups.py $O/rgcnprof --steps 43 --out $O/rgcn_step_groups.json > /dev/null || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/gatprof -o run \
  --output-format csv -- python examples/gat/train.py --dataset pubmed --gpu 0 --epochs 60 --hip-graph \
  > $O/gatprof.log 2>&1 || exit $?
tail -2 $O/gatprof.log
python tools/trace_groups.py $O/gatprof --steps 60 --out $O/gat_pubmed_groups.json > /dev/null || exit $?
timeout -k 10 400 python -u tools/gat_bwd_sweep.py --rounds 2 --out $O/gat_bwd_sweep_packed.json > $O/gat_bwd_sweep.log 2>&1 || exit $?
tail -1 $O/gat_bwd_sweep.log
echo done
