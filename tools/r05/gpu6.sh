#!/bin/bash
# r05 call 6: the model legs after the DistMult / NodeLinear / fused-Adam /
# lazy-schedule changes: their GPU tests, kernel traces grouped, the legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_distmult.py tests/test_gat_fused.py tests/test_examples.py tests/test_typed_block.py tests/test_nn.py tests/test_message_passing.py tests/test_sddmm_walk.py tests/test_edge_order.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_models.log 2>&1
rc=$?; tail -3 $O/pytest_models.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rgcnprof2 -o run --output-format csv -- python tools/rgcn_step.py --steps 20 > $O/rgcnprof2.log 2>&1 || exit $?
tail -1 $O/rgcnprof2.log
python tools/trace_groups.py $O/rgcnprof2 --steps 43 --out $O/rgcn_step_groups2.json > /dev/null || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gatprof2 -o run --output-format csv -- python examples/gat/train.py --dataset pubmed --gpu 0 --epochs 60 --hip-graph > $O/gatprof2.log 2>&1 || exit $?
tail -1 $O/gatprof2.log
python tools/trace_groups.py $O/gatprof2 --steps 60 --out $O/gat_pubmed_groups2.json > /dev/null || exit $?
timeout -k 10 400 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-train-leg --no-cpu-baseline > $O/bench_models.json 2> $O/bench_models.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_models.json').read().strip().splitlines()[-1])
print('headline', d['ms_per_step']); print('rgcn', d['rgcn']['ms_per_step']); print('gat_pubmed', d['gat_pubmed']['ms_per_epoch_hip_graph'], d['gat_pubmed']['ms_per_epoch']); print('gat', d['gat']['ms_per_step']); print('sage', d['sage']['ms_per_epoch'])"
echo done
