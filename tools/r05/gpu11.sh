#!/bin/bash
# r05 call 11: model legs after the small-n split-K weight gradient
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_node_linear.py tests/test_gat_fused.py tests/test_examples.py tests/test_nn.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_models2.log 2>&1
rc=$?; tail -2 $O/pytest_models2.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gatprof3 -o run --output-format csv -- python examples/gat/train.py --dataset pubmed --gpu 0 --epochs 60 --hip-graph > $O/gatprof3.log 2>&1 || exit $?
python tools/trace_groups.py $O/gatprof3 --steps 60 --out $O/gat_pubmed_groups3.json > /dev/null || exit $?
timeout -k 10 400 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-train-leg --no-cpu-baseline --no-one-launch-leg > $O/bench_models2.json 2> $O/bench_models2.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_models2.json').read().strip().splitlines()[-1])
print('headline', d['ms_per_step']); print('rgcn', d['rgcn']['ms_per_step']); print('gat_pubmed', d['gat_pubmed']['ms_per_epoch_hip_graph'], d['gat_pubmed']['ms_per_epoch']); print('gat', d['gat']['ms_per_step']); print('sage', d['sage']['ms_per_epoch'])"
echo done
