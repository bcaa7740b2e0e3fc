set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_typed_block.py tests/test_distmult.py tests/test_examples.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "typed or distmult or rgcn or grouping" > gpurun_out/tb_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tb_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg \
    --no-train-leg --no-one-launch-leg --no-cpu-baseline --model-legs rgcn > gpurun_out/rgcn_leg.json 2> gpurun_out/rgcn_leg.err
rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/rgcn_leg.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/rgcn_leg.json'))['rgcn']; print(d['ms_per_step'], d['kernel_ms'], d['launches_per_step'])"
done
timeout -k 10 400 python -u tools/rgcn_host_study.py --blas rocblas --out gpurun_out/rgcn_host.json > gpurun_out/rgcn_host.log 2>&1
rc=$?; tail -1 gpurun_out/rgcn_host.log; exit $rc
