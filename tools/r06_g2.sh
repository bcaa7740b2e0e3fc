set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_typed_block.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tb_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tb_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1 0 1; do
  DGLHIP_TYPED_MESSAGES=$m timeout -k 10 200 python -u tools/rgcn_step.py --kernels --out gpurun_out/rgcn_msg$m.json > gpurun_out/rgcn_msg$m.log 2>&1
  rc=$?; tail -1 gpurun_out/rgcn_msg$m.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
for m in 0 1; do
  DGLHIP_TYPED_MESSAGES=$m timeout -k 10 300 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg \
    --no-train-leg --no-one-launch-leg --no-cpu-baseline --model-legs rgcn > gpurun_out/rgcn_leg$m.json 2> gpurun_out/rgcn_leg$m.err
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/rgcn_leg$m.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/rgcn_leg$m.json'))['rgcn']; print($m, d['ms_per_step'], d['kernel_ms'], d['typed_block_kernels']['forward']['ms'], d['typed_block_kernels']['dH_ms'], d['typed_block_kernels']['dW_ms'])"
done
