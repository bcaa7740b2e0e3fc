set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/sagerm -o run --output-format csv -- python bench.py --no-traffic --no-train-leg --no-one-launch-leg --no-cpu-baseline --no-model-legs > gpurun_out/sagerm.json 2> gpurun_out/sagerm.log
rc=$?; tail -2 gpurun_out/sagerm.log; [ $rc -eq 0 ] || exit $rc
for w in 0 1 2 3; do python tools/window_stats.py gpurun_out/sagerm/run_kernel_trace.csv --window $w --out gpurun_out/sagerm/w$w.csv || true; done
