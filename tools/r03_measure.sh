#!/bin/bash
# round-3 measurement: -m gpu suite, the default bench line, its kernel trace,
# and a DRAM-destined vs all-request PMC pass on the RMAT-26 g-SpMM
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03m
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo "bench failed"; tail -20 $OUT/bench_n1.err; exit 1; }
echo "bench ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 25 --warmup 5 --no-traffic --no-rmat-leg --no-cpu-baseline --no-train-leg > "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.err" || { echo "rocprof bench failed"; exit 1; }
echo "rocprof ok"
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d "$GRAFT_REPO_ROOT/$OUT/pmc_dram" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload rmat --rmat-scale 26 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > "$GRAFT_REPO_ROOT/$OUT/pmc_dram.out" 2>&1
echo "pmc dram rc=$?"
