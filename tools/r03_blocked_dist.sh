#!/bin/bash
# Blocked schedule inside the pipelined partition's segments: GPU tests, then
# emulated ranks of the weak-scaled graph (x2, x4, x8) with blocking on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03bd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_blocked.py tests/test_distributed.py > gpurun_out/r03bd/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03bd/tests.log; exit 1; }
tail -1 gpurun_out/r03bd/tests.log
for W in 2 4 8; do
  for P in auto off; do
    DGLHIP_BLOCKED=$P timeout -k 10 300 python bench.py --emulate-world $W --steps 10 --warmup 3 --no-traffic > gpurun_out/r03bd/emu_${W}_${P}.json 2> gpurun_out/r03bd/emu_${W}_${P}.err || { echo "emu $W $P failed"; tail gpurun_out/r03bd/emu_${W}_${P}.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r03bd/emu_${W}_${P}.json').read().strip().splitlines()[-1]); print('$W', '$P', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
