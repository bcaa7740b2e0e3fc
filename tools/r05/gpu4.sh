#!/bin/bash
# r05 call 4: why the headline update_all call runs slower than the direct call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
timeout -k 10 300 python -u tools/r05/diag_headline.py > $O/diag_headline.log 2>&1 || exit $?
tail -1 $O/diag_headline.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/diagprof -o run --output-format csv -- python -u tools/r05/diag_headline.py > $O/diagprof.log 2>&1 || exit $?
echo done
