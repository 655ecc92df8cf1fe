#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_adapt_batch.py tests/test_gpu_tab.py tests/test_gpu_parity.py -x -q -k "4096 or adapt or stage or enc_mode or tab" --timeout 600 --timeout-method thread > gpurun_out/par_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/par_parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --only-configs C4,C4m,A512,mixed,C3 --steps 2 > gpurun_out/par_bench.log 2>&1
rc=$?; echo "bench rc=$rc"
exit $rc
