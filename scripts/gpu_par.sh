#!/bin/bash
# GPU-box check of the parallel block-boundary pass: its tests, the serial pass's tests, the
# adaptive parity tests (C4 digests), then the adaptive bench configs with their stage times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bounds_par.py tests/test_gpu_adaptive_bounds.py tests/test_gpu_adapt_batch.py -x -q --timeout 600 --timeout-method thread > gpurun_out/par_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/par_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "4096 or adapt" --timeout 600 --timeout-method thread > gpurun_out/par_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/par_parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --only-configs ${CONFIGS:-C4,C4m,A512} --steps 2 > gpurun_out/par_bench.log 2>&1
rc=$?; echo "bench rc=$rc"
exit $rc
