#!/bin/bash
# adaptive-path GPU check: parity tests, then the adaptive bench configs under rocprofv3 stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests/test_gpu_adapt_batch.py tests/test_gpu_adaptive_bounds.py tests/test_gpu_parity.py tests/test_fuzz.py tests/test_cli.py tests/test_host_batch.py -m gpu -x -v -rf --timeout 200 --timeout-method thread > gpurun_out/adapt_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAIL|Error" gpurun_out/adapt_tests.log | tail -15
[ $rc -ne 0 ] && exit $rc
[ -n "$NOBENCH" ] && exit 0
bash scripts/gpu_bench_adapt.sh
