cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_adapt_batch.py tests/test_gpu_adaptive_bounds.py tests/test_gpu_parity.py tests/test_fuzz.py tests/test_cli.py tests/test_host_batch.py -m gpu -x -v -rf --timeout 200 --timeout-method thread > gpurun_out/adapt_tests.log 2>&1
rc=$?
tail -30 gpurun_out/adapt_tests.log
exit $rc
