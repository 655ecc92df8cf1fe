cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests/test_gpu_adapt_batch.py tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "adapt or digest" > gpurun_out/t73.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/t73.log; exit 1; }
tail -2 gpurun_out/t73.log
for v in H0 N H0 N; do
  HC_LIB_PATH=abvar/$v/libhcodec.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/tc$v -o tc -- python3 bench.py --only-configs A512 > gpurun_out/tc$v.log 2>&1 || exit 1
  echo $v; python3 scripts/trace_summary.py gpurun_out/prof/tc$v/tc_kernel_trace.csv | grep -E "emit_tile"; rm -rf gpurun_out/prof/tc$v
done
