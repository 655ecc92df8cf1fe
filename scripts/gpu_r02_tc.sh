cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
rm -f gpurun_out/t34.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adapt_batch.py tests/test_gpu_adaptive_bounds.py tests/test_gpu_huge.py tests/test_host_batch.py tests/test_gpu_window.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/t34.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/t34.log; exit 1; }
tail -3 gpurun_out/t34.log
for v in B C3; do
  HC_LIB_PATH=build_ab/$v/libhcodec.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/tc$v -o tc -- python3 bench.py --only-configs A512 > gpurun_out/tc$v.log 2>&1 || exit 1
  echo $v; python3 scripts/trace_summary.py gpurun_out/prof/tc$v/tc_kernel_trace.csv | grep -E "tile_cost|emit_tile|big_cost|unblock_tile|bounds|undiff|chunk_sum"; rm -rf gpurun_out/prof/tc$v
done
for v in B C3; do
  HC_LIB_PATH=build_ab/$v/libhcodec.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/pmc$v -o pmc -- python3 bench.py --only-configs A512 > gpurun_out/pmc$v.log 2>&1 || exit 1
  echo pmc $v done
done
