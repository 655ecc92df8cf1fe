cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/t54.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_tab.py tests/test_gpu_parity.py tests/test_gpu_huge.py tests/test_gpu_wide.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/t54.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/t54.log; exit 1; }
tail -2 gpurun_out/t54.log
bash scripts/abn.sh "build_ab/K2 build_ab/M" 2 --only-configs C3,noise,C4 || exit 1
