#!/bin/bash
# round-2 closing run: GPU tests, the adaptive configs under rocprofv3 (kernel trace + stats, one
# PMC pass on A512), then the full bench line. Every GPU step has its own limit; a failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
rm -rf gpurun_out/prof/close_adapt gpurun_out/prof/close_pmc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread --durations=5 > gpurun_out/close_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/close_tests.log; exit 1; }
tail -2 gpurun_out/close_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/close_adapt -o adapt -- python3 bench.py --only-configs C4,C4m,A512 > gpurun_out/close_adapt.log 2>&1 || { echo "adapt prof rc=$?"; tail -20 gpurun_out/close_adapt.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/close_pmc -o pmc -- python3 bench.py --only-configs A512 > gpurun_out/close_pmc.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
timeout -k 10 900 python -u bench.py > gpurun_out/close_bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/close_bench.log; exit 1; }
tail -1 gpurun_out/close_bench.log | cut -c1-400
