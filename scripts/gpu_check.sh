#!/bin/bash
# GPU-box check: parity tests, then (only if the tests did not crash or time out) a bench run.
#   bash scripts/gpu_check.sh [bench args...]
# Every GPU step has its own time limit; a fault / abort / timeout ends the script there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <log> <seconds> <cmd...>: run one GPU step, stop the script on crash/timeout
    local log=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" >> "gpurun_out/$log" 2>&1
    local rc=$?
    echo "[$log] rc=$rc: $*" | tee -a "gpurun_out/$log"
    if [ $rc -gt 1 ]; then
        echo "stopping after exit $rc"
        exit $rc
    fi
    return $rc
}
rm -f gpurun_out/gpu_tests.log gpurun_out/bench.log
step gpu_tests.log 1000 python -u -m pytest tests -m gpu -v -rf --timeout 600 --timeout-method thread --durations=15 -k "not 4096"
step gpu_tests.log 600 python -u -m pytest tests -m gpu -v -rf --timeout 500 --timeout-method thread -k "4096"
step bench.log 600 python -u bench.py "$@"
tail -3 gpurun_out/bench.log
