#!/bin/bash
# round-2 closing run on the GPU box: GPU tests, rocprofv3 stats + PMC passes of the headline
# (profiles/ refresh), then the full bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/final_tests.log gpurun_out/final_bench.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread --durations=5 > gpurun_out/final_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/final_tests.log; exit 1; }
tail -4 gpurun_out/final_tests.log
PASSES="${PASSES:-stats inst wait fetch write}" bash scripts/profile.sh "${TAG:-r02f}" --no-configs --steps 2 --warmup 1 || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/final_bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | cut -c1-600
