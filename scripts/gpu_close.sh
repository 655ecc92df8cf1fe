#!/bin/bash
# Closing run on the GPU box: the whole -m gpu suite, smoke, then the default bench line, with a
# one-screen summary. Logs: gpurun_out/<tag>_{tests,smoke,bench}.log
#   bash scripts/gpu_close.sh <tag> [bench args...]
# Every GPU step has its own time limit; a failure, fault or timeout ends the script there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-close}
shift
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
    || { tail -10 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 900 python3 -u bench.py "$@" > gpurun_out/${tag}_bench.log 2>&1 || { tail -10 gpurun_out/${tag}_bench.log; exit 1; }
python3 scripts/bench_summary.py gpurun_out/${tag}_bench.log
