#!/bin/bash
# GPU-box: the -m gpu parity tests on the in-tree library, then (only if they pass) an A/B
# timing of two builds (scripts/ab.sh).
#   bash scripts/test_ab.sh <dirA> <dirB> [rounds] [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
tail -15 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
bash scripts/ab.sh "$@"
