#!/bin/bash
# GPU-box: parity tests on the in-tree library, then A/B timings of two builds on the headline
# config (-c -m) and on -c (scripts/ab.sh).
#   bash scripts/test_ab2.sh <dirA> <dirB> [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/test_ab.sh "$1" "$2" "${3:-2}" || exit $?
cp gpurun_out/ab.log gpurun_out/ab_m.log
bash scripts/ab.sh "$1" "$2" "${3:-2}" --no-diff
