#!/bin/bash
# Round-3 (second session): A/B of the adaptive tile kernels (abvar/<dirs>), then the full
# GPU check (parity tests + bench). Every GPU step has its own limit; a crash ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$AB_DIRS" ]; then
    timeout -k 10 300 python -u scripts/tile_exp.py --reps 5 $AB_DIRS > gpurun_out/ab.log 2>&1
    rc=$?; echo "[ab] rc=$rc"; tail -30 gpurun_out/ab.log
    [ $rc -ne 0 ] && exit $rc
fi
[ -n "$AB_ONLY" ] && exit 0
bash scripts/gpu_check.sh "$@"
