#!/bin/bash
# A/B of adaptive-stage builds (AB_DIRS, scripts/tile_exp.py), then the GPU parity suite on the
# in-tree library; no bench. Each GPU step has its own limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/tile_exp.py --reps 5 $AB_DIRS > gpurun_out/ab.log 2>&1
rc=$?; echo "[ab] rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/gpu_tests.log
exit $rc
