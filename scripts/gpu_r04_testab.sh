#!/bin/bash
# round 4: the whole GPU suite on the current build, then an A/B of VARIANTS (parity subset + timing)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r04_testab.log 2>&1 || { tail -40 gpurun_out/r04_testab.log; exit 1; }
tail -1 gpurun_out/r04_testab.log
bash scripts/gpu_r04_varab.sh
