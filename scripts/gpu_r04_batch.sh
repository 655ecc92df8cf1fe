#!/bin/bash
# round 4: batched encoder hot path — parity of every encoder path, then A/B against the one-symbol loop
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tab.py tests/test_gpu_window.py tests/test_gpu_wide.py tests/test_gpu_huge.py tests/test_gpu_c5.py > gpurun_out/r04_batch_tests.log 2>&1 || { tail -40 gpurun_out/r04_batch_tests.log; exit 1; }
tail -1 gpurun_out/r04_batch_tests.log
VARIANTS="cur nobatch" CFGS=grad,C2,noise,C4m bash scripts/gpu_r04_encab.sh
