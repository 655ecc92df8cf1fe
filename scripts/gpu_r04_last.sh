#!/bin/bash
# round 4, last kernel change: the whole GPU suite, the closing counters, the path profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r04_last_tests.log 2>&1 || { tail -40 gpurun_out/r04_last_tests.log; exit 1; }
tail -1 gpurun_out/r04_last_tests.log
bash scripts/gpu_prof_r04.sh > gpurun_out/prof_r04.log 2>&1 || { tail -20 gpurun_out/prof_r04.log; exit 1; }
tail -1 gpurun_out/prof_r04.log
HC_DBG_LIB_PATH=abvar/P/libhcodec.so timeout -k 10 300 python3 scripts/path_prof.py --streams 8192 > gpurun_out/pprof.log 2>&1 && cat gpurun_out/pprof.log
