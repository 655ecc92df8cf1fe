#!/bin/bash
# round-4 session start: headline C5 and the grad / C2 configs on the current tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-configs --steps 3 > gpurun_out/r04_base_c5.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --only-configs grad,C2,C3,noise > gpurun_out/r04_base_cfg.log 2>&1 || exit $?
echo done
