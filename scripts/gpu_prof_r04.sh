#!/bin/bash
# Round-4 closing counter evidence on the final kernels: C5 (65536 photo -c -m), C3 (4096 photo
# -c) and grad (8192 -c -m) as scripts/profile.sh passes, then the A512 kernel stats. Each pass is
# a run of its own with its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
bash scripts/profile.sh r04 --steps 2 --warmup 1 --no-configs || exit $?
bash scripts/profile.sh r04c3 --streams 4096 --no-diff --steps 3 --warmup 1 --no-configs || exit $?
bash scripts/profile.sh r04g --kind grad --streams 8192 --steps 3 --warmup 1 --no-configs || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r04a_stats -o stats \
    -- python3 bench.py --only-configs A512 > gpurun_out/prof/r04a_stats.log 2>&1 || exit $?
echo done
