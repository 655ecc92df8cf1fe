#!/bin/bash
# adaptive configs only, under rocprofv3 kernel trace (per-kernel times of the adaptive stages)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u bench.py --only-configs ${CONFIGS:-C4,C4m,A512} > gpurun_out/adapt_bench.log 2>&1 || { tail -20 gpurun_out/adapt_bench.log; exit 1; }
tail -2 gpurun_out/adapt_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/adapt -o adapt -- python3 bench.py --only-configs ${CONFIGS:-C4,C4m,A512} > gpurun_out/adapt_prof.log 2>&1 || { tail -20 gpurun_out/adapt_prof.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/prof/adapt/adapt_kernel_trace.csv
