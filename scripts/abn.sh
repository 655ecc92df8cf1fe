#!/bin/bash
# A/B/... timing of several builds of libhcodec.so on the GPU box, alternating, in one call:
#   bash scripts/abn.sh "<dir1> <dir2> ..." [rounds] [bench args...]
# (dirX/libhcodec.so; each bench run's kernel times go to gpurun_out/abn.log)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$1; R=${2:-2}; shift 2
rm -f gpurun_out/abn.log
for r in $(seq "$R"); do
    for v in $V; do
        HC_LIB_PATH="$v/libhcodec.so" timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/abn_run.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/abn_run.log; exit 1; }
        echo "$v $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/abn_run.log | tr '\n' ' ')" | tee -a gpurun_out/abn.log
    done
done
