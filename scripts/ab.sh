#!/bin/bash
# A/B timing of two builds of libhcodec.so on the GPU box, alternating, in one call:
#   bash scripts/ab.sh <dirA> <dirB> [rounds] [bench args...]
# (dirX/libhcodec.so; each bench run prints its JSON line to gpurun_out/ab.log)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=$1; B=$2; R=${3:-2}; shift 3
rm -f gpurun_out/ab.log
for r in $(seq "$R"); do
    for v in "$A" "$B"; do
        HC_LIB_PATH="$v/libhcodec.so" timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_run.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/ab_run.log; exit 1; }
        echo "$v $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/ab_run.log)" | tee -a gpurun_out/ab.log
    done
done
