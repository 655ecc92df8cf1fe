#!/bin/bash
# A/B of whole-library variants on the C5 headline (bench.py --no-configs) and lone streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
for v in "$@"; do
  HC_LIB_PATH=abvar/$v/libhcodec_dbg.so HC_DBG_LIB_PATH=abvar/$v/libhcodec_dbg.so timeout -k 10 300 \
    python3 -u bench.py --no-cpu-baseline --no-configs --steps 3 > gpurun_out/c5_ab_$v.log 2>&1 || exit $?
  echo "$v C5 $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/c5_ab_$v.log)"
done
done
