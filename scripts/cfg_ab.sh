#!/bin/bash
# A/B of whole-library variants (abvar/<v>/libhcodec_dbg.so) on bench configs:
#   CONFIGS=C3,noise bash scripts/cfg_ab.sh base variant ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
for v in "$@"; do
  HC_LIB_PATH=abvar/$v/libhcodec_dbg.so HC_DBG_LIB_PATH=abvar/$v/libhcodec_dbg.so timeout -k 10 400 \
    python3 -u bench.py --only-configs ${CONFIGS:-C3} > gpurun_out/cfg_ab_$v.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import json, sys
for line in open(f"gpurun_out/cfg_ab_{sys.argv[1]}.log"):
    if line.startswith("{"):
        d = json.loads(line)
print(sys.argv[1], {c: (v.get("encode_ms"), v.get("decode_ms"), v.get("reference_digests_identical", v.get("round_trip_exact"))) for c, v in d["configs"].items()}, flush=True)
PY
done
done
