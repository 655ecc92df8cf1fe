#!/bin/bash
# A/B of parallel-pass variants (abvar/<v>/libhcodec_dbg.so) on C4 / C4m: bench stages
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  HC_LIB_PATH=abvar/$v/libhcodec_dbg.so HC_DBG_LIB_PATH=abvar/$v/libhcodec_dbg.so timeout -k 10 300 \
    python3 -u bench.py --only-configs C4,C4m > gpurun_out/par_ab_$v.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import json, sys
for line in open(f"gpurun_out/par_ab_{sys.argv[1]}.log"):
    if line.startswith("{"):
        d = json.loads(line)
for c in ("C4", "C4m"):
    st = d["configs"][c]["stages"]["decode"]
    print(sys.argv[1], c, {k: st[k]["ms"] for k in ("par_z", "par_scan", "par_walk", "block_boundaries") if k in st},
          "exact:", d["configs"][c].get("reference_digests_identical", d["configs"][c].get("round_trip_exact")))
PY
done
