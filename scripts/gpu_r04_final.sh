#!/bin/bash
# round 4 closing run: the whole GPU suite and smoke on the current build, an A/B of VARIANTS
# (one round), then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r04_final_tests.log 2>&1 || { tail -40 gpurun_out/r04_final_tests.log; exit 1; }
tail -1 gpurun_out/r04_final_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || { tail -10 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
if [ -n "$VARIANTS" ]; then ROUNDS=1 bash scripts/gpu_r04_encab.sh || exit 1; fi
timeout -k 10 600 python3 -u bench.py > gpurun_out/r04_bench.log 2>&1 || { tail -10 gpurun_out/r04_bench.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r04_bench.log"):
    if l.startswith("{"):
        r = json.loads(l)
        print("C5", r["value"], r["encode_ms"], r["decode_ms"], r["roofline"]["frac"], (r.get("cpu_baseline") or {}).get("value"))
        for k, v in r.get("configs", {}).items():
            print(k, v.get("encode_ms"), v.get("decode_ms"), v.get("GiBps"), v.get("round_trip_exact"), v.get("reference_digests_identical"))
PY
