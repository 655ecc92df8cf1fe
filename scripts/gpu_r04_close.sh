#!/bin/bash
# round 4: the new parity test, then the default bench line (its fields summarised)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r04_close_tests.log 2>&1 || { tail -30 gpurun_out/r04_close_tests.log; exit 1; }
tail -1 gpurun_out/r04_close_tests.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r04_bench_final.log 2>&1 || { tail -10 gpurun_out/r04_bench_final.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r04_bench_final.log"):
    if l.startswith("{"):
        r = json.loads(l)
        print(r["value"], r["encode_ms"], r["decode_ms"], json.dumps(r["roofline"]), json.dumps(r.get("issue")))
        for k, v in r["configs"].items():
            print(k, v.get("encode_ms"), v.get("decode_ms"), v.get("GiBps"), v.get("traffic") is not None, v.get("round_trip_exact"))
PY
