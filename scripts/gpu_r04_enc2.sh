#!/bin/bash
# round 4: encoder chunk loop, quick parity + timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tab.py tests/test_gpu_window.py > gpurun_out/r04_enc_tests.log 2>&1 || { tail -30 gpurun_out/r04_enc_tests.log; exit 1; }
tail -1 gpurun_out/r04_enc_tests.log
timeout -k 10 300 python3 -u bench.py --only-configs ${CFGS:-grad,C3,C2} > gpurun_out/r04_enc_cfg.log 2>&1 || { tail -5 gpurun_out/r04_enc_cfg.log; exit 1; }
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-configs --steps 2 > gpurun_out/r04_enc_c5.log 2>&1 || { tail -5 gpurun_out/r04_enc_c5.log; exit 1; }
echo "C5 $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/r04_enc_c5.log)"
python3 - <<'PY'
import json
for l in open("gpurun_out/r04_enc_cfg.log"):
    if l.startswith("{"):
        for k, v in json.loads(l)["configs"].items():
            print(k, v["encode_ms"], v["decode_ms"], v["round_trip_exact"], v.get("reference_digests_identical"))
PY
