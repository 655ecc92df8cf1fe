#!/bin/bash
# round 4: tile_cost Ev-word variant, A512 stage times (alternating, 3 rounds) + adaptive parity
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
HC_LIB_PATH=abvar/ev/libhcodec.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_adapt_batch.py > gpurun_out/ev_parity.log 2>&1 || { tail -20 gpurun_out/ev_parity.log; exit 1; }
echo "ev parity $(tail -1 gpurun_out/ev_parity.log)"
for r in 1 2 3; do
for v in cur ev; do
  if [ $v = cur ]; then L=huffman-codec_amd/lib/libhcodec.so; else L=abvar/$v/libhcodec.so; fi
  HC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --only-configs A512 > gpurun_out/ev_$v.log 2>&1 || { tail -5 gpurun_out/ev_$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/ev_{sys.argv[1]}.log"):
    if l.startswith("{"):
        c = json.loads(l)["configs"]["A512"]
        print(sys.argv[1], c["encode_ms"], c["decode_ms"], "tile_cost", c["stages"]["encode"]["tile_cost"]["ms"], "emit_tile", c["stages"]["encode"]["emit_tile"]["ms"])
PY
done
done
