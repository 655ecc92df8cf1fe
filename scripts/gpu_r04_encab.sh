#!/bin/bash
# round 4: encoder variants, C5 / grad / C2 A/B (alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in ${ROUNDS:-1 2}; do
for v in ${VARIANTS:-cur shallow base}; do
  if [ $v = cur ]; then L=huffman-codec_amd/lib/libhcodec.so; else L=abvar/$v/libhcodec.so; fi
  HC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-configs --steps 2 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  HC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --only-configs ${CFGS:-grad,C2} > gpurun_out/abc_$v.log 2>&1 || { tail -5 gpurun_out/abc_$v.log; exit 1; }
  echo "$v C5 $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/ab_$v.log) $(python3 -c "
import json
for l in open('gpurun_out/abc_$v.log'):
    if l.startswith('{'):
        print(' '.join(f\"{k} {v['encode_ms']:.3f}/{v['decode_ms']:.3f}\" for k, v in json.loads(l)['configs'].items()))
")"
done
done
