#!/bin/bash
# round 4: two streams per wavefront in the decoder — parity, then C5 A/B against one per wave
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c5.py > gpurun_out/r04_pair_tests.log 2>&1 || { tail -30 gpurun_out/r04_pair_tests.log; exit 1; }
tail -3 gpurun_out/r04_pair_tests.log
for r in 1 2; do
for v in pair single; do
  if [ $v = pair ]; then L=huffman-codec_amd/lib/libhcodec.so; else L=abvar/single/libhcodec.so; fi
  HC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-configs --steps 3 > gpurun_out/r04_pair_$v.log 2>&1 || { tail -5 gpurun_out/r04_pair_$v.log; exit 1; }
  echo "$v C5 $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/r04_pair_$v.log)"
done
done
