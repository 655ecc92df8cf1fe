#!/bin/bash
# round 4: encoder variants — a parity subset per variant, then C5 / C2 / C4m timing (alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  if [ $v = cur ]; then L=huffman-codec_amd/lib/libhcodec.so; else L=abvar/$v/libhcodec.so; fi
  HC_LIB_PATH=$L timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "digests or mixed or deep or edge or corpus" > gpurun_out/var_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -20 gpurun_out/var_$v.log; exit 1; }
  echo "$v parity $(tail -1 gpurun_out/var_$v.log)"
done
ROUNDS="1 2" VARIANTS="${VARIANTS}" CFGS=${CFGS:-C2,C4m} bash scripts/gpu_r04_encab.sh
