#!/bin/bash
# round 4: pair decoder variants against one stream per wave (C5 decode), then the pair's counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r04_pair_tests.log 2>&1 || { tail -30 gpurun_out/r04_pair_tests.log; exit 1; }
tail -1 gpurun_out/r04_pair_tests.log
for v in ${VARIANTS:-pair prio single}; do
  if [ $v = pair ]; then L=huffman-codec_amd/lib/libhcodec.so; else L=abvar/$v/libhcodec.so; fi
  HC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-configs --steps 2 > gpurun_out/r04_pair_$v.log 2>&1 || { tail -5 gpurun_out/r04_pair_$v.log; exit 1; }
  echo "$v C5 $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/r04_pair_$v.log)"
done
HC_LIB_PATH=huffman-codec_amd/lib/libhcodec.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pp/pair2_wait -o wait -- python3 bench.py --no-cpu-baseline --no-configs --streams 8192 --steps 1 --warmup 1 > gpurun_out/pp/pair2_wait.log 2>&1; echo "pmc rc=$?"
