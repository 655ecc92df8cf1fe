#!/bin/bash
# round 4: counters of the pair decoder against the one-stream decoder (8192 photo -c -m streams)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pp
mkdir -p $out
for v in pair single; do
  if [ $v = pair ]; then L=huffman-codec_amd/lib/libhcodec.so; else L=abvar/single/libhcodec.so; fi
  export HC_LIB_PATH=$L
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $out/${v}_inst -o inst -- python3 bench.py --no-cpu-baseline --no-configs --streams 8192 --steps 1 --warmup 1 > $out/${v}_inst.log 2>&1 || { echo "$v inst rc=$?"; tail -3 $out/${v}_inst.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT --output-format csv -d $out/${v}_wait -o wait -- python3 bench.py --no-cpu-baseline --no-configs --streams 8192 --steps 1 --warmup 1 > $out/${v}_wait.log 2>&1 || { echo "$v wait rc=$?"; tail -3 $out/${v}_wait.log; exit 1; }
  echo "$v ok"
done
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES GRBM_GUI_ACTIVE --output-format csv -d $out/pair_ic -o ic -- python3 bench.py --no-cpu-baseline --no-configs --streams 8192 --steps 1 --warmup 1 > $out/pair_ic.log 2>&1; echo "icache rc=$?"
echo done
