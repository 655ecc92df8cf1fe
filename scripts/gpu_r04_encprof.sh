#!/bin/bash
# round 4: counters of the encoder (8192 photo -c -m streams): instructions and waits
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ep
mkdir -p $out
B="python3 bench.py --no-cpu-baseline --no-configs --streams 8192 --steps 1 --warmup 1 ${BARGS}"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $out/inst -o inst -- $B > $out/inst.log 2>&1 || { echo "inst rc=$?"; tail -3 $out/inst.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $out/wait -o wait -- $B > $out/wait.log 2>&1 || { echo "wait rc=$?"; exit 1; }
echo done
