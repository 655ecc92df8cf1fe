#!/bin/bash
# round 4: counters of the grad -c -m batch (8192 streams): instructions, waits, HBM bytes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/gp
mkdir -p $out
B="python3 bench.py --no-cpu-baseline --no-configs --kind grad --streams 8192 --steps 1 --warmup 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o stats -- $B > $out/stats.log 2>&1 || { echo "stats rc=$?"; tail -3 $out/stats.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $out/inst -o inst -- $B > $out/inst.log 2>&1 || { echo "inst rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $out/wait -o wait -- $B > $out/wait.log 2>&1 || { echo "wait rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- $B > $out/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- $B > $out/write.log 2>&1 || { echo "write rc=$?"; exit 1; }
echo done
