#!/bin/bash
# PMC passes over the parallel boundary pass on the 4096^2 streams (scripts/par_diag.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/par_inst -o inst -- python3 scripts/par_diag.py > gpurun_out/prof/par_inst.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH --output-format csv -d gpurun_out/prof/par_wait -o wait -- python3 scripts/par_diag.py > gpurun_out/prof/par_wait.log 2>&1
