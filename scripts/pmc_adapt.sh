#!/bin/bash
# one PMC pass over the adaptive A512 config (counters never combined with tracing)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE} --output-format csv -d gpurun_out/prof/pmc_${TAG:-adapt} -o pmc -- python3 bench.py --only-configs ${CONFIGS:-A512} > gpurun_out/pmc_${TAG:-adapt}.log 2>&1
rc=$?
tail -3 gpurun_out/pmc_${TAG:-adapt}.log
exit $rc
