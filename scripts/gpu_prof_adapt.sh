#!/bin/bash
# Adaptive evidence on A512 (8192 x 512^2 photo -c -a -m): kernel trace + stats, then two
# PMC passes (instruction mix; waits and HBM bytes), each a run of its own.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${TAG0:-r05a}_stats -o stats \
    -- python3 bench.py --only-configs A512 > gpurun_out/prof/${TAG0:-r05a}_stats.log 2>&1 || exit $?
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
    TAG=${TAG0:-r05a}_inst bash scripts/pmc_adapt.sh || exit $?
PMC="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU FETCH_SIZE" TAG=${TAG0:-r05a}_wait bash scripts/pmc_adapt.sh || exit $?
PMC="SQ_WAVES WRITE_SIZE" TAG=${TAG0:-r05a}_write bash scripts/pmc_adapt.sh || exit $?
echo done
