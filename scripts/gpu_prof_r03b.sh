#!/bin/bash
# Round-3 closing counter evidence on the final kernels: the C5 headline (65536 photo -c -m
# streams) and C3 (4096 photo -c) as scripts/profile.sh passes, then the A512 adaptive kernel
# stats and PMC passes (scripts/pmc_adapt.sh). Each pass is a run of its own with its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
bash scripts/profile.sh r03b --steps 2 --warmup 1 --no-configs || exit $?
bash scripts/profile.sh r03bc3 --streams 4096 --no-diff --steps 3 --warmup 1 --no-configs || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r03ba_stats -o stats \
    -- python3 bench.py --only-configs A512 > gpurun_out/prof/r03ba_stats.log 2>&1 || exit $?
echo "[adapt stats] done"
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
    TAG=r03ba_inst bash scripts/pmc_adapt.sh || exit $?
PMC="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU FETCH_SIZE" TAG=r03ba_wait bash scripts/pmc_adapt.sh || exit $?
PMC="SQ_WAVES WRITE_SIZE" TAG=r03ba_write bash scripts/pmc_adapt.sh || exit $?
echo done
