#!/bin/bash
# rocprofv3 on the GPU box: a kernel-trace/stats pass, then separate PMC passes (counters never
# combined with runtime / sys tracing). Outputs under gpurun_out/prof/<tag>_*.
#   bash scripts/profile.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-run}
shift
mkdir -p gpurun_out/prof
out=gpurun_out/prof
run() {  # run <name> <seconds> <rocprof args...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" rocprofv3 "$@" --output-format csv -d "$out/${tag}_$name" -o "$name" \
        -- python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}" > "$out/${tag}_$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"
    tail -2 "$out/${tag}_$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
BENCH_ARGS=("$@")
PASSES=${PASSES:-stats inst wait fetch write}  # subset: PASSES="inst wait" bash scripts/profile.sh ...
for p in $PASSES; do
    case $p in
    stats) run stats 600 --kernel-trace --stats ;;
    inst) run pmc_inst 600 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE ;;
    wait) run pmc_wait 600 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT ;;
    branch) run pmc_branch 600 --kernel-trace --pmc SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INSTS_VMEM SQ_INSTS_FLAT GRBM_GUI_ACTIVE ;;
    occ) run pmc_occ 600 --kernel-trace --pmc SQ_LEVEL_WAVES SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES ;;
    fetch) run pmc_fetch 600 --kernel-trace --pmc FETCH_SIZE ;;
    write) run pmc_write 600 --kernel-trace --pmc WRITE_SIZE ;;
    esac
done
echo done
