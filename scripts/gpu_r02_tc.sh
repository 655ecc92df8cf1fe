cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --only-configs A512,C4m > gpurun_out/stages.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/stages.log; exit 1; }
tail -1 gpurun_out/stages.log | cut -c1-300
