cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for v in x0 x1; do
  HC_LIB_PATH=abvar/$v/libhcodec_dbg.so HC_DBG_LIB_PATH=abvar/$v/libhcodec_dbg.so timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES FETCH_SIZE --output-format csv -d gpurun_out/prof/xcd_$v -o pmc -- python3 bench.py --only-configs A512 > gpurun_out/xcd_$v.log 2>&1 || exit $?
done
