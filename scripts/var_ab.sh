#!/bin/bash
# A/B of library variants on the GPU box, alternating: a parity subset per variant, then per round
# the C5 headline (bench.py --no-configs) and the configs CFGS (bench.py --only-configs).
#   VARIANTS="cur v1 v2" ROUNDS="1 2" CFGS=grad,C2 bash scripts/var_ab.sh
# cur = the in-tree build; v = abvar/v/ (scripts/build_rel.sh: libhcodec.so, or build_var.sh:
# libhcodec_dbg.so, loaded for both). CFGS=none skips the configs; C5=0 skips the headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
lib() {
    if [ "$1" = cur ]; then echo huffman-codec_amd/lib/libhcodec.so
    elif [ -f "abvar/$1/libhcodec.so" ]; then echo "abvar/$1/libhcodec.so"
    else echo "abvar/$1/libhcodec_dbg.so"; fi
}
dbg() { if [ -f "abvar/$1/libhcodec_dbg.so" ]; then echo "abvar/$1/libhcodec_dbg.so"; fi; }
for v in ${VARIANTS:-cur}; do
    HC_LIB_PATH=$(lib $v) HC_DBG_LIB_PATH=$(dbg $v) timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
        --timeout-method thread tests/test_gpu_parity.py -k "${PARITY_K:-digests or mixed or deep or edge or corpus}" \
        > gpurun_out/var_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -20 gpurun_out/var_$v.log; exit 1; }
    echo "$v parity $(tail -1 gpurun_out/var_$v.log)"
done
for r in ${ROUNDS:-1 2}; do
    for v in ${VARIANTS:-cur}; do
        line="$v"
        if [ "${C5:-1}" != 0 ]; then
            HC_LIB_PATH=$(lib $v) HC_DBG_LIB_PATH=$(dbg $v) timeout -k 10 300 python3 -u bench.py --no-cpu-baseline \
                --no-configs --steps ${STEPS:-2} > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
            line="$line C5 $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/ab_$v.log)"
        fi
        if [ "${CFGS:-grad,C2}" != none ]; then
            HC_LIB_PATH=$(lib $v) HC_DBG_LIB_PATH=$(dbg $v) timeout -k 10 400 python3 -u bench.py \
                --only-configs ${CFGS:-grad,C2} > gpurun_out/abc_$v.log 2>&1 || { tail -5 gpurun_out/abc_$v.log; exit 1; }
            line="$line $(python3 -c "
import json
for l in open('gpurun_out/abc_$v.log'):
    if l.startswith('{'):
        print(' '.join(f\"{k} {c.get('encode_ms', 0):.3f}/{c.get('decode_ms', 0):.3f}\" for k, c in json.loads(l)['configs'].items() if k != 'C1'))
")"
        fi
        echo "$line" | tee -a gpurun_out/var_ab.log
    done
done
