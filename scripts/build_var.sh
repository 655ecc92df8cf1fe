#!/bin/bash
# Build a variant of libhcodec_dbg.so with extra compiler flags into abvar/<name>/:
#   bash scripts/build_var.sh <name> [flags...]      e.g. build_var.sh nostore -DHC_EXP_NOSTORE
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=abvar/$name
mkdir -p "$out/obj"
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Ihuffman-codec_amd/csrc -Wall -Wno-pass-failed -mllvm -structurizecfg-skip-uniform-regions=1 -DHC_DEBUG_HOOKS"
pids=()
for s in hc_fgk hc_adapt hc_capi hc_synth hc_pipe; do
    /opt/rocm/bin/hipcc $FLAGS "$@" -c huffman-codec_amd/csrc/$s.hip -o "$out/obj/$s.o" &
    pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libhcodec_dbg.so" "$out"/obj/*.o
rm -rf "$out/obj"
echo "built $out/libhcodec_dbg.so"
