#!/bin/bash
# Build a variant of the shipping libhcodec.so with extra flags on hc_fgk.hip only (the other
# objects come from huffman-codec_amd/build) into abvar/<name>/:
#   bash scripts/build_rel.sh <name> [flags...]      e.g. build_rel.sh single -DHC_DEC_PAIR=0
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=abvar/$name
mkdir -p "$out"
make -s -C huffman-codec_amd build/hc_adapt.o build/hc_capi.o build/hc_synth.o build/hc_pipe.o
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Ihuffman-codec_amd/csrc -Wall -Wno-pass-failed \
    -mllvm -structurizecfg-skip-uniform-regions=1 "$@" -c huffman-codec_amd/csrc/hc_fgk.hip -o "$out/hc_fgk.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libhcodec.so" "$out/hc_fgk.o" \
    huffman-codec_amd/build/hc_adapt.o huffman-codec_amd/build/hc_capi.o huffman-codec_amd/build/hc_synth.o huffman-codec_amd/build/hc_pipe.o
rm -f "$out/hc_fgk.o"
echo "built $out/libhcodec.so"
