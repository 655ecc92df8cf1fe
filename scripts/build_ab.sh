#!/bin/bash
# Build abvar/A from git HEAD (stash the working tree) and abvar/B from the working tree.
set -e
cd "$(dirname "$0")/.."
git stash -q
make -s -j4 -C huffman-codec_amd ARCH=gfx950 >/dev/null 2>&1 || { git stash pop -q; exit 1; }
mkdir -p abvar/A abvar/B
cp huffman-codec_amd/lib/libhcodec.so abvar/A/
git stash pop -q
make -s -j4 -C huffman-codec_amd ARCH=gfx950 2>&1 | grep -i error || true
cp huffman-codec_amd/lib/libhcodec.so abvar/B/
md5sum abvar/A/libhcodec.so abvar/B/libhcodec.so
