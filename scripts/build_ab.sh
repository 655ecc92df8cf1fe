#!/bin/bash
# Build build_ab/A from git HEAD (stash the working tree) and build_ab/B from the working tree.
set -e
cd "$(dirname "$0")/.."
git stash -q
make -s -j4 -C huffman-codec_amd ARCH=gfx950 >/dev/null 2>&1 || { git stash pop -q; exit 1; }
mkdir -p build_ab/A build_ab/B
cp huffman-codec_amd/lib/libhcodec.so build_ab/A/
git stash pop -q
make -s -j4 -C huffman-codec_amd ARCH=gfx950 2>&1 | grep -i error || true
cp huffman-codec_amd/lib/libhcodec.so build_ab/B/
md5sum build_ab/A/libhcodec.so build_ab/B/libhcodec.so
