#!/bin/bash
# builds scripts/micro/first_call against the in-tree libhcodec.so
cd "$(dirname "$0")/../.."
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude -o scripts/micro/first_call scripts/micro/first_call.cpp \
    -Lhuffman-codec_amd/lib -lhcodec -Wl,-rpath,'$ORIGIN/../../huffman-codec_amd/lib'
