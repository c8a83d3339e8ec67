#!/bin/bash
# Build libsks.so with extra compile definitions into variants/libsks_<tag>.so
# (for A/B runs through SKS_LIB=...; *.so stays out of git but ships to the box).
#   bash tools/build_variant.sh slots1024 -DSKS_JOIN_LOG_SLOTS=10
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/pkg"
cp -r "$R/include" "$T/"
cp -r "$R/spaced-kmer-sketching_amd/csrc" "$R/spaced-kmer-sketching_amd/cpp" "$R/spaced-kmer-sketching_amd/Makefile" "$R/spaced-kmer-sketching_amd/srchash.py" "$T/pkg/"
make -s -C "$T/pkg" -j8 CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result $*" lib/libsks.so
mkdir -p "$R/variants"
cp "$T/pkg/lib/libsks.so" "$R/variants/libsks_$TAG.so"
rm -rf "$T"
echo "variants/libsks_$TAG.so"
