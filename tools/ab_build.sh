#!/bin/bash
# Builds a variant of libneurokmer.so for an A/B timing on one box:
#   tools/ab_build.sh <tag> "<extra hipcc flags>"  ->  tools/bin/ab/<tag>/libneurokmer.so
# then: NK_AB_LIB=tools/bin/ab/<tag>/libneurokmer.so python bench.py ...
set -eu
TAG=$1
EXTRA=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/bin/ab/$TAG
mkdir -p "$OUT/obj"
make -s -j8 -C "$ROOT/neurokmer_amd/csrc" OBJDIR="$OUT/obj" LIBDIR="$OUT" \
  CXXFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -I$ROOT/include $EXTRA" \
  "$OUT/libneurokmer.so"
echo "$OUT/libneurokmer.so"
