#!/bin/bash
# Variant build of libragen_amd.so for A/B timing (diagnostic): one source recompiled with extra
# -D flags, linked with the regular objects of ragen_amd/_build.
#   tools/build_variant.sh NAME SOURCE.hip [-DFLAG=...]   -> tools/_build/libragen_amd_NAME.so
set -eu
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; shift 2
OUTD=${VARIANT_DIR:-tools/_build}  # (tools/_build stays here; VARIANT_DIR=variants ships to the GPU box)
mkdir -p tools/_build "$OUTD"
B=$(basename "$SRC")
/opt/rocm/bin/hipcc -c -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden \
  -Iinclude -Iragen_amd/csrc "$@" "ragen_amd/csrc/$B" -o "tools/_build/${B}_$NAME.o"
OBJS=$(ls ragen_amd/_build/*.o | grep -v "/$B.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUTD/libragen_amd_$NAME.so" $OBJS \
  "tools/_build/${B}_$NAME.o" -lpthread
echo "$OUTD/libragen_amd_$NAME.so"
