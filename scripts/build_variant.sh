#!/bin/bash
# Development: a variant of libsgxamd.so with extra compile flags, for A/B runs through
# SGXAMD_LIB_PATH (scripts/ab_lib.sh).  Usage: bash scripts/build_variant.sh <name> "<flags>"
# Only the sources in $VARIANT_SRC (default: the join kernels) are compiled with the
# flags; every other object comes from the in-tree build (run make first).
set -e
NAME=$1; FLAGS=$2
SRC=${VARIANT_SRC:-csrc/rho_kernels.hip}
cd "$(dirname "$0")/../sgxv2-analytical-query-processing-benchmarks_amd"
OUT=../varlib/$NAME
mkdir -p "$OUT"
OBJS=""
for o in build/*.o; do
  b=$(basename "$o" .o)
  skip=0
  for f in $SRC; do [ "$(basename "${f%.*}")" = "$b" ] && skip=1; done
  [ $skip = 1 ] || OBJS="$OBJS $o"
done
for f in $SRC; do
  b=$(basename "${f%.*}")
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../include -Icsrc $FLAGS \
    $([ "${f##*.}" = hip ] && echo "-x hip") -c "$f" -o "$OUT/$b.o" &
  OBJS="$OBJS $OUT/$b.o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$OUT/libsgxamd.so" $OBJS -lpthread
rm -f "$OUT"/*.o
echo "built $OUT/libsgxamd.so"
