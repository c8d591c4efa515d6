#!/bin/bash
# Development: a variant of libsgxamd.so with extra compile flags, for A/B runs through
# SGXAMD_LIB_PATH (scripts/ab_lib.sh).  Usage: bash scripts/build_variant.sh <name> "<flags>"
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../sgxv2-analytical-query-processing-benchmarks_amd"
OUT=../varlib/$NAME
mkdir -p "$OUT"
OBJS=""
for f in csrc/*.hip csrc/*.cpp; do
  b=$(basename "$f"); b=${b%.*}
  [ "$b" = generator ] && continue
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../include -Icsrc $FLAGS \
    $([ "${f##*.}" = hip ] && echo "-x hip") -c "$f" -o "$OUT/$b.o" &
  OBJS="$OBJS $OUT/$b.o"
done
g++ -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc -c csrc/generator.cpp -o "$OUT/generator.host.o" &
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$OUT/libsgxamd.so" $OBJS "$OUT/generator.host.o" -lpthread
rm -f "$OUT"/*.o
echo "built $OUT/libsgxamd.so"
