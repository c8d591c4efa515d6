#!/bin/bash
# Development: config-1 small-join timing (scripts/dev/c1_time.py) of library variants,
# alternating, twice.  Usage (through gpurun): bash scripts/dev/c1_ab.sh <tag> "<names>"
set -o pipefail
TAG=$1; NAMES=$2
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for v in $NAMES; do
    if [ "$v" = base ]; then LP=""; else LP="$PWD/varlib/$v/libsgxamd.so"; fi
    SGXAMD_LIB_PATH=$LP timeout -k 10 120 python scripts/dev/c1_time.py 300 >> "$OUT/c1_ab.log" 2>&1 \
      || { echo "c1 $v failed"; tail -20 "$OUT/c1_ab.log"; exit 1; }
  done
done
cat "$OUT/c1_ab.log"
