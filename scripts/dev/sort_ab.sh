#!/bin/bash
# Development: k_sort_blk compile-time variants (varlib/<name>; "base" = the in-tree build):
# the join bench A/B (scripts/ab_lib.sh) and one WRITE_SIZE pass per variant over
# scripts/dev/pass2_ab.py.  Usage (through gpurun): bash scripts/dev/sort_ab.sh <tag> "<names>"
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
TAG=$1; NAMES=$2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
bash scripts/ab_lib.sh "$TAG/ab" "$NAMES" > "$OUT/ab.log" 2>&1 || { cat "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
for v in $NAMES; do
  if [ "$v" = base ]; then LP=""; else LP="$PWD/varlib/$v/libsgxamd.so"; fi
  SGXAMD_LIB_PATH=$LP timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/w_$v" -o w --output-format csv \
    -- python3 scripts/dev/pass2_ab.py > "$OUT/w_$v.log" 2>&1 || { echo "pmc $v failed"; tail -5 "$OUT/w_$v.log"; exit 1; }
done
echo done
