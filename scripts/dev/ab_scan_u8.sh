#!/bin/bash
# Development: uint8 scan kernel times (scripts/dev/scan_u8_ab.py) for library variants
# (varlib/<name>; "base" = the in-tree build), alternating, twice.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for rep in 1 2; do
  for v in $1; do
    if [ "$v" = base ]; then LP=""; else LP="$PWD/varlib/$v/libsgxamd.so"; fi
    echo "== $v rep $rep"
    SGXAMD_LIB_PATH=$LP timeout -k 10 120 python3 scripts/dev/scan_u8_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
