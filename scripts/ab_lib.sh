#!/bin/bash
# A/B of library variants (varlib/<name>/libsgxamd.so; "base" = the in-tree build) on one
# GPU box, alternating, twice:  bash scripts/ab_lib.sh <tag> "<names>" [bench args]
set -o pipefail
TAG=$1; NAMES=$2; shift 2
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for v in $NAMES; do
    if [ "$v" = base ]; then LP=""; else LP="$PWD/varlib/$v/libsgxamd.so"; fi
    SGXAMD_LIB_PATH=$LP timeout -k 10 300 python bench.py --no-scan --no-tpch --no-cpu-baseline --no-paper --no-configs "$@" \
      > "$OUT/bench_${v}_$rep.json" 2> "$OUT/bench_${v}_$rep.err" || { echo "bench $v failed"; tail -20 "$OUT/bench_${v}_$rep.err"; exit 1; }
    python3 -c "
import json; b=json.load(open('$OUT/bench_${v}_$rep.json')); k=b['rho']['kernel_ms_avg']
print('$v rep $rep', b['ms_per_step'], {x: k[x] for x in k if 'scatter' in x or 'hist' in x or 'join_b' in x})"
  done
done
