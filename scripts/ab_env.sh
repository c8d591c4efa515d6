#!/bin/bash
# A/B of one environment switch on one GPU box (development):
#   bash scripts/ab_env.sh <tag> <VAR> "<values>" [bench args]
# runs bench.py --no-scan --no-tpch --no-cpu-baseline for every value, twice, alternating.
set -o pipefail
TAG=$1; VAR=$2; VALS=$3; shift 3
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --no-scan --no-tpch --no-cpu-baseline --no-paper --no-configs "$@" \
      > "$OUT/bench_${v}_$rep.json" 2> "$OUT/bench_${v}_$rep.err" || { echo "bench $v failed"; tail -20 "$OUT/bench_${v}_$rep.err"; exit 1; }
    python3 -c "
import json,sys; b=json.load(open('$OUT/bench_${v}_$rep.json')); k=b['rho']['kernel_ms_avg']
print('$VAR=$v rep $rep', b['ms_per_step'], {x: k[x] for x in k if 'scatter' in x or 'hist' in x or 'join_b' in x})"
  done
done
