#!/bin/bash
# A/B of several environment settings on one GPU box (development), alternating:
#   bash scripts/ab_cfg.sh <tag> <reps> "<label>:<VAR=v,VAR2=v2>" ... [-- bench args]
# A label with an empty setting ("base:") runs the defaults.  Prints one line per run:
# ms/step and the big kernels' HIP-event averages.
set -o pipefail
TAG=$1; REPS=$2; shift 2
CFGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do CFGS+=("$1"); shift; done
[ "$1" = "--" ] && shift
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for c in "${CFGS[@]}"; do
    label=${c%%:*}; envs=${c#*:}
    ENVARGS=()
    IFS=',' read -ra KV <<< "$envs"
    for kv in "${KV[@]}"; do [ -n "$kv" ] && ENVARGS+=("$kv"); done
    env "${ENVARGS[@]}" timeout -k 10 300 python bench.py --no-scan --no-tpch --no-cpu-baseline --no-paper --no-configs "$@" \
      > "$OUT/bench_${label}_$rep.json" 2> "$OUT/bench_${label}_$rep.err" \
      || { echo "bench $label failed"; tail -20 "$OUT/bench_${label}_$rep.err"; exit 1; }
    python3 - "$OUT/bench_${label}_$rep.json" "$label" "$rep" <<'EOF'
import json, sys
b = json.load(open(sys.argv[1]))
k = b["rho"]["kernel_ms_avg"]
print(sys.argv[2], "rep", sys.argv[3], b["ms_per_step"],
      {x: round(k[x], 4) for x in k if any(s in x for s in ("scatter", "hist", "join_b", "place"))}, flush=True)
EOF
  done
done
