#!/bin/bash
# Partition microbenchmark on the GPU box (development):
#   bash scripts/part_bench.sh <log2n> "<bits list>" "<variant list>"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}/sgxv2-analytical-query-processing-benchmarks_amd/tools" || exit 1
[ -x part_bench ] || { echo "part_bench not built"; exit 1; }
for b in $2; do
  for v in $3; do
    echo "== part_bench $1 $b $v"
    timeout -k 10 120 ./part_bench "$1" "$b" "$v" | grep -E "scatter|verify|FAIL|bad" || exit 1
  done
done
