#!/bin/bash
# GPU-box run: selected -m gpu tests (args after the tag), then the default bench line.
# Usage (through gpurun):  bash scripts/gpu_bench_tests.sh <tag> [pytest selectors]
set -o pipefail
TAG=${1:-r02}
shift || true
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|Error|assert" "$OUT/gpu_tests.log" | tail -30; exit 1; }
  grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -3
fi
timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
