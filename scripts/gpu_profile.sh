#!/bin/bash
# GPU-box profiling run: parity tests, bench line, rocprofv3 kernel-trace stats and
# separate FETCH_SIZE / WRITE_SIZE PMC passes (never combined with other tracing).
# Usage (from the repo root, through gpurun):  bash scripts/gpu_profile.sh <tag> [bench args]
set -o pipefail
TAG=${1:-r01}
shift || true
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"

if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1 \
    || { echo "gpu tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -2 "$OUT/gpu_tests.log"
fi

timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"

[ -n "$SKIP_PROF" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-tpch --no-paper --no-configs --no-tuple-layout "$@" > "$OUT/kt.log" 2>&1 \
  || { echo "kernel-trace failed"; tail -30 "$OUT/kt.log"; exit 1; }
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -30 "$OUT/kernel_stats.csv"

timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o fetch --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-tpch --no-paper --no-configs --no-tuple-layout "$@" > "$OUT/fetch.log" 2>&1 \
  || { echo "pmc FETCH_SIZE failed"; tail -30 "$OUT/fetch.log"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o write --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-tpch --no-paper --no-configs --no-tuple-layout "$@" > "$OUT/write.log" 2>&1 \
  || { echo "pmc WRITE_SIZE failed"; tail -30 "$OUT/write.log"; exit 1; }
find "$OUT/fetch" "$OUT/write" -name "*counter_collection.csv" | head
echo done
