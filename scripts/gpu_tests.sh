#!/bin/bash
# GPU-box parity run: the whole -m gpu suite (or the tests named in $@), one process,
# per-test timeout; the log goes to gpurun_out/<tag>/gpu_tests.log.
# Usage (through gpurun):  bash scripts/gpu_tests.sh <tag> [pytest selectors]
set -o pipefail
TAG=${1:-r02}
shift || true
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
SEL=${@:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gpu_tests.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -30
exit $rc
