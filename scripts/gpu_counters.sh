#!/bin/bash
# SQ / LDS counter passes over the headline join (one rocprofv3 --pmc pass per group,
# never combined with other tracing), summarised per kernel into
# gpurun_out/<tag>/sq_summary.md.  Usage (through gpurun): bash scripts/gpu_counters.sh <tag> [bench args]
set -o pipefail
TAG=${1:-r03}
shift || true
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/sq$i" -o sq$i --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-scan --no-tpch --no-paper --no-configs --no-tuple-layout \
       --no-cpu-baseline "$@" > "$OUT/sq$i.log" 2>&1 \
    || { echo "pmc pass $i failed"; tail -20 "$OUT/sq$i.log"; exit 1; }
done
python3 scripts/sq_summary.py "$OUT" "$OUT/sq_summary.md" "${COMMIT:-unknown}"
