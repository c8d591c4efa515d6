#!/bin/bash
# Development: SQ / LDS counters of the uint8 scan kernels (scripts/dev/scan_u8_ab.py),
# one rocprofv3 --pmc pass per group, summarised by scripts/sq_summary.py.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${1:-r03sq8}; mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp -d "$OUT/sq$i" -o sq$i --output-format csv \
    -- python3 scripts/dev/scan_u8_ab.py > "$OUT/sq$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/sq$i.log"; exit 1; }
done
python3 scripts/sq_summary.py "$OUT" "$OUT/sq_summary.md" "${COMMIT:-unknown}" k_select k_predicate
