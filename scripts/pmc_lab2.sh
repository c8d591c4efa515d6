#!/bin/bash
# PMC passes (FETCH_SIZE, then SQ / TCC groups) over one command.
# Usage: bash scripts/pmc_lab2.sh <tag> <cmd...>
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1 \
    || { echo "pmc pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
echo done
