#!/bin/bash
# Development: WRITE_SIZE per launch of one kernel for library variants (one PMC pass
# each, nothing else traced).  Usage (through gpurun):
#   bash scripts/dev/write_ab.sh <tag> "<names>" <kernel>
set -o pipefail
TAG=$1; NAMES=$2; KERNEL=$3
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in $NAMES; do
  if [ "$v" = base ]; then LP=""; else LP="$PWD/varlib/$v/libsgxamd.so"; fi
  SGXAMD_LIB_PATH=$LP timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/w_$v" -o w --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-scan --no-tpch --no-cpu-baseline --no-paper --no-configs \
    --no-tuple-layout > "$OUT/w_$v.log" 2>&1 || { echo "pmc $v failed"; tail -20 "$OUT/w_$v.log"; exit 1; }
  python3 - "$OUT/w_$v" "$KERNEL" "$v" <<'EOF'
import csv, glob, sys
d, k, v = sys.argv[1:4]
vals = []
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "WRITE_SIZE" and r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1] == k:
            vals.append(float(r["Counter_Value"]) * 1024 / 1e9)
big = sorted(x for x in vals if x > 0.01)
print(v, k, "GB written per launch:", [round(x, 4) for x in big])
EOF
done
