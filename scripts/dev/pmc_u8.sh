set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/r03n; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/f -o f --output-format csv -- python3 scripts/dev/scan_u8_ab.py > $OUT/f.log 2>&1 || { tail -5 $OUT/f.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/w -o w --output-format csv -- python3 scripts/dev/scan_u8_ab.py > $OUT/w.log 2>&1 || { tail -5 $OUT/w.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for c in ("f", "w"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r03n/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[(r["Kernel_Name"].split("(")[0][-60:], r["Grid_Size"])].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        if "predicate" in k[0] or "select" in k[0]:
            print(c, k, len(v), sum(v) / len(v))
PY
