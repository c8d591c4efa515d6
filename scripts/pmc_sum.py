"""Summarise rocprofv3 counter_collection.csv files: mean counter value per kernel."""
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for k, cs in acc.items():
    if filt not in k: continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:26s} {sum(v)/len(v):16.0f}  (n={len(v)})")
