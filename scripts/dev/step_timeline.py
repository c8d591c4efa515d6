"""Development: one join step's kernels from a rocprofv3 kernel trace (the launches
between two consecutive R pass-1 scatters of the bench's timed loop): duration of each
kernel and the gap before it, their sums, and the step's span.
Usage: python scripts/dev/step_timeline.py <kt_kernel_trace.csv> [which step, default 2]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].strip()
# a step opens with R's pass-1 scatter: a k_scatter_pool that follows the previous
# step's tail (k_reduce and its result copy), not a pass-2 kernel or a guarded repeat
bounds = [i for i, r in enumerate(rows) if name(r) == "k_scatter_pool" and i > 0
          and name(rows[i - 1]) in ("k_reduce", "__amd_rocclr_copyBuffer", "k_join_x", "k_join_n")]
a, b = bounds[which], bounds[which + 1]
ksum = gsum = 0.0
t0 = int(rows[a]["Start_Timestamp"])
last_end = None
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - last_end) / 1e3 if last_end else 0.0
    d = (e - s) / 1e3
    ksum += d
    gsum += max(gap, 0.0)
    print(f"{name(r):24s} {d:9.1f} us  gap {gap:6.1f}")
    last_end = e
print(f"kernels {b - a}: sum {ksum:.1f} us, gaps {gsum:.1f} us, span {(last_end - t0) / 1e3:.1f} us")
