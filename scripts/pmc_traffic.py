#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so fetched bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is
exact for full-line streaming stores (WRITE_SIZE * 1024).  Counters are in KiB.

The profiled command may launch the same kernel at several sizes (bench.py's RHO
passes at 2^28 beside small TPC-H joins): per bench timer name only the launches of
the bench's size are averaged, i.e. those within 2x of the kernel's largest launch.

usage: pmc_traffic.py <run dir with fetch/ and write/> <log2n> <out.json> [summary.md]
"""
import collections
import csv
import glob
import json
import os
import sys

# rocprof kernel name -> bench.py timer names (|R| = |S| in the bench, so the launches
# of one kernel at the bench's size move the same bytes)
ALIASES = {
    "k_hist": ["R_pass1_hist", "S_pass1_hist"],
    "k_hist_side": ["R_pass2_hist", "S_pass2_hist"],
    # pooled two-pass plans (one kernel per pass; listed after BY_GRID, so they win)
    "k_scatter_pool": ["R_pass1_scatter", "S_pass1_scatter"],
    "k_scatter_blk": ["R_pass2_scatter", "S_pass2_scatter"],
    "k_sort_blk": ["R_pass2_scatter", "S_pass2_scatter"],
    "k_hist_side_blk": ["R_pass2_hist", "S_pass2_hist"],
    "k_hist_chain": ["R_pass2_hist", "S_pass2_hist"],  # chain-histogram plans (round 6)
    "k_join": ["join_build_probe"],
    "k_join_tag": ["join_build_probe"],
    "k_join_x": ["join_build_probe"],
    "k_predicate": ["scan_count", "scan_bitvector"],
    "k_select": ["scan_select_index"],
    # narrow plans (round 5): the segment placement and the one-task-per-workgroup
    # build/probe; k_sort_blk / k_join_x are then launched beside them and return at once
    # (their near-empty launches are skipped below)
    "k_place_seg": ["R_pass2_scatter", "S_pass2_scatter"],
    "k_join_n": ["join_build_probe"],
}
# kernels whose bench-size launches differ per pass, told apart by grid size (pass 2's
# grid is its segments + one per pass-1 bin, larger than pass 1's): smallest grid first
BY_GRID = {"k_scatter": [["R_pass1_scatter", "S_pass1_scatter"], ["R_pass2_scatter", "S_pass2_scatter"]]}


def base_name(k: str) -> str:
    """'void sgxamd::rho::k_scatter<8, 8, 512, true>(...)' -> 'k_scatter'."""
    k = k.split("(")[0].split("<")[0]
    return k.split("::")[-1].split()[-1]


def load(pattern, counter):
    """kernel -> [(dispatch id, grid size, value)] in dispatch order."""
    vals = collections.defaultdict(list)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[base_name(r["Kernel_Name"])].append(
                    (int(r["Dispatch_Id"]), int(r["Grid_Size"]), float(r["Counter_Value"])))
    return {k: sorted(v) for k, v in vals.items()}


def mean(v):
    return sum(v) / len(v) if v else 0.0


def main():
    run, log2n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    fetch = load(f"{run}/fetch/**/*counter_collection.csv", "FETCH_SIZE")
    write = load(f"{run}/write/**/*counter_collection.csv", "WRITE_SIZE")
    per_kernel = {}
    grids = {}
    for k in sorted(set(fetch) | set(write)):
        rd = [2 * x[2] * 1024 for x in fetch.get(k, [])]
        wr = [x[2] * 1024 for x in write.get(k, [])]
        gs = [x[1] for x in (fetch.get(k) or write.get(k))]
        n = min(len(rd), len(wr)) if rd and wr else max(len(rd), len(wr))
        rd = (rd or [0.0] * n)[:n]
        wr = (wr or [0.0] * n)[:n]
        # bench-size launches: total bytes within 2x of the largest launch (both passes
        # launch the kernels in the same order, so index i is the same launch)
        tot = [a + b for a, b in zip(rd, wr)]
        top = max(tot) if tot else 0.0
        sel = [i for i, t in enumerate(tot) if t >= top / 2]
        per_kernel[k] = {"read_bytes": round(mean([rd[i] for i in sel])),
                         "write_bytes": round(mean([wr[i] for i in sel])),
                         "total_bytes": round(mean([tot[i] for i in sel])), "launches": len(sel),
                         "launches_all_sizes": n}
        by_grid = collections.defaultdict(list)
        for i in sel:
            by_grid[gs[i]].append(tot[i])
        grids[k] = {g: round(mean(v)) for g, v in sorted(by_grid.items())}
        if len(grids[k]) > 1:
            per_kernel[k]["total_bytes_by_grid"] = grids[k]
    bytes_per_launch = {}
    for k, groups in BY_GRID.items():
        if k in grids:
            vals = list(grids[k].values())
            for i, names in enumerate(groups):
                for name in names:
                    bytes_per_launch[name] = vals[min(i, len(vals) - 1)]
    for k, names in ALIASES.items():
        if k in per_kernel and per_kernel[k]["total_bytes"] > 1e6:
            for name in names:
                bytes_per_launch[name] = per_kernel[k]["total_bytes"]
    json.dump({"log2n": log2n, "source": run, "commit": os.environ.get("COMMIT", "unknown"),
               "correction": "read = 2 * FETCH_SIZE KiB (gfx950), write = WRITE_SIZE KiB; per kernel, the mean "
                             "over launches within 2x of its largest launch (the bench-size ones)",
               "bytes_per_launch": bytes_per_launch, "per_kernel": per_kernel}, open(out, "w"), indent=1)
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            f.write("| kernel | bench-size launches | HBM read (GB/launch) | HBM write (GB/launch) |\n"
                    "|---|---|---|---|\n")
            for k, v in per_kernel.items():
                if v["total_bytes"] > 1e6:
                    f.write(f"| {k} | {v['launches']} | {v['read_bytes'] / 1e9:.3f} | {v['write_bytes'] / 1e9:.3f} |\n")


if __name__ == "__main__":
    main()
