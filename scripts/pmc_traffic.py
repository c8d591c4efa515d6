#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so fetched bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is
exact for full-line streaming stores (WRITE_SIZE * 1024).  Counters are in KiB.

usage: pmc_traffic.py <run dir with fetch/ and write/> <log2n> <out.json> [summary.md]
"""
import collections
import csv
import glob
import json
import sys

# rocprof kernel name -> bench.py timer names (all launches of one kernel have the
# same size in the bench: |R| = |S|)
ALIASES = {
    "k_hist": ["R_pass1_hist", "S_pass1_hist", "R_pass2_hist", "S_pass2_hist"],
    "k_scatter": ["R_pass1_scatter", "S_pass1_scatter", "R_pass2_scatter", "S_pass2_scatter"],
    "k_join": ["join_build_probe"],
    "k_predicate": ["scan_count", "scan_bitvector"],
    "k_expand": ["scan_expand_index"],
}


def load(pattern, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    run, log2n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    fetch, nf = load(f"{run}/fetch/**/*counter_collection.csv", "FETCH_SIZE")
    write, nw = load(f"{run}/write/**/*counter_collection.csv", "WRITE_SIZE")
    per_kernel = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2 * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        per_kernel[k] = {"read_bytes": round(rd), "write_bytes": round(wr), "total_bytes": round(rd + wr),
                         "launches": nf.get(k, 0)}
    bytes_per_launch = {}
    for k, names in ALIASES.items():
        if k in per_kernel:
            for n in names:
                bytes_per_launch[n] = per_kernel[k]["total_bytes"]
    json.dump({"log2n": log2n, "source": run, "correction": "read = 2 * FETCH_SIZE KiB (gfx950), write = WRITE_SIZE KiB",
               "bytes_per_launch": bytes_per_launch, "per_kernel": per_kernel}, open(out, "w"), indent=1)
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            f.write("| kernel | launches | HBM read (GB/launch) | HBM write (GB/launch) |\n|---|---|---|---|\n")
            for k, v in per_kernel.items():
                if v["total_bytes"] > 1e6:
                    f.write(f"| {k} | {v['launches']} | {v['read_bytes'] / 1e9:.3f} | {v['write_bytes'] / 1e9:.3f} |\n")


if __name__ == "__main__":
    main()
