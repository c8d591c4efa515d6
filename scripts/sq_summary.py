"""SQ / LDS counter summary per kernel (rocprofv3 --pmc passes of scripts/gpu_counters.sh).

Usage: python3 scripts/sq_summary.py <pmc dir> <out.md> <commit> [kernel substrings...]
Per kernel (mean over its dispatches): the raw counters and
  wait %        = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (wave-cycles spent waiting)
  VALU issue %  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES  (wave-cycles issuing VALU)
  LDS busy %    = SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES
  bank conflict % = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS-array cycles
                  of all LDS-array cycles, MI355X_MICROARCH.md §LDS)
  VALU / wave, LDS instr / wave = SQ_INSTS_VALU, SQ_INSTS_LDS over SQ_WAVES."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    src, out, commit = sys.argv[1:4]
    want = sys.argv[4:] or ["k_scatter_pool", "k_place_seg", "k_join_n", "k_hist_chain", "k_scatter_blk", "k_sort_blk",
                            "k_join_x", "k_join_hist_big", "k_hist_side_blk"]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(src + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            for w in want:
                if w in name:
                    # the template arguments tell variants apart (digit bits, items, key/tuple)
                    key = name.split("(")[0].replace("void sgxamd::rho::", "")[:90]
                    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = [f"# SQ / LDS counters per kernel (commit {commit})", "",
             "Mean per dispatch over the bench's launches (`scripts/gpu_counters.sh`, one rocprofv3 --pmc pass per "
             "counter group, no other tracing).", ""]
    for k in sorted(acc):
        c = {n: sum(v) / len(v) for n, v in acc[k].items()}
        n = {n: len(v) for n, v in acc[k].items()}

        def ratio(a, b, pct=True):
            if a in c and b in c and c[b]:
                return f"{100 * c[a] / c[b]:.1f} %" if pct else f"{c[a] / c[b]:.1f}"
            return "—"

        lines += [f"## `{k}`", "",
                  f"- dispatches: {max(n.values())}",
                  f"- wait: {ratio('SQ_WAIT_ANY', 'SQ_WAVE_CYCLES')}, VALU issue: "
                  f"{ratio('SQ_ACTIVE_INST_VALU', 'SQ_WAVE_CYCLES')}, LDS issue: "
                  f"{ratio('SQ_ACTIVE_INST_LDS', 'SQ_WAVE_CYCLES')}",
                  f"- LDS bank conflicts: {ratio('SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE')} of LDS-array cycles",
                  f"- per wave: VALU {ratio('SQ_INSTS_VALU', 'SQ_WAVES', False)}, LDS {ratio('SQ_INSTS_LDS', 'SQ_WAVES', False)}, "
                  f"SALU {ratio('SQ_INSTS_SALU', 'SQ_WAVES', False)}, VMEM rd {ratio('SQ_INSTS_VMEM_RD', 'SQ_WAVES', False)}, "
                  f"VMEM wr {ratio('SQ_INSTS_VMEM_WR', 'SQ_WAVES', False)}", "",
                  "| counter | mean |", "|---|---|"]
        lines += [f"| {name} | {val:,.0f} |" for name, val in sorted(c.items())]
        lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
