#!/usr/bin/env python3
"""Per-instantiation kernel table from a rocprofv3 --kernel-trace CSV.

    python3 tools/kernel_table.py gpurun_out/prof_<tag>/run_kernel_trace.csv [--md]

rocprofv3's --stats file aggregates by base name (every fps_v2_kernel<...> instantiation in
one row); this splits by full template signature so each SA/FP layer's kernel gets its own
mean / min duration (ns -> us)."""
import csv
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("pn2::", "")
    return name.split("(")[0]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    acc = defaultdict(list)
    for r in rows:
        key = short(r["Kernel_Name"])
        if "<" not in key:  # truncated names (-T): tell launches apart by their shape
            g = "x".join(r.get(f"Grid_Size_{a}", "?") for a in "XYZ")
            key += f" [grid {g}, wg {r.get('Workgroup_Size_X', '?')}]"
        acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tab = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    md = "--md" in sys.argv
    if md:
        print("| kernel | launches | mean us | min us | total us |\n|---|---|---|---|---|")
    for k, v in tab:
        if md:
            print(f"| `{k[:70]}` | {len(v)} | {statistics.mean(v):.1f} | {min(v):.1f} | {sum(v):.0f} |")
        else:
            print(f"{k[:80]:80s} n={len(v):5d} mean={statistics.mean(v):9.1f} min={min(v):9.1f} us")


if __name__ == "__main__":
    main()
