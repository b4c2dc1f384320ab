#!/usr/bin/env python3
"""Per kernel: GRBM_GUI_ACTIVE (GPU clock cycles while busy) over the dispatch's duration, from
a `rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace` run: the effective clock each kernel ran at.
The counter's rows of one dispatch (one per XCD / instance) are reduced with max; durations come
from the run's kernel_trace.csv (Dispatch_Id).

    python3 tools/clock_report.py <rocprofv3 output dir>
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].replace("pn2::", "")


def main():
    d = sys.argv[1]
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc or not kt:
        raise SystemExit(f"need counter_collection.csv and kernel_trace.csv under {d}")
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            dur[(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cyc = defaultdict(float)
    names = {}
    for f in cc:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != "GRBM_GUI_ACTIVE":
                continue
            k = r["Dispatch_Id"]
            cyc[k] = max(cyc[k], float(r["Counter_Value"]))
            names[k] = short(r.get("Kernel_Name", "?"))
    per = defaultdict(list)
    for k, c in cyc.items():
        t = dur.get(k)
        if t and t > 0:
            per[names[k]].append((c, t, c / (t * 1e-3)))
    for name, v in sorted(per.items(), key=lambda kv: -len(kv[1])):
        print(f"{len(v):5d} {name[:60]:60s} us {statistics.median(t for _, t, _ in v) / 1e3:9.1f}"
              f"  cycles {statistics.median(c for c, _, _ in v):11.0f}"
              f"  MHz {statistics.median(m for _, _, m in v):7.0f}")


if __name__ == "__main__":
    main()
