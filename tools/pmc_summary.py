#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

    python3 tools/pmc_summary.py <fetch_pass_dir> <write_pass_dir> > pmc_traffic.json

Units and corrections follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are
reported in KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane)
coalesced read, so `fetch_bytes_x2` is the corrected figure for such kernels and
`fetch_bytes` the raw one (other access widths are uncalibrated). WRITE_SIZE is exact for
16 B/lane stores and float atomics. Every figure is a mean over the kernel's dispatches.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: defaultdict(float))  # kernel -> dispatch -> value
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = row.get("Kernel_Name", "?")
                acc[k][(f, row.get("Dispatch_Id"))] += float(row["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in acc.items()}


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].replace("pn2::", "")


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (None, 0))
        w, nw = write.get(k, (None, 0))
        out[short(k)] = {
            "dispatches": max(nf, nw),
            "fetch_bytes": None if f is None else f * 1024,
            "fetch_bytes_x2": None if f is None else 2 * f * 1024,
            "write_bytes": None if w is None else w * 1024,
        }
    json.dump({"unit": "bytes per launch (mean over dispatches)", "kernels": out}, sys.stdout,
              indent=1)
    print()


if __name__ == "__main__":
    main()
