#!/usr/bin/env python3
"""Why the SA1 samplers of a pipelined run do not start back to back, from a rocprofv3
--kernel-trace CSV of bench.py.

    python tools/sampler_gaps.py <kernel_trace.csv> [--skip 30]

Per sampler queue: the gap between a sampler's end and the next sampler's start on the same
queue; how many samplers run at once; and which kernels were running in the 3 us before each
sampler started (the sampler workgroup needs a whole CU -- 16 waves x 128 VGPRs fill every
SIMD's register file, 155 KB of LDS -- so it cannot start beside any side-lane workgroup)."""
import argparse
import bisect
import collections
import csv
import statistics


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").replace("pn2::", "") \
        .split("(")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=int, default=30)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    samp = [r for r in rows if "fps_hotcull" in r["Kernel_Name"]]
    byq = collections.defaultdict(list)
    for r in samp:
        byq[r["Queue_Id"]].append(r)
    gaps = []
    for q, lst in byq.items():
        for x, y in zip(lst, lst[1:]):
            gaps.append((int(x["End_Timestamp"]), int(y["Start_Timestamp"])))
    gaps = sorted(gaps)[a.skip:]
    g = [(e - s) / 1e3 for s, e in gaps]
    print(f"{len(samp)} sampler launches on {len(byq)} queues; gap to the next sampler on the "
          f"same queue: median {statistics.median(g):.1f} us (min {min(g):.1f}, max {max(g):.1f})")
    conc = collections.Counter()
    for r in samp[a.skip:]:
        s = int(r["Start_Timestamp"])
        conc[sum(1 for x in samp if int(x["Start_Timestamp"]) <= s < int(x["End_Timestamp"]))] += 1
    print("samplers running when a sampler starts (itself included):", dict(sorted(conc.items())))
    ends = collections.Counter()
    starts = [int(r["Start_Timestamp"]) for r in samp[a.skip:]]
    for s in starts:
        for r in rows:
            rs, re_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if rs < s and s - 3000 <= re_ <= s and "fps_hotcull" not in r["Kernel_Name"]:
                ends[short(r["Kernel_Name"])] += 1
    print(f"kernels that ENDED within 3 us before a sampler started ({len(starts)} starts):")
    for k, v in ends.most_common(8):
        print(f"  {v:4d}  {k}")


if __name__ == "__main__":
    main()
