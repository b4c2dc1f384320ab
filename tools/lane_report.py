#!/usr/bin/env python3
"""Per-queue occupancy of a pipelined bench run, from a rocprofv3 --kernel-trace CSV.

    python tools/lane_report.py <kernel_trace.csv> [steps]

The window is the last `steps` SA1 sampler launches (default: all but the first quarter).
For every hardware queue: busy time (union of its kernels' intervals) per step, the sum of
kernel durations per step, and the kernels that take the most of it. The queue whose busy
time per step is closest to the measured step time is the one that sets the step."""
import csv
import sys
from collections import defaultdict


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").replace("pn2::", "") \
        .split("(")[0][:56]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
sa1 = [r for r in rows if r["Kernel_Name"].find("fps_hotcull") >= 0
       or (r["Kernel_Name"].find("fps_v9") >= 0 and r.get("Grid_Size_X") in ("4096", "8192", "16384"))]
if not sa1:
    sys.exit("no SA1 sampler launches in the trace")
steps = int(sys.argv[2]) if len(sys.argv) > 2 else max(1, len(sa1) - len(sa1) // 4 - 1)
win = sa1[-steps - 1:]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["Start_Timestamp"])
nsteps = len(win) - 1
per_q = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e <= t0 or s >= t1:
        continue
    per_q[r.get("Queue_Id", "?")].append((max(s, t0), min(e, t1), r["Kernel_Name"]))
span = (t1 - t0) / 1e3
print(f"window: {nsteps} steps, {span:.1f} us, {span / nsteps:.1f} us per step (SA1 start to SA1 start)")
for q in sorted(per_q, key=lambda q: int(q) if q.isdigit() else 99):
    iv = sorted(per_q[q])
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    by = defaultdict(float)
    for s, e, n in iv:
        by[short(n)] += (e - s) / 1e3
    tot = sum(by.values())
    print(f"q{q:>2}: busy {busy / 1e3 / nsteps:7.1f} us/step ({busy / (t1 - t0):5.1%}), kernel sum "
          f"{tot / nsteps:7.1f} us/step, {len(iv) / nsteps:.1f} launches/step")
    for n, v in sorted(by.items(), key=lambda x: -x[1])[:8]:
        print(f"       {v / nsteps:7.1f}  {n}")
