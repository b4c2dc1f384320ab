#!/usr/bin/env python3
"""Report of tools/bench_gaps.py's trace: gap (us) from each FPS launch's end to the next
gather's start, by case (gather grid size)."""
import csv
import statistics
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = {256: "same", 512: "event", 768: "waitidle", 1024: "cross", 1280: "graph"}
gaps = defaultdict(list)
last_fps_end = None
for r in rows:
    if "fps_v" in r["Kernel_Name"]:
        last_fps_end = int(r["End_Timestamp"])
    elif "gather_point_kernel" in r["Kernel_Name"] and last_fps_end is not None:
        g = int(r["Grid_Size_X"])
        gaps[names.get(g, g)].append((int(r["Start_Timestamp"]) - last_fps_end) / 1e3)
        last_fps_end = None
for k, v in gaps.items():
    print(f"{k:10s} n={len(v)} median gap {statistics.median(v):7.2f} us  min {min(v):7.2f}  max {max(v):7.2f}")
