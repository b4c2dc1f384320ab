#!/usr/bin/env python3
"""Print the kernel timeline of one step from a rocprofv3 --kernel-trace CSV of bench.py:
the last occurrence of the SA1 sampler marks a step; kernels are listed from its start to
the start of the next step, with start/end offsets in us and the queue they ran on."""
import csv
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").replace("pn2::", "").split("(")[0][:60]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "fps_v" in r["Kernel_Name"]
          and r.get("Grid_Size_X") in ("4096", "8192", "16384")]
if not starts:
    starts = [i for i, r in enumerate(rows) if "fps_chain" in r["Kernel_Name"]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -3
i0 = starts[which]
i1 = starts[which + 1] if which + 1 < len(starts) else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0 - 2:i1]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q{r.get('Queue_Id', '?'):>2}  {short(r['Kernel_Name'])} [{r.get('Grid_Size_X')}x{r.get('Grid_Size_Y')}]")

ch = [rows[i] for i in starts]
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(ch, ch[1:])]
durs = [(int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3 for a in ch]
if gaps:
    gs = sorted(gaps)
    print(f"sampler launches {len(ch)}: mean {sum(durs) / len(durs):.1f} us; gap between "
          f"consecutive launches median {gs[len(gs) // 2]:.1f} us (min {gs[0]:.1f}, max {gs[-1]:.1f})")
