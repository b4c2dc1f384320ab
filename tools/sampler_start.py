#!/usr/bin/env python3
"""Why does a pipelined step's SA1 sampler start late? Attribution from one rocprofv3 run with
--kernel-trace and --hip-runtime-trace (CSV; both tables carry Correlation_Id, and their
timestamps share one clock).

    python tools/sampler_start.py <dir with *kernel_trace.csv and *hip_api_trace.csv> [--skip 20]

For every SA1 sampler launch (fps_hotcull / fps_v9 kernels; BASELINE cfg2's 8192 -> 1024):
  pred_end   end of the previous kernel on the same hardware queue (Queue_Id)
  api_end    end of the host API call that enqueued it (matched by Correlation_Id)
  delay      start - pred_end  (what lanes_cfg2.txt calls the sampler's start delay)
  host       max(0, api_end - pred_end): the queue was empty because the host had not yet
             enqueued the launch
  dispatch   start - max(pred_end, api_end): enqueued and its queue free, but its workgroups
             not yet running (the CP had not processed the packet or no CU was free: a sampler
             workgroup needs a whole CU -- 16 waves x 128 VGPRs, ~150 KB of LDS)
Also the host side: per HIP API function, calls and mean microseconds per step, so the host's
enqueue cost per step is visible beside the GPU step time."""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict

SAMPLER = ("fps_hotcull", "fps_v9")


def find(d, suffix):
    f = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not f:
        raise SystemExit(f"no *{suffix} under {d}")
    return f[0]


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=20, help="sampler launches skipped (warm-up)")
    a = ap.parse_args()
    kr = list(csv.DictReader(open(find(a.dir, "kernel_trace.csv"))))
    ar = list(csv.DictReader(open(find(a.dir, "hip_api_trace.csv"))))
    api = {r["Correlation_Id"]: r for r in ar}
    byq = defaultdict(list)
    for r in kr:
        byq[r.get("Queue_Id", "?")].append(r)
    for q in byq:
        byq[q].sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = []
    for q, lst in byq.items():
        for prev, r in zip(lst, lst[1:]):
            if not any(s in r["Kernel_Name"] for s in SAMPLER):
                continue
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            pe = int(prev["End_Timestamp"])
            c = api.get(r["Correlation_Id"])
            ae = int(c["End_Timestamp"]) if c else None
            rows.append({"q": q, "s": s, "e": e, "pred_end": pe, "api_end": ae,
                         "pred": prev["Kernel_Name"][:40]})
    rows.sort(key=lambda x: x["s"])
    rows = rows[a.skip:]
    if not rows:
        raise SystemExit("no sampler launches after the skip")
    us = lambda ns: ns / 1e3  # noqa: E731
    delay = [us(r["s"] - r["pred_end"]) for r in rows]
    host = [us(max(0, r["api_end"] - r["pred_end"])) for r in rows if r["api_end"] is not None]
    disp = [us(r["s"] - max(r["pred_end"], r["api_end"])) for r in rows if r["api_end"] is not None]
    dur = [us(r["e"] - r["s"]) for r in rows]
    ahead = [us(r["pred_end"] - r["api_end"]) for r in rows if r["api_end"] is not None]
    print(f"{len(rows)} SA1 sampler launches (after {a.skip} skipped), "
          f"{len(set(r['q'] for r in rows))} sampler queues")
    for name, v in (("start delay after the queue predecessor's end", delay),
                    ("  of which: not yet enqueued by the host", host),
                    ("  of which: enqueued, queue free, not yet running (dispatch)", disp),
                    ("host enqueue ahead of the predecessor's end (negative: late)", ahead),
                    ("sampler kernel duration", dur)):
        print(f"{name:64s} median {statistics.median(v):8.1f} us  p10 {pct(v, .1):8.1f}  "
              f"p90 {pct(v, .9):8.1f}")
    span = (rows[-1]["s"] - rows[0]["s"]) / max(1, len(rows) - 1)
    print(f"sampler start to next sampler start (any queue): {us(span):.1f} us")
    # host API cost per step (one SA1 sampler per step)
    t0, t1 = rows[0]["s"], rows[-1]["s"]
    steps = len(rows) - 1
    fn = defaultdict(lambda: [0, 0])
    for r in ar:
        s = int(r["Start_Timestamp"])
        if t0 <= s < t1:
            f = fn[r["Function"]]
            f[0] += 1
            f[1] += int(r["End_Timestamp"]) - s
    tot = sum(v[1] for v in fn.values())
    print(f"host HIP API time per step: {us(tot) / steps:.1f} us over {steps} steps "
          f"(the runtime trace itself adds to each call)")
    for k, (n, t) in sorted(fn.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {k:32s} {n / steps:6.2f} calls/step  {us(t) / max(1, n):7.2f} us/call  "
              f"{us(t) / steps:7.1f} us/step")


if __name__ == "__main__":
    main()
