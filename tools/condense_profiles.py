#!/usr/bin/env python3
"""Condense an A/B sweep directory under profiles/: every bench.py JSON line in it (recursively)
becomes one row of <dir>/summary.jsonl (file name, value, ms_per_step, the SA1 sampler's launch
time, the layout fields of `config`, e2e value), and the raw .json / .err files are removed.
Other files (logs, csv) stay.

    python tools/condense_profiles.py profiles/r3/plan profiles/r3/layouts ...
"""
import json
import os
import sys

KEEP_CFG = ("config", "clouds_per_gpu", "hw_queues", "streams", "launch",
            "lane0_priority")


def condense(d):
    rows, drop = [], []
    for root, _, files in os.walk(d):
        for f in sorted(files):
            p = os.path.join(root, f)
            if f.endswith(".err"):
                drop.append(p)
                continue
            if not f.endswith(".json") or f == "summary.jsonl":
                continue
            try:
                with open(p) as fh:
                    txt = fh.read().strip().splitlines()
                obj = json.loads([ln for ln in txt if ln.startswith("{")][-1])
            except (ValueError, IndexError):
                continue
            if "value" not in obj:
                continue
            cfg = obj.get("config") or {}
            rows.append({"file": os.path.relpath(p, d), "value": obj.get("value"),
                         "ms_per_step": obj.get("ms_per_step"), "steps": obj.get("steps"),
                         "sa1_ms": (obj.get("roofline") or {}).get("avg_launch_ms"),
                         "e2e": (obj.get("e2e") or {}).get("value"),
                         "diagnostic": obj.get("diagnostic"),
                         "config": {k: cfg[k] for k in KEEP_CFG if k in cfg}})
            drop.append(p)
    if not rows:
        return 0
    with open(os.path.join(d, "summary.jsonl"), "a") as fh:
        for r in rows:
            fh.write(json.dumps(r) + "\n")
    for p in drop:
        os.remove(p)
    for root, dirs, files in os.walk(d, topdown=False):
        if root != d and not os.listdir(root):
            os.rmdir(root)
    return len(rows)


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(d, condense(d))
