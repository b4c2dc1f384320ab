#!/usr/bin/env python3
"""Condense an A/B sweep directory under profiles/: every bench.py JSON line in it (recursively)
becomes one row of <dir>/summary.jsonl (file name, value, ms_per_step, the SA1 sampler's launch
time, the layout fields of `config`, e2e value); every other JSON object (tools/bench_*.py
results) one row {"file", "data"} of <dir>/tools.jsonl; the raw .json / .err files are
removed. Other files (logs, csv, txt) stay.

    python tools/condense_profiles.py profiles/r3/plan profiles/r3/layouts ...
"""
import json
import os
import sys

KEEP_CFG = ("config", "clouds_per_gpu", "hw_queues", "streams", "launch",
            "lane0_priority")


def condense(d):
    rows, other, drop = [], [], []
    for root, _, files in os.walk(d):
        for f in sorted(files):
            p = os.path.join(root, f)
            if f.endswith(".err"):
                drop.append(p)
                continue
            if not f.endswith(".json"):
                continue
            try:
                with open(p) as fh:
                    raw = fh.read().strip()
                try:
                    obj = json.loads(raw)  # (an indented tool result)
                except ValueError:
                    obj = json.loads([ln for ln in raw.splitlines() if ln.startswith("{")][-1])
            except (ValueError, IndexError):
                continue
            if not isinstance(obj, dict) or "value" not in obj or "metric" not in obj:
                other.append({"file": os.path.relpath(p, d), "data": obj})
                drop.append(p)
                continue
            cfg = obj.get("config") or {}
            rows.append({"file": os.path.relpath(p, d), "value": obj.get("value"),
                         "ms_per_step": obj.get("ms_per_step"), "steps": obj.get("steps"),
                         "sa1_ms": (obj.get("roofline") or {}).get("avg_launch_ms"),
                         "e2e": (obj.get("e2e") or {}).get("value"),
                         "diagnostic": obj.get("diagnostic"),
                         "config": {k: cfg[k] for k in KEEP_CFG if k in cfg}})
            drop.append(p)
    if not rows and not other:
        return 0
    for name, lst in (("summary.jsonl", rows), ("tools.jsonl", other)):
        if lst:
            with open(os.path.join(d, name), "a") as fh:
                for r in lst:
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
