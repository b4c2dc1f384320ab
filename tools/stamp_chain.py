#!/usr/bin/env python3
"""Diagnostic: the hot-set chain stages' rounds (csrc/fps.hip fps_hot_body) for cloud 0 of
B = 16 ScanNet crops, SA2..SA4 samplers (1024 -> 256 -> 64 -> 16), from the stamped build
(make -C .../csrc variant VFILE=fps VNAME=hst VFLAGS=-DPN2_HOT_STAMP=1; run with PN2HIP_LIB
pointing at it). Per stage: rounds, picks per round, tries, and the cycles of each round's
parts: select (block max -> the hot set fits), hot (the picks), cold lag (first cold wave's
end after the hot wave's), and the rest (round end -> next round's block max)."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    L = pkg.lib()
    L.pn2_hot_stamps.argtypes = [ctypes.c_void_p]
    B, N, npts = 16, 8192, [1024, 256, 64, 16]
    x = torch.from_numpy(pkg.synth.batch(range(B), N, "scannet")[0]).to(dev)
    ts = pkg.tf_sampling
    x1 = ts.farthest_point_sample_and_gather(npts[0], x)[1]
    for _ in range(3):
        ts.farthest_point_sample_chain(npts[1:], x1)
    torch.cuda.synchronize()
    buf = np.zeros(3 * 64 * 8, np.uint64)
    assert L.pn2_hot_stamps(buf.ctypes.data) == 0
    ev = buf.reshape(3, 64, 8).astype(np.int64)
    res = {}
    for si, name in enumerate(["1024", "256", "64"]):
        e = ev[si]
        t_start = e[63, 0]
        rounds = [r for r in range(63) if e[r, 0] > 0 and e[r, 0] >= t_start]
        if not rounds and e[63, 1] > t_start:
            res[name] = {"rounds": 0, "picks_end": int(e[63, 1] - t_start)}
            continue
        if not rounds:
            res[name] = {"rounds": 0}
            continue
        picks, prev_j = [], 1
        sel, hot, lag, rest = [], [], [], []
        for i, r in enumerate(rounds):
            picks.append(int(e[r, 3] - prev_j))
            prev_j = int(e[r, 3])
            sel.append(int(e[r, 1] - e[r, 0]))
            hot.append(int(e[r, 2] - e[r, 1]))
            lag.append(int(e[r, 5] - e[r, 2]))
            if i + 1 < len(rounds):
                rest.append(int(e[rounds[i + 1], 0] - max(e[r, 2], e[r, 5])))
        res[name] = {"rounds": len(rounds), "picks": picks,
                     "exact_phase": int(e[63, 2] - t_start) if e[63, 2] else None,
                     "picks_end": int(e[63, 1] - t_start),
                     "last_round_end": int(max(e[rounds[-1], 2], e[rounds[-1], 5]) - t_start),
                     "tries": [int(e[r, 4]) for r in rounds],
                     "first_round_at": int(e[rounds[0], 0] - t_start),
                     "select": sel, "hot": hot, "cold_lag": lag, "rest": rest,
                     "sum": {"select": sum(sel), "hot": sum(hot), "cold_lag": sum(lag),
                             "rest": sum(rest)},
                     "hot_cycles_per_pick": round(sum(hot) / max(1, sum(picks)), 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
