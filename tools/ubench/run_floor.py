#!/usr/bin/env python3
"""Latency floors of the culled sampler (tools/ubench/pick_floor.hip), alone on one CU:
cycles per pick of the dependent chain (var 0) and of the kernel's full pick step (var 1,
+ publish), cycles per round of the round end's synchronisation skeleton (16 waves, three
barriers and the two cross-wave reductions). Writes JSON (bench.py's roofline.latency reads
it):

    python tools/ubench/run_floor.py [--out profiles/r3/sampler_floor.json]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    args = ap.parse_args()
    import importlib
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "libfloor.so"))
    P = ctypes.c_void_p
    dev = torch.device("cuda:0")
    xyz = torch.from_numpy(pkg.synth.batch([0], 8192, "uniform")[0]).to(dev)
    out = torch.zeros(1024, dtype=torch.int32, device=dev)
    cyc = torch.zeros(1, dtype=torch.int64, device=dev)
    res = {}
    reps, picks = 50, 128
    for var, name in ((0, "pick_chain"), (1, "pick_step")):
        vals = []
        for _ in range(7):
            assert L.pn2_pick_floor(P(xyz.data_ptr()), var, reps, picks, P(out.data_ptr()),
                                    P(cyc.data_ptr())) == 0
            vals.append(cyc.item() / (reps * picks))
        res[name + "_cycles"] = round(statistics.median(vals[2:]), 1)
    vals = []
    rounds = 2000
    for _ in range(7):
        assert L.pn2_round_floor(rounds, P(out.data_ptr()), P(cyc.data_ptr())) == 0
        vals.append(cyc.item() / rounds)
    res["round_sync_cycles"] = round(statistics.median(vals[2:]), 1)
    res["note"] = ("s_memtime cycles, one workgroup alone on the GPU: pick_chain = the dependent "
                   "chain of one pick (lane best of 4, 64-lane max, winner lane, coordinates, "
                   "update), pick_step = + the publish (the kernel's pick step), "
                   "round_sync = 3 barriers + the 2 cross-wave reductions of a round end, 16 waves")
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
