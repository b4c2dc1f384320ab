#!/usr/bin/env python3
"""Micro-benchmark of the grid build and of cfg5's three SA1 grouped queries (B = 8 clouds of
16,384 points, 512 centres, r = 0.1 / 0.2 / 0.4, ns = 16 / 32 / 128): one grid per radius
(edge = radius) against ONE grid for all three radii (edge 0.1, 0.2, 0.4), and the three radii in one launch per grid; every variant's
idx / grouped_xyz must equal the per-radius one bit for bit. HIP events, median of 20."""
import importlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    pu, tg = pkg.pointnet_util, pkg.tf_grouping

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); fn(); b.record(); b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return statistics.median(ts)

    res = {}
    for name, B, N in (("cfg2", 16, 8192), ("cfg5", 8, 16384)):
        x = torch.from_numpy(pkg.synth.batch(range(B), N, "scannet")[0]).to(dev)
        res[f"build {name} edge 0.1 (us)"] = timeit(lambda: pkg.grid.PointGrid(x, 0.1))
    B, N, M = 8, 16384, 512
    radii, nss = (0.1, 0.2, 0.4), (16, 32, 128)
    x = torch.from_numpy(pkg.synth.batch(range(B), N, "scannet")[0]).to(dev)
    _, q = pkg.tf_sampling.farthest_point_sample_and_gather(M, x)
    grids = {r: tg.BallGrid(x, r) for r in radii}
    ref = [pu.ball_group_xyz(r, ns, x, q, grids[r]) for r, ns in zip(radii, nss)]
    for r, ns in zip(radii, nss):
        res[f"query r={r} own grid (us)"] = timeit(lambda: pu.ball_group_xyz(r, ns, x, q, grids[r]))
    for edge in (0.1, 0.2, 0.4):
        g = tg.BallGrid(x, edge)
        tot = 0.0
        for (r, ns), (ri, rc, rg) in zip(zip(radii, nss), ref):
            i, c, gx = pu.ball_group_xyz(r, ns, x, q, g)
            assert torch.equal(i, ri) and torch.equal(c, rc)
            assert torch.equal(gx.view(torch.int32), rg.view(torch.int32))
            t = timeit(lambda: pu.ball_group_xyz(r, ns, x, q, g))
            res[f"query r={r} on one grid edge {edge} (us)"] = t
            tot += t
        res[f"three queries on one grid edge {edge} (us)"] = tot
        # all three radii in ONE launch (pn2_ball_group_xyz_grid_radii), bit for bit
        outs = pu.ball_group_xyz_radii(radii, nss, x, q, g)
        for (i, c, gx), (ri, rc, rg) in zip(outs, ref):
            assert torch.equal(i, ri) and torch.equal(c, rc)
            assert torch.equal(gx.view(torch.int32), rg.view(torch.int32))
        res[f"three radii in one launch, grid edge {edge} (us)"] = timeit(
            lambda: pu.ball_group_xyz_radii(radii, nss, x, q, g))
    print(json.dumps({k: round(v, 1) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
