#!/usr/bin/env python3
"""Micro-benchmark of the multi-layer launches at the cfg2 step's shapes (B = 16 ScanNet crops):

  SA2..SA4  six launches (ball query + group_concat per layer) vs ONE pn2_ball_group_layers,
            and each layer alone through the fused kernel;
  FP3..FP1  three pn2_fp_fused launches vs ONE pn2_fp_fused_layers, and each layer alone.

`inner` repetitions captured in one hipGraph, HIP events around its replay, median of 15; us per repetition and GB/s
over the algorithmic output bytes.

    python tools/bench_layers.py [--config cfg2|cfg3] [--json out.json]
"""
import argparse
import importlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    S = pkg.stack
    dev = torch.device("cuda:0")
    inp = S.make_inputs(args.config, list(range(16)), dev)
    xyz = [inp["xyz"]]
    for npoint, _, _, _ in S.SSG_SA:
        xyz.append(pkg.tf_sampling.farthest_point_sample_and_gather(npoint, xyz[-1])[1])
    points = [inp["feats"]] + list(inp["sa_out"])
    fp_feat = [inp["sa_out"][3]] + list(inp["fp_out"])
    torch.cuda.synchronize()

    def timeit(fn, reps=15, inner=10):
        # `inner` calls captured into one hipGraph and replayed: GPU time only (the Python
        # wrappers cost more host time per call than these kernels take)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(inner):
                    fn()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / inner)
        return statistics.median(ts)

    PU = pkg.pointnet_util
    res = {}
    one = torch.zeros((1, 1, 3), device=dev)
    oi = torch.zeros((1, 1), dtype=torch.int32, device=dev)
    oo = torch.empty((1, 1, 3), device=dev)
    L = pkg.lib()
    res["one_block_kernel_us"] = timeit(lambda: L.pn2_gather_point(
        one.data_ptr(), oi.data_ptr(), 1, 1, 1, oo.data_ptr(), torch.cuda.current_stream().cuda_stream))
    sa = [(S.SSG_SA[i][1], S.SSG_SA[i][2], xyz[i], points[i], xyz[i + 1]) for i in (1, 2, 3)]

    def sa_sep():
        for r, ns, x, p, q in sa:
            idx, _ = pkg.tf_grouping.query_ball_point(r, ns, x, q)
            PU.group_concat(x, p, q, idx, want_grouped_xyz=False)
    out_b = sum(16 * q.shape[1] * ns * ((p.shape[2] if p is not None else 0) + 3) * 4
                for _, ns, _, p, q in sa)
    res["sa234_six_launches_us"] = timeit(sa_sep)
    res["sa234_fused_us"] = timeit(lambda: PU.ball_group_layers(sa))
    res["sa234_fused_GBps"] = out_b / res["sa234_fused_us"] / 1e3
    for i, spec in zip((2, 3, 4), sa):
        res[f"sa{i}_fused_alone_us"] = timeit(lambda spec=spec: PU.ball_group_layers([spec]))
    fp = [(xyz[i], xyz[i + 1], points[i], fp_feat[3 - i]) for i in (1, 2, 3)]
    out_f = sum(16 * x1.shape[1] * (p2.shape[2] + (p1.shape[2] if p1 is not None else 0)) * 4
                for x1, _, p1, p2 in fp)
    res["fp123_three_launches_us"] = timeit(lambda: [PU.fp_interpolate(*f) for f in fp])
    res["fp123_fused_us"] = timeit(lambda: PU.fp_interpolate_layers(fp))
    res["fp123_fused_GBps"] = out_f / res["fp123_fused_us"] / 1e3
    for k, f in zip((3, 2, 1), fp):
        res[f"fp{k}_alone_us"] = timeit(lambda f=f: PU.fp_interpolate(*f))
    res = {k: round(v, 2) for k, v in res.items()}
    print(json.dumps(res))
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(dict(res, config=args.config), fh, indent=1)


if __name__ == "__main__":
    main()
