#!/usr/bin/env python3
"""Time the SA1 sampler alone (B = 16 ScanNet crops, 8192 -> 1024, nothing else on the GPU):
the culled sampler as the pipelined step launches it (pn2_fps_chain_grid, one stage, gridding
its picks: fps_hotcull_grid_kernel) and without the grid (pn2_fps_gather: fps_hotcull_kernel).
`inner` launches captured in one hipGraph, HIP events around a replay, median of `reps`; the
grid form's outputs are checked equal to the plain form's (the parity tests pin both).

    [PN2HIP_LIB=<variant .so>] python tools/bench_sampler.py [--reps 15] [--inner 10]
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
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--inner", type=int, default=10)
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    ts = pkg.tf_sampling
    dev = torch.device("cuda:0")
    B, N, M = 16, 8192, 1024
    x = torch.from_numpy(pkg.synth.batch(range(B), N, "scannet")[0]).to(dev)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    out = [(torch.empty((B, M), dtype=torch.int32, device=dev),
            torch.empty((B, M, 3), dtype=torch.float32, device=dev))]
    kgrid = pkg.grid.PointGrid(out[0][1], 0.0, build=False)

    def timeit(fn):
        with torch.cuda.stream(st):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for _ in range(args.inner):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            t = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                g.replay()
                b.record(st)
                b.synchronize()
                t.append(a.elapsed_time(b) * 1e3 / args.inner)
        return statistics.median(t)

    res = {"lib": os.environ.get("PN2HIP_LIB") or "product",
           "grid_us": timeit(lambda: ts.farthest_point_sample_chain([M], x, out=out, grid0=kgrid)),
           "plain_us": timeit(lambda: ts.farthest_point_sample_and_gather(M, x))}
    ri, rx = ts.farthest_point_sample_and_gather(M, x)
    res["exact"] = bool(torch.equal(out[0][0], ri) and torch.equal(out[0][1], rx))
    print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in res.items()}))


if __name__ == "__main__":
    main()
