#!/usr/bin/env python3
"""Micro-benchmark of the fused SA grouping (pn2_group_concat, group_concat_kernel) at the
cfg3 SSG shapes (B = 16; layer inputs N x C -> M centres x 32 neighbours, [xyz, points]).
Random neighbour lists inside each cloud (the cost is the gather, not the ball query).
Launches captured in a hipGraph, HIP events around the replay, median of 15; GB/s over output
+ rows read once. Also cfg5's MSG SA2 radii. PN2HIP_LIB selects an A/B build."""
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
    L = pkg.lib()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(3)

    def timeit(fn, reps=15, inner=10):
        # `inner` launches captured in one hipGraph, HIP events around the replay
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            with torch.cuda.graph(gr, stream=cs):
                for _ in range(inner):
                    fn(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            gr.replay()
            b.record(); b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / inner)
        return statistics.median(ts)

    B, ns = 16, 32
    res = {}
    for name, N, C, M in (("sa1", 8192, 9, 1024), ("sa2", 1024, 64, 256), ("sa3", 256, 128, 64),
                          ("sa4", 64, 256, 16)):
        xyz = torch.rand((B, N, 3), generator=g).to(dev)
        pts = torch.rand((B, N, C), generator=g).to(dev)
        nx = torch.rand((B, M, 3), generator=g).to(dev)
        idx = torch.randint(0, N, (B, M, ns), generator=g, dtype=torch.int32).to(dev)
        out = torch.empty((B, M, ns, C + 3), device=dev)
        gx = torch.empty((B, M, ns, 3), device=dev)

        def run(stream=None):
            assert L.pn2_group_concat(xyz.data_ptr(), pts.data_ptr(), nx.data_ptr(),
                                      idx.data_ptr(), B, N, C, M, ns, 1, gx.data_ptr(),
                                      out.data_ptr(), stream or st) == 0
        us = timeit(run)
        nbytes = out.numel() * 4 + gx.numel() * 4 + idx.numel() * 4 + (xyz.numel() + pts.numel()) * 4
        res[name] = {"us": round(us, 1), "GBps": round(nbytes / us / 1e3, 0)}
    # cfg5's MSG SA2 radii (B = 8, [points, xyz] order, no grouped_xyz output)
    B = 8
    for name, ns in (("msg2_r0", 32), ("msg2_r1", 64), ("msg2_r2", 128)):
        N, C, M = 512, 320, 128
        xyz = torch.rand((B, N, 3), generator=g).to(dev)
        pts = torch.rand((B, N, C), generator=g).to(dev)
        nx = torch.rand((B, M, 3), generator=g).to(dev)
        idx = torch.randint(0, N, (B, M, ns), generator=g, dtype=torch.int32).to(dev)
        out = torch.empty((B, M, ns, C + 3), device=dev)

        def run(stream=None):
            assert L.pn2_group_concat(xyz.data_ptr(), pts.data_ptr(), nx.data_ptr(),
                                      idx.data_ptr(), B, N, C, M, ns, 3, None,
                                      out.data_ptr(), stream or st) == 0
        us = timeit(run)
        nbytes = out.numel() * 4 + idx.numel() * 4 + (xyz.numel() + pts.numel()) * 4
        res[name] = {"us": round(us, 1), "GBps": round(nbytes / us / 1e3, 0)}
    print(json.dumps({"lib": os.environ.get("PN2HIP_LIB", "default"), **res}), flush=True)


if __name__ == "__main__":
    main()
