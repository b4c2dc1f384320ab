#!/usr/bin/env python3
"""Micro-benchmark of the fused FP interpolation + concat (pn2_fp_apply, fp_fused_kernel) at
the FP4 sizes of cfg2 (C1 = 0) and cfg3 (C1 = 9 channels, scalar path) and an FP2-like size,
with and without the unknown-grid row order. HIP events, median of 20; GB/s over the
algorithmic bytes (output + points1 + dist/idx + points2 once).

    python tools/bench_fp.py
"""
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
    g = torch.Generator(device="cpu").manual_seed(7)

    def timeit(fn, reps=20, inner=20):
        # `inner` launches between the events: one launch alone would time the host's
        # launch latency (the GPU idles between the first event and the kernel)
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(inner):
                fn()
            b.record(); b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / inner)
        return statistics.median(ts)

    res = {}
    B = 16
    for name, n, m, C1, C2 in (("fp4_cfg2", 8192, 1024, 0, 128), ("fp4_cfg3", 8192, 1024, 9, 128),
                               ("fp2", 1024, 256, 128, 256)):
        x = pkg.synth.batch(range(B), n, "scannet")[0]
        t1 = torch.from_numpy(x).to(dev)
        _, k = pkg.tf_sampling.farthest_point_sample_and_gather(m, t1)
        dist = torch.empty((B, n, 3), device=dev)
        idx = torch.empty((B, n, 3), dtype=torch.int32, device=dev)
        assert L.pn2_three_nn(t1.data_ptr(), k.data_ptr(), B, n, m, dist.data_ptr(),
                              idx.data_ptr(), st) == 0
        p1 = torch.rand((B, n, C1), generator=g).to(dev) if C1 else None
        p2 = torch.rand((B, m, C2), generator=g).to(dev)
        out = torch.empty((B, n, C1 + C2), device=dev)
        nbytes = out.numel() * 4 + (p1.numel() * 4 if C1 else 0) + B * n * 24 + p2.numel() * 4
        ug = pkg.grid.PointGrid(t1, 0.1)
        for order, u in (("rows", None), ("grid", ug)):
            def run():
                assert L.pn2_fp_apply(dist.data_ptr(), idx.data_ptr(),
                                      None if u is None else u.buf.data_ptr(),
                                      p1.data_ptr() if C1 else None, C1, p2.data_ptr(), C2, B,
                                      n, m, out.data_ptr(), st) == 0
            us = timeit(run)
            res[f"{name} {order}"] = {"us": round(us, 1), "GBps": round(nbytes / us / 1e3, 0)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
