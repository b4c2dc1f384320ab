#!/usr/bin/env python3
"""Micro-benchmark of the three_nn paths at FP4 size (B=16, n=8192 cloud points, m=1024 FPS
centres): brute-force scan, grid search (LDS-staged / global), with and without the unknown
grid ordering; FP4 whole as three launches vs pn2_fp_grid_fused. HIP events, median of 20."""
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
    from oracle import oracle as O
    dev = torch.device("cuda:0")
    B, n, m = 16, 8192, 1024
    x = pkg.synth.batch(range(B), n, "scannet")[0]
    t1 = torch.from_numpy(x).to(dev)
    _, k = pkg.tf_sampling.farthest_point_sample_and_gather(m, t1)
    L = pkg.lib()
    st = torch.cuda.current_stream().cuda_stream
    dist = torch.empty((B, n, 3), device=dev)
    idx = torch.empty((B, n, 3), dtype=torch.int32, device=dev)

    def timeit(fn, reps=20):
        ts = []
        for _ in range(3):
            fn()
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); fn(); b.record(); b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return statistics.median(ts)

    ug = pkg.grid.PointGrid(t1, 0.1)
    res = {}
    res["scan"] = timeit(lambda: L.pn2_three_nn(t1.data_ptr(), k.data_ptr(), B, n, m, dist.data_ptr(), idx.data_ptr(), st))
    ref = (dist.clone(), idx.clone())
    for edge in (0.0, 0.15, 0.2, 0.28, 0.4):
        kg = pkg.grid.PointGrid(k, edge)
        for name, u in (("rand", None), ("sorted", ug)):
            r = timeit(lambda: L.pn2_three_nn_grid(kg.buf.data_ptr(), None if u is None else u.buf.data_ptr(), t1.data_ptr(), B, n, m, dist.data_ptr(), idx.data_ptr(), st))
            assert torch.equal(idx, ref[1]) and torch.equal(dist, ref[0])
            res[f"grid edge={edge} {name}"] = r
    # FP4 whole: grid build + three_nn_grid + fp_apply (three launches) vs pn2_fp_grid_fused
    p2 = torch.rand((B, m, 128), device=dev)
    out = torch.empty((B, n, 128), device=dev)
    out2 = torch.empty((B, n, 128), device=dev)

    def three_launches():
        kg = pkg.grid.PointGrid(k, 0.0)
        L.pn2_three_nn_grid(kg.buf.data_ptr(), ug.buf.data_ptr(), t1.data_ptr(), B, n, m,
                            dist.data_ptr(), idx.data_ptr(), st)
        L.pn2_fp_apply(dist.data_ptr(), idx.data_ptr(), ug.buf.data_ptr(), None, 0,
                       p2.data_ptr(), 128, B, n, m, out.data_ptr(), st)
    res["fp4 three launches"] = timeit(three_launches)
    res["fp4 apply only"] = timeit(lambda: L.pn2_fp_apply(
        dist.data_ptr(), idx.data_ptr(), ug.buf.data_ptr(), None, 0, p2.data_ptr(), 128, B, n, m,
        out.data_ptr(), st))
    # the same rows in index order (sequential writes, scattered neighbour gathers)
    res["fp4 apply only (index order)"] = timeit(lambda: L.pn2_fp_apply(
        dist.data_ptr(), idx.data_ptr(), None, None, 0, p2.data_ptr(), 128, B, n, m,
        out.data_ptr(), st))
    # a copy of the FP4 output size (67 MB read + 67 MB written): the write-rate reference
    big = torch.empty((B, n, 128), device=dev)
    res["fp4-size copy (read+write 67 MB each)"] = timeit(lambda: L.pn2_copy_f4(
        out.data_ptr(), big.data_ptr(), B * n * 128 * 4, 256, st))
    res["fp4 grid fused"] = timeit(lambda: L.pn2_fp_grid_fused(
        None, k.data_ptr(), ug.buf.data_ptr(), None, 0, p2.data_ptr(), 128, B, n, m,
        out2.data_ptr(), None, None, st))
    res["fp4 grid fused +nn"] = timeit(lambda: L.pn2_fp_grid_fused(
        None, k.data_ptr(), ug.buf.data_ptr(), None, 0, p2.data_ptr(), 128, B, n, m,
        out2.data_ptr(), dist.data_ptr(), idx.data_ptr(), st))
    assert torch.equal(out, out2) and torch.equal(idx, ref[1])
    kg0 = pkg.grid.PointGrid(k, 0.0)
    out3 = torch.empty((B, n, 128), device=dev)
    res["fp4 grid fused known"] = timeit(lambda: L.pn2_fp_grid_fused_known(
        kg0.buf.data_ptr(), None, k.data_ptr(), ug.buf.data_ptr(), None, 0, p2.data_ptr(), 128,
        B, n, m, out3.data_ptr(), None, None, st))
    assert torch.equal(out, out3)
    # cfg3's FP4: points1 = rgb + normals (C1 = 9, rows of 137 floats: not 16-B aligned)
    p1 = torch.rand((B, n, 9), device=dev)
    o3 = torch.empty((B, n, 137), device=dev)
    o3b = torch.empty((B, n, 137), device=dev)
    res["cfg3 fp4 apply only"] = timeit(lambda: L.pn2_fp_apply(
        dist.data_ptr(), idx.data_ptr(), ug.buf.data_ptr(), p1.data_ptr(), 9, p2.data_ptr(), 128,
        B, n, m, o3.data_ptr(), st))
    res["cfg3 fp4 grid fused"] = timeit(lambda: L.pn2_fp_grid_fused(
        None, k.data_ptr(), ug.buf.data_ptr(), p1.data_ptr(), 9, p2.data_ptr(), 128, B, n, m,
        o3b.data_ptr(), None, None, st))
    assert torch.equal(o3, o3b)
    res["build known grid"] = timeit(lambda: pkg.grid.PointGrid(k, 0.0))
    res["build cloud grid"] = timeit(lambda: pkg.grid.PointGrid(t1, 0.1))
    # the build launches alone, into fixed buffers (no allocation between the events)
    gk = pkg.grid.PointGrid(k, 0.0)
    gc = pkg.grid.PointGrid(t1, 0.1)
    res["build known grid launch"] = timeit(lambda: L.pn2_grid_build(
        k.data_ptr(), B, m, 0.0, gk.buf.data_ptr(), gk.nbytes, st))
    res["build cloud grid launch"] = timeit(lambda: L.pn2_grid_build(
        t1.data_ptr(), B, n, 0.1, gc.buf.data_ptr(), gc.nbytes, st))
    x5 = torch.from_numpy(pkg.synth.batch(range(8), 16384, "scannet")[0]).to(dev)
    g5 = pkg.grid.PointGrid(x5, 0.1)
    res["build msg grid launch"] = timeit(lambda: L.pn2_grid_build(
        x5.data_ptr(), 8, 16384, 0.1, g5.buf.data_ptr(), g5.nbytes, st))
    print(json.dumps({k_: round(v, 1) for k_, v in res.items()}))


if __name__ == "__main__":
    main()
