#!/usr/bin/env python3
"""Time FP4 alone (B = 16 ScanNet crops, n = 8192 <- m = 1024, C2 = 128, C1 = 0 and cfg3's
C1 = 6), HIP events, median of 20, no parity assertions (tests/test_gpu_parity.py holds those):
pn2_fp_grid_fused (each workgroup grids the known points itself) against
pn2_fp_grid_fused_known over the grid the SA1 sampler built, and the SA1 sampler launch with
and without that grid (pn2_fps_chain vs pn2_fps_chain_grid). Any build (PN2HIP_LIB=...)."""
import importlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    B, n, m = 16, 8192, 1024
    t1 = torch.from_numpy(pkg.synth.batch(range(B), n, "scannet")[0]).to(dev)
    _, k = pkg.tf_sampling.farthest_point_sample_and_gather(m, t1)
    ug = pkg.grid.PointGrid(t1, 0.1)
    L = pkg.lib()
    st = torch.cuda.current_stream().cuda_stream
    p2 = torch.rand((B, m, 128), device=dev)
    p1 = torch.rand((B, n, 6), device=dev)
    out = torch.empty((B, n, 128), device=dev)
    o3 = torch.empty((B, n, 134), device=dev)

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); fn(); b.record(); b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return statistics.median(ts)
    res = {"lib": os.path.basename(os.environ.get("PN2HIP_LIB") or "libpn2hip.so")}
    res["cfg2_fp4_us"] = timeit(lambda: L.pn2_fp_grid_fused(
        None, k.data_ptr(), ug.buf.data_ptr(), None, 0, p2.data_ptr(), 128, B, n, m,
        out.data_ptr(), None, None, st))
    res["cfg3_fp4_us"] = timeit(lambda: L.pn2_fp_grid_fused(
        None, k.data_ptr(), ug.buf.data_ptr(), p1.data_ptr(), 6, p2.data_ptr(), 128, B, n, m,
        o3.data_ptr(), None, None, st))
    idx = torch.empty((B, m), dtype=torch.int32, device=dev)
    nx = torch.empty((B, m, 3), device=dev)
    kg = pkg.grid.PointGrid(nx, build=False)
    pkg.tf_sampling.farthest_point_sample_chain([m], t1, out=[(idx, nx)], grid0=kg)
    assert torch.equal(nx, k)
    res["cfg2_fp4_known_us"] = timeit(lambda: L.pn2_fp_grid_fused_known(
        kg.buf.data_ptr(), None, k.data_ptr(), ug.buf.data_ptr(), None, 0, p2.data_ptr(), 128, B,
        n, m, out.data_ptr(), None, None, st))
    res["cfg3_fp4_known_us"] = timeit(lambda: L.pn2_fp_grid_fused_known(
        kg.buf.data_ptr(), None, k.data_ptr(), ug.buf.data_ptr(), p1.data_ptr(), 6, p2.data_ptr(),
        128, B, n, m, o3.data_ptr(), None, None, st))
    res["sa1_sampler_us"] = timeit(lambda: pkg.tf_sampling.farthest_point_sample_chain(
        [m], t1, out=[(idx, nx)]), reps=10)
    res["sa1_sampler_grid_us"] = timeit(lambda: pkg.tf_sampling.farthest_point_sample_chain(
        [m], t1, out=[(idx, nx)], grid0=kg), reps=10)
    print(json.dumps({k_: (round(v, 2) if isinstance(v, float) else v) for k_, v in res.items()}))


if __name__ == "__main__":
    main()
