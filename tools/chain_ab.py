#!/usr/bin/env python3
"""A/B of the fused SSG sampler chain's tail (pn2_fps_chain on the SA1 output: 1024 -> 256 ->
64 -> 16, what the step's lane-4 task runs) for alternative builds of libpn2hip.so (--lib
NAME=PATH), index-exact against the product build, HIP events, B = 16 ScanNet crops."""
import argparse, ctypes, importlib, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    B = 16
    x = torch.from_numpy(pkg.synth.batch(range(B), 8192, "scannet")[0]).to(dev)
    _, x1 = pkg.tf_sampling.farthest_point_sample_and_gather(1024, x)
    libs = {"product": pkg._lib.lib()}
    for spec in args.lib:
        n, pth = spec.split("=", 1)
        h = ctypes.CDLL(os.path.abspath(pth))
        h.pn2_fps_chain.restype, h.pn2_fps_chain.argtypes = pkg._lib.SIGNATURES["pn2_fps_chain"]
        libs[n] = h
    npts = [256, 64, 16]
    outs = {}
    st = torch.cuda.current_stream()

    def run(h):
        idx = [torch.empty((B, m), dtype=torch.int32, device=dev) for m in npts]
        nx = [torch.empty((B, m, 3), dtype=torch.float32, device=dev) for m in npts]
        ia = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in idx])
        na = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in nx])
        pa = (ctypes.c_int * 3)(*npts)
        def f():
            assert h.pn2_fps_chain(x1.data_ptr(), B, 1024, 3, pa, ia, na, st.cuda_stream) == 0
        return f, idx
    fns = {n: run(h) for n, h in libs.items()}
    for n, (f, idx) in fns.items():
        f()
        torch.cuda.synchronize()
        outs[n] = [t.cpu() for t in idx]
    exact = all(all(torch.equal(a, b) for a, b in zip(outs[n], outs["product"])) for n in outs)
    times = {n: [] for n in fns}
    for r in range(args.reps + 3):
        for n, (f, _) in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            b.synchronize()
            if r >= 3:
                times[n].append(a.elapsed_time(b) * 1e3)
    print(json.dumps({"us": {n: round(statistics.median(v), 1) for n, v in times.items()},
                      "exact_vs_product": exact}))
    return 0 if exact else 1


if __name__ == "__main__":
    sys.exit(main())
