#!/usr/bin/env python3
"""GPU A/B of the large-cloud samplers, per call (pn2_fps_gather_sched):
  0 = the default (culled hot set), 1 = v9 block scan, 6 = culled hot set with 128 entries
  (--msg: the MSG SA1 size, 8192 < N <= 16384, where 0 is the culled sampler reading
  coordinates from L2 and 1 the v9 512 x 32 block scan),
and alternative builds of the library (--lib NAME=PATH, e.g. a lab variant of fps_cull.h built
by `make -C pointcloud-segmentation-attention_amd/csrc variant`), timed with its default
schedule in the same process, interleaved with the others:
index-exact against the oracle on tie-heavy and ScanNet-like clouds, then HIP-event kernel
times at the cfg2 SA1 shape (B = 16, 8192 -> 1024).

    python tools/fps_hot_check.py [--reps 20] [--quick] [--lib new=path/libpn2hip.so]
"""
import argparse
import ctypes
import importlib
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def cloud(pkg, kind, B, N, seed=0):
    if kind in ("scannet", "uniform"):
        return pkg.synth.batch(range(seed, seed + B), N, kind)[0]
    if kind == "dup":
        return np.tile(np.array([[0.25, 0.5, 0.75]], np.float32), (B, N, 1))
    if kind == "grid":
        g = np.stack(np.meshgrid(*[np.arange(16)] * 3, indexing="ij"), -1).reshape(-1, 3)
        rng = np.random.default_rng(seed)
        return np.stack([g[rng.integers(0, len(g), N)] for _ in range(B)]).astype(np.float32)
    if kind == "fewuniq":  # 300 distinct points drawn with replacement: M > #unique
        rng = np.random.default_rng(seed)
        u = rng.random((300, 3)).astype(np.float32)
        return np.stack([u[rng.integers(0, 300, N)] for _ in range(B)])
    raise ValueError(kind)


SSG_CASES = [("scannet", 16, 8192, 1024), ("uniform", 4, 8192, 1024), ("grid", 4, 8192, 1024),
             ("grid", 2, 8192, 4000), ("dup", 2, 5000, 40), ("fewuniq", 2, 8192, 600),
             ("scannet", 2, 4097, 4097), ("uniform", 2, 6000, 7000), ("scannet", 3, 8192, 2),
             ("scannet", 3, 8192, 1), ("scannet", 2, 7777, 1500)]
MSG_CASES = [("scannet", 8, 16384, 512), ("uniform", 2, 16384, 512), ("grid", 2, 16384, 1024),
             ("grid", 1, 16384, 4000), ("dup", 1, 12000, 40), ("fewuniq", 2, 16384, 600),
             ("scannet", 1, 8193, 8193), ("uniform", 1, 12000, 13000), ("scannet", 2, 16384, 1),
             ("scannet", 2, 11111, 2000)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--algos", default="1,0", help="schedules of the product library to time")
    ap.add_argument("--lib", action="append", default=[],
                    help="NAME=PATH: another build of libpn2hip.so, checked and timed too")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--shape", default="16,8192,1024", help="B,N,M of the timed launch")
    ap.add_argument("--msg", action="store_true",
                    help="check the MSG SA1 size (8192 < N <= 16384) instead of the SA1 cases")
    args = ap.parse_args()
    import torch
    from conftest import PKG_NAME
    from oracle import oracle as O
    O.set_threads(16)
    pkg = importlib.import_module(PKG_NAME)
    lib = pkg._lib.lib()
    dev = torch.device("cuda:0")
    P = ctypes.c_void_p
    sig = pkg._lib.SIGNATURES["pn2_fps_gather_sched"]
    libs = {}
    for spec in args.lib:
        name, path = spec.split("=", 1)
        h = ctypes.CDLL(os.path.abspath(path))
        h.pn2_fps_gather_sched.restype, h.pn2_fps_gather_sched.argtypes = sig
        libs[name] = h
    # variants: (label, library handle, schedule)
    names = {0: "default", 1: "v9", 6: "cull_k128"}
    variants = [(names.get(a, str(a)), lib, a) for a in (int(v) for v in args.algos.split(","))]
    variants += [(n, h, 0) for n, h in libs.items()]

    def launch(h, sched, xt, idx, nx, B, N, M, s):
        rc = h.pn2_fps_gather_sched(P(xt.data_ptr()), B, N, M, P(idx.data_ptr()),
                                    P(nx.data_ptr()), sched, P(s.cuda_stream))
        assert rc == 0, rc

    cases = MSG_CASES if args.msg else SSG_CASES
    if args.quick:
        cases = cases[:3]
    if args.no_check:
        cases = []
    ok = True
    s = torch.cuda.current_stream()
    for kind, B, N, M in cases:
        x = cloud(pkg, kind, B, N)
        xt = torch.from_numpy(x).to(dev)
        ref = O.fps(x, M)
        rnx = O.gather_point(x, ref).view(np.int32)
        row = {"case": [kind, B, N, M]}
        for label, h, sched in variants:
            idx = torch.empty((B, M), dtype=torch.int32, device=dev)
            nx = torch.empty((B, M, 3), dtype=torch.float32, device=dev)
            launch(h, sched, xt, idx, nx, B, N, M, s)
            torch.cuda.synchronize()
            i, n = idx.cpu().numpy(), nx.cpu().numpy()
            e = int((i != ref).sum()) + int((n.view(np.int32) != rnx).sum())
            row[label] = e
            ok &= e == 0
        print(json.dumps(row), flush=True)
    # timing at the given shape (default: the cfg2 SA1 shape), variants interleaved
    TB, TN, TM = (int(v) for v in args.shape.split(","))
    x = cloud(pkg, "scannet", TB, TN)
    xt = torch.from_numpy(x).to(dev)
    idx = torch.empty((TB, TM), dtype=torch.int32, device=dev)
    nx = torch.empty((TB, TM, 3), dtype=torch.float32, device=dev)
    times = {v[0]: [] for v in variants}
    for r in range(args.reps + 2):
        for label, h, sched in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            launch(h, sched, xt, idx, nx, TB, TN, TM, s)
            e1.record(s)
            torch.cuda.synchronize()
            if r >= 2:
                times[label].append(e0.elapsed_time(e1))
    out = {"shape": [TB, TN, TM],
           "ms": {k: {"median": statistics.median(v), "min": min(v)} for k, v in times.items()},
           "all_exact": ok}
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
