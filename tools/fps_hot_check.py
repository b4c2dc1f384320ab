#!/usr/bin/env python3
"""GPU A/B of the SA1 samplers (pn2_fps_set_algo: 0 = culled hot set, 1 = v9 block scan,
6 = culled hot set with 128 hot entries; --msg: the MSG SA1 size, 8192 < N <= 16384, where 0 is
the culled sampler reading coordinates from L2 and 1 the v9 512 x 32 block scan):
index-exact against the oracle and against each other on tie-heavy and ScanNet-like clouds,
then HIP-event kernel times at the cfg2 SA1 shape (B = 16, 8192 -> 1024).

    python tools/fps_hot_check.py [--reps 20] [--quick]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--algo", type=int, default=0)
    ap.add_argument("--algos", default="1,0")
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
    ts = pkg.tf_sampling

    def run(algo, xt, M):
        old = lib.pn2_fps_set_algo(algo)
        try:
            i, nx = ts.farthest_point_sample_and_gather(M, xt)
            torch.cuda.synchronize()
        finally:
            lib.pn2_fps_set_algo(old)
        return i.cpu().numpy(), nx.cpu().numpy()

    cases = [("scannet", 16, 8192, 1024), ("uniform", 4, 8192, 1024), ("grid", 4, 8192, 1024),
             ("grid", 2, 8192, 4000), ("dup", 2, 5000, 40), ("fewuniq", 2, 8192, 600),
             ("scannet", 2, 4097, 4097), ("uniform", 2, 6000, 7000), ("scannet", 3, 8192, 2),
             ("scannet", 3, 8192, 1), ("scannet", 2, 7777, 1500)]
    if args.msg:
        cases = [("scannet", 8, 16384, 512), ("uniform", 2, 16384, 512), ("grid", 2, 16384, 1024),
                 ("grid", 1, 16384, 4000), ("dup", 1, 12000, 40), ("fewuniq", 2, 16384, 600),
                 ("scannet", 1, 8193, 8193), ("uniform", 1, 12000, 13000), ("scannet", 2, 16384, 1),
                 ("scannet", 2, 11111, 2000)]
    if args.quick:
        cases = cases[:3]
    if args.no_check:
        cases = []
    ok = True
    for kind, B, N, M in cases:
        x = cloud(pkg, kind, B, N)
        xt = torch.from_numpy(x).to(dev)
        i2, n2 = run(args.algo, xt, M)
        i1, n1 = run(1, xt, M)
        ref = O.fps(x, M)
        e2 = int((i2 != ref).sum())
        e1 = int((i1 != ref).sum())
        nxe = int((n2.view(np.int32) != O.gather_point(x, ref).view(np.int32)).sum())
        good = e2 == 0 and e1 == 0 and nxe == 0
        ok &= good
        first = int(np.argmax((i2 != ref).any(0))) if e2 else -1
        print(json.dumps({"case": [kind, B, N, M], "hot_idx_diff": e2, "v9_idx_diff": e1,
                          "hot_new_xyz_diff": nxe, "first_bad_j": first, "ok": good}), flush=True)
    # timing at the given shape (default: the cfg2 SA1 shape)
    TB, TN, TM = (int(v) for v in args.shape.split(","))
    x = cloud(pkg, "scannet", TB, TN)
    xt = torch.from_numpy(x).to(dev)
    idx = torch.empty((TB, TM), dtype=torch.int32, device=dev)
    nx = torch.empty((TB, TM, 3), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream()
    algos = [int(a) for a in args.algos.split(",")]
    times = {a: [] for a in algos}
    for r in range(args.reps + 2):
        for algo in algos:
            old = lib.pn2_fps_set_algo(algo)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            rc = lib.pn2_fps_gather(ctypes.c_void_p(xt.data_ptr()), TB, TN, TM,
                                    ctypes.c_void_p(idx.data_ptr()), ctypes.c_void_p(nx.data_ptr()),
                                    ctypes.c_void_p(s.cuda_stream))
            e1.record(s)
            torch.cuda.synchronize()
            lib.pn2_fps_set_algo(old)
            assert rc == 0
            if r >= 2:
                times[algo].append(e0.elapsed_time(e1))
    out = {"shape": [TB, TN, TM],
           "ms": {{0: "default", 1: "v9", 6: "cull_k128", }.get(a, str(a)): {"median": statistics.median(v),
                                                          "min": min(v)} for a, v in times.items()},
           "all_exact": ok}
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
