#!/usr/bin/env python3
"""Sweep the FPS launch table on the GPU: every (variant, block, points-per-thread) of
pn2_fps_tune (tools/fps_lab/libpn2fpslab.so: v2 and v9 with G = 1/2/4) for the SA layer sizes, interleaved rounds in ONE process (methodology rule 24),
each result checked index-exact against the production entry point. Prints one JSON line per
(N, config) with the median and min kernel time (HIP events, B clouds per launch)."""
import ctypes
import importlib
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


LAB_SO = os.path.join(ROOT, "tools", "fps_lab", "libpn2fpslab.so")
V2 = [(64, 1), (64, 2), (64, 4), (64, 8), (64, 16), (128, 4), (128, 8), (128, 16), (256, 1),
      (256, 2), (256, 4), (256, 8), (256, 16), (512, 2), (512, 4), (512, 8), (512, 16),
      (1024, 1), (1024, 2), (1024, 4), (1024, 8), (1024, 16)]
V9 = [(bl, pp, g) for bl, pp in [(64, 4), (64, 8), (128, 4), (128, 8), (256, 4), (256, 8),
                                 (256, 16), (512, 4), (512, 8), (512, 16), (256, 32)]
      for g in (1, 2, 4)] + [(64, 1, 1), (64, 2, 1), (64, 2, 2), (128, 2, 2), (256, 2, 2),
                             (512, 32, 4), (256, 64, 4), (128, 16, 4), (128, 1, 1),
                             (64, 16, 4), (64, 32, 4), (128, 32, 4)]


V11 = [(64, 1, 1), (64, 2, 2), (64, 4, 4), (64, 8, 4), (256, 4, 4), (256, 8, 4), (256, 16, 4),
       (256, 32, 4), (512, 16, 4), (512, 32, 4), (128, 8, 4), (64, 16, 4), (128, 4, 4),
       (256, 32, 2), (512, 16, 2), (256, 64, 4)]


V9L = [(256, 32, 4), (256, 32, 2), (512, 16, 4), (256, 4, 4), (256, 4, 2), (256, 16, 4),
       (64, 4, 4), (64, 4, 2), (128, 8, 4), (256, 8, 4), (64, 16, 4), (256, 64, 4), (64, 8, 4),
       (64, 8, 2), (256, 8, 2), (256, 16, 2), (512, 32, 4), (64, 2, 2), (512, 32, 2), (128, 4, 2)]
V9A = [(256, 32, 4), (256, 32, 2), (512, 16, 4), (256, 4, 4), (256, 4, 2), (256, 16, 4),
       (256, 8, 4), (256, 8, 2), (256, 16, 2), (512, 32, 4), (512, 32, 2), (128, 4, 2),
       (128, 8, 4), (512, 8, 2), (512, 4, 2)]
ONLY = os.environ.get("TUNE_ONLY")  # e.g. "91-96": restrict to these variant numbers


def candidates(N, slack):
    c = _candidates(N, slack)
    if ONLY:
        lo, hi = (int(x) for x in ONLY.split("-"))
        c = [x for x in c if lo <= x[0] <= hi]
    return c


def _candidates(N, slack):
    c = [(2, bl, pp) for bl, pp in V2 if N <= bl * pp <= max(slack * N, 64)]
    c += [(95 if g == 4 else 96, bl, pp) for bl, pp, g in V9L if N <= bl * pp <= max(slack * N, 64)]
    c += [(97 if g == 4 else 98, bl, pp) for bl, pp, g in V9A if N <= bl * pp <= max(slack * N, 64)]
    c += [(110 + g, bl, pp) for bl, pp, g in V11 if N <= bl * pp <= max(slack * N, 64)]
    c += [(90 + g, bl, pp) for bl, pp, g in V9 if N <= bl * pp <= max(slack * N, 64)]
    c += [(120, 256, 32)] if N <= 8192 <= max(slack * N, 64) else []  # v12 cells
    return c


def main():
    import torch  # first: the lab .so then shares torch's HIP runtime
    from oracle import oracle as O
    O.set_threads(16)
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    L = ctypes.CDLL(LAB_SO)
    L.pn2_fps_tune.restype = ctypes.c_int
    L.pn2_fps_tune.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    B = int(os.environ.get("TUNE_B", "16"))
    rounds = int(os.environ.get("TUNE_ROUNDS", "5"))
    sizes = [(64, 16), (128, 32), (256, 64), (512, 128), (1024, 256), (2048, 256), (4096, 512),
             (8192, 1024), (16384, 512)]
    if os.environ.get("TUNE_SIZES"):  # e.g. "8192:1024,1024:256"
        sizes = [tuple(int(v) for v in t.split(":")) for t in os.environ["TUNE_SIZES"].split(",")]
    stream = torch.cuda.current_stream().cuda_stream
    # exactness of every candidate on tie-heavy inputs first (grid lattice, duplicates, uniform)
    rng = np.random.default_rng(0)
    g = np.stack(np.meshgrid(*[np.arange(16)] * 3, indexing="ij"), -1).reshape(-1, 3)
    for N, M in sizes + [(100, 37), (700, 200), (3000, 300)]:
        tests = [np.stack([g[rng.integers(0, len(g), N)] for _ in range(4)]).astype(np.float32),
                 pkg.synth.batch(range(4), N, "uniform")[0],
                 np.repeat(pkg.synth.batch(range(4), N // 3 + 1, "scannet")[0], 3, axis=1)[:, :N]]
        for x in tests:
            x = np.ascontiguousarray(x)
            xt = torch.from_numpy(x).to(dev)
            ref = torch.from_numpy(O.fps(x, M)).to(dev)
            out = torch.empty((4, M), dtype=torch.int32, device=dev)
            for v, bl, pp in candidates(N, 4):
                assert L.pn2_fps_tune(xt.data_ptr(), 4, N, M, out.data_ptr(), None, v, bl, pp,
                                      stream) == 0, (v, bl, pp)
                torch.cuda.synchronize()
                assert torch.equal(out, ref), f"variant {(v, bl, pp)} differs at N={N}"
    print(json.dumps({"exactness": "all v2/v9 configs index-exact vs the oracle on grid/uniform/dup inputs"}),
          flush=True)
    for N, M in sizes:
        x = pkg.synth.batch(range(B), N, "scannet")[0]
        xyz = torch.from_numpy(x).to(dev)
        ref = torch.from_numpy(O.fps(x, M)).to(dev)
        cand = candidates(N, 2)
        times = {c: [] for c in cand}
        out = torch.empty((B, M), dtype=torch.int32, device=dev)
        nx = torch.empty((B, M, 3), dtype=torch.float32, device=dev)
        for c in cand:  # warm + verify
            rc = L.pn2_fps_tune(xyz.data_ptr(), B, N, M, out.data_ptr(), nx.data_ptr(), *c, stream)
            assert rc == 0, (c, rc)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), f"config {c} differs at N={N}"
        for _ in range(rounds):
            for c in cand:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                L.pn2_fps_tune(xyz.data_ptr(), B, N, M, out.data_ptr(), nx.data_ptr(), *c, stream)
                b.record()
                b.synchronize()
                times[c].append(a.elapsed_time(b) * 1e3)
        best = min(cand, key=lambda c: statistics.median(times[c]))
        for c in cand:
            print(json.dumps({"N": N, "M": M, "B": B, "variant": c[0], "block": c[1], "ppt": c[2],
                              "median_us": statistics.median(times[c]), "min_us": min(times[c]),
                              "us_per_iter": statistics.median(times[c]) / (M - 1),
                              "best": c == best}), flush=True)


if __name__ == "__main__":
    main()
