#!/usr/bin/env python3
"""Diagnostic: phase cycles of the asynchronous hot-set sampler (fps_hota_kernel, stamped lab
build), B = 16 SA1 clouds, checked index-exact against the production v9 sampler."""
import ctypes, importlib, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from conftest import PKG_NAME  # noqa: E402
pkg = importlib.import_module(PKG_NAME)
L = ctypes.CDLL(os.path.join(ROOT, "tools", "fps_lab", "libpn2fpslab.so"))
L.pn2_fps_hota_stamp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]
NAMES = ["B1_wait", "write_out", "catch_up", "top3_extract", "B2_wait", "hot_setup", "loop"]
dev = torch.device("cuda:0")
lib = pkg._lib.lib()
for kind in ("scannet", "uniform"):
    B, N, M = 16, 8192, 1024
    x = torch.from_numpy(pkg.synth.batch(range(B), N, kind)[0]).to(dev)
    idx = torch.empty((B, M), dtype=torch.int32, device=dev)
    buf = np.zeros(16 * 16 * 8, np.uint64)
    for _ in range(2):
        assert L.pn2_fps_hota_stamp(x.data_ptr(), B, N, M, idx.data_ptr(), buf.ctypes.data) == 0
    old = lib.pn2_fps_set_algo(1)
    ref = pkg.tf_sampling.farthest_point_sample(M, x)
    lib.pn2_fps_set_algo(old)
    a = buf.reshape(16, 16, 8).astype(np.float64)
    x12 = a[:, 12, :]
    rounds = x12[:, 2].mean()
    print(json.dumps({
        "kind": kind, "exact_vs_v9": bool(torch.equal(ref, idx)),
        "kernel_us": round(x12[:, 1].mean() / 100, 1), "clock_GHz": round(x12[:, 0].mean() / (x12[:, 1].mean() * 10), 3),
        "rounds": rounds, "hot_picks": x12[:, 3].mean(), "tie_frac": round(x12[:, 4].mean() / 1023, 3),
        "async_applied_w1": x12[:, 5].mean(), "spins_w1": x12[:, 6].mean(),
        "hot_wave": {n: round(v) for n, v in zip(NAMES, a[:, 0, :7].mean(0))},
        "cold_waves": {n: round(v) for n, v in zip(NAMES, a[:, 1:8, :7].mean((0, 1)))},
        "cold_B1_wait_by_wave": [round(v) for v in a[:, 1:8, 0].mean(0)],
        "hot_loop_per_pick": round(a[:, 0, 6].mean() / max(x12[:, 3].mean(), 1)),
    }), flush=True)
