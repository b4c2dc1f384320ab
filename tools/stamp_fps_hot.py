#!/usr/bin/env python3
"""Diagnostic: where the hot-set sampler (csrc/fps_hot.h) spends its cycles -- s_memtime phase
stamps from the stamped lab build (tools/fps_lab, pn2_fps_hot_stamp), per cloud of a B = 16
SA1 batch: refresh rounds, hot picks, and the cycles per phase (wave 0 and the mean of the
other waves), checked index-exact against the production sampler."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from conftest import PKG_NAME  # noqa: E402

pkg = importlib.import_module(PKG_NAME)
L = ctypes.CDLL(os.path.join(ROOT, "tools", "fps_lab", "libpn2fpslab.so"))
L.pn2_fps_hot_stamp.restype = ctypes.c_int
L.pn2_fps_hot_stamp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_void_p, ctypes.c_void_p]
NAMES = ["cold_pass", "top3", "extract", "extract_barrier", "hot_or_wait", "top_barrier"]
dev = torch.device("cuda:0")
for kind, N, M in [("scannet", 8192, 1024), ("uniform", 8192, 1024)]:
    B = 16
    x = torch.from_numpy(pkg.synth.batch(range(B), N, kind)[0]).to(dev)
    idx = torch.empty((B, M), dtype=torch.int32, device=dev)
    buf = np.zeros(16 * 16 * 8, np.uint64)
    for _ in range(2):
        rc = L.pn2_fps_hot_stamp(x.data_ptr(), B, N, M, idx.data_ptr(), buf.ctypes.data)
        assert rc == 0, rc
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    rc = L.pn2_fps_hot_stamp(x.data_ptr(), B, N, M, idx.data_ptr(), buf.ctypes.data)
    ev[1].record()
    old = pkg._lib.lib().pn2_fps_set_algo(2)
    ev[2].record()
    ref = pkg.tf_sampling.farthest_point_sample(M, x)
    ev[3].record()
    torch.cuda.synchronize()
    pkg._lib.lib().pn2_fps_set_algo(old)
    t_stamped, t_prod = ev[0].elapsed_time(ev[1]), ev[2].elapsed_time(ev[3])
    assert torch.equal(ref, idx), "stamped hot sampler differs"
    a = buf.reshape(16, 16, 8).astype(np.float64)
    w0 = a[:, 0, :6].mean(0)
    wo = a[:, 1:4, :6].mean((0, 1))
    refresh = a[:, 0, 6]
    hot = a[:, 0, 7]
    tot = a[:, 0, :6].sum(1).mean()
    kclk = a[:, 8, 0].mean()
    krt_us = a[:, 8, 1].mean() / 100.0
    print(json.dumps({"kind": kind, "N": N, "M": M,
                      "refresh_rounds_mean": refresh.mean(), "refresh_rounds_max": refresh.max(),
                      "hot_picks_mean": hot.mean(),
                      "wave0_cycles": {n: round(v) for n, v in zip(NAMES, w0)},
                      "other_waves_cycles": {n: round(v) for n, v in zip(NAMES, wo)},
                      "total_cycles_wave0": round(tot),
                      "kernel_cycles": round(kclk), "kernel_us_realtime": round(krt_us, 1),
                      "clock_GHz": round(kclk / krt_us / 1e3, 3),
                      "event_ms_stamped_call": round(t_stamped, 3), "event_ms_production": round(t_prod, 3),
                      "per_refresh": {n: round(v / refresh.mean()) for n, v in zip(NAMES, w0)},
                      "hot_setup_per_refresh": round(a[:, 8, 2].mean() / refresh.mean()),
                      "hot_loop_cycles_per_pick": round(a[:, 8, 3].mean() / max(hot.mean(), 1)),
                      "tie_path_frac": round(a[:, 8, 4].mean() / max(hot.mean(), 1), 3),
                      "hot_cycles_per_pick": round(w0[4] / max(hot.mean(), 1))}), flush=True)
