#!/usr/bin/env python3
"""Diagnostic: phase cycles of the culled hot-set sampler (fps_cull_kernel, stamped lab build),
B = 16 SA1 clouds, index-exact against the production v9 sampler: refreshes, stalls, applied
(cell, centre) pairs, cycles per phase (wave 0 and the mean of the other waves)."""
import ctypes, importlib, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from conftest import PKG_NAME  # noqa: E402
pkg = importlib.import_module(PKG_NAME)
L = ctypes.CDLL(os.path.join(ROOT, "tools", "fps_lab", "libpn2fpslab.so"))
L.pn2_fps_cull_stamp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
NAMES = ["cold_async", "tmax", "B_A", "out_count", "B_B", "append", "B_C", "hot_setup"]
dev = torch.device("cuda:0")
lib = pkg._lib.lib()
for kind in ("scannet", "uniform"):
    B, N, M = 16, 8192, 1024
    x = torch.from_numpy(pkg.synth.batch(range(B), N, kind)[0]).to(dev)
    idx = torch.empty((B, M), dtype=torch.int32, device=dev)
    buf = np.zeros(16 * 16 * 8, np.uint64)
    stats = np.zeros(16 * 8, np.uint64)
    for _ in range(2):
        rc = L.pn2_fps_cull_stamp(x.data_ptr(), B, N, M, idx.data_ptr(), buf.ctypes.data,
                                  stats.ctypes.data)
        assert rc == 0, rc
    old = lib.pn2_fps_set_algo(1)
    ref = pkg.tf_sampling.farthest_point_sample(M, x)
    lib.pn2_fps_set_algo(old)
    wv = np.zeros(16 * 16 * 4, np.uint64)
    L.pn2_fps_cull_waves.argtypes = [ctypes.c_void_p]
    assert L.pn2_fps_cull_waves(wv.ctypes.data) == 0
    wv = wv.reshape(16, 16, 4).astype(np.float64)
    print(json.dumps({"kind": kind, "per_wave_groups": [round(v) for v in wv[:, :, 0].mean(0)],
                      "per_wave_cyc_per_group": [round(v) for v in (wv[:, :, 1] / np.maximum(wv[:, :, 0], 1)).mean(0)],
                      "per_wave_pairs": [round(v) for v in wv[:, :, 2].mean(0)],
                      "per_wave_polls": [round(v) for v in wv[:, :, 3].mean(0)]}), flush=True)
    a = buf.reshape(16, 16, 8).astype(np.float64)
    st = stats.reshape(16, 8).astype(np.float64)
    print(json.dumps({
        "kind": kind, "exact_vs_v9": bool(torch.equal(ref, idx)),
        "kernel_cycles": round(st[:, 0].mean()), "refresh": st[:, 1].mean(), "stall": st[:, 2].mean(),
        "pairs_w1": st[:, 3].mean(), "pairs_w2": st[:, 5].mean(), "hot_picks": st[:, 4].mean(), "tail_cycles_w1": st[:, 6].mean(), "tail_groups_w1": st[:, 7].mean(),
        "wave0": {n: round(v) for n, v in zip(NAMES, a[:, 0, :].mean(0))},
        "others": {n: round(v) for n, v in zip(NAMES, a[:, 1:, :].mean((0, 1)))},
    }), flush=True)
# per-round timeline of cloud 0 (STAMP build, g_iter, cycles from the round's B2 of round 0):
# hot phase start/end/picks, wave 1 round start / counts done / stop seen / loop end, wave 0
# after B1 / after the choice / after B2, wave 1 before B2; wave 1 lag at stop, group cycles
if hasattr(L, "pn2_fps_cull_trace"):
    tr = np.zeros(4096, np.uint64)
    L.pn2_fps_cull_trace.argtypes = [ctypes.c_void_p]
    assert L.pn2_fps_cull_trace(tr.ctypes.data) == 0
    r = tr.reshape(256, 16).astype(np.int64)
    for i in list(range(0, 12)) + list(range(20, 26)):
        base = r[i, 6]
        rel = lambda v: int(v - base) if v else None
        x = int(r[i, 5])
        print(json.dumps({"round": i, "picks": int(r[i, 2]), "w0_B1": 0, "w0_choice": rel(r[i, 7]),
                          "w1_pre_B2": rel(r[i, 9]), "w0_B2": rel(r[i, 8]),
                          "next_w1_start": rel(r[i + 1, 10]), "next_w1_counts": rel(r[i + 1, 11]),
                          "next_hot": [rel(r[i + 1, 0]), rel(r[i + 1, 1])], "next_picks": int(r[i + 1, 2]),
                          "next_w1_stop_end": [rel(r[i + 1, 3]), rel(r[i + 1, 4])],
                          "next_B1": rel(r[i + 1, 6]),
                          "next_w1_lag": int(r[i + 1, 5]) & 0xFFFF, "next_w1_grp": (int(r[i + 1, 5]) >> 16) & 0xFFFF}), flush=True)
    for i in (20, 21, 22, 23, 24, 25, 40):
        base = r[i, 1]
        ends = [int(v - base) for v in r[128 + i // 16][(i % 16):(i % 16) + 1]] if False else None
        ends = [int(tr[2048 + i * 16 + v]) - int(r[i, 1]) if r[i, 1] else None for v in range(1, 16)]
        print(json.dumps({"round": i, "picks": int(r[i, 2]), "cold_end_minus_hot_end": ends}), flush=True)
    gaps = [int(r[i, 6] - r[i, 1]) for i in range(1, 60) if r[i, 2] > 0 and r[i, 6] > r[i, 1]]
    nxt = [int(r[i + 1, 0] - r[i, 6]) for i in range(1, 60) if r[i + 1, 2] > 0 and r[i + 1, 0] > r[i, 6]]
    picks = [int(r[i, 2]) for i in range(1, 60) if r[i, 2] > 0]
    print(json.dumps({"hot_end_to_B1": gaps, "B1_to_next_hot": nxt, "picks": picks}), flush=True)
    for i in range(20, 31):
        ends = [int(tr[2048 + i * 16 + v]) for v in range(1, 16)]
        he = int(r[i, 1])
        print(json.dumps({"round": i, "picks": int(r[i, 2]), "cold_end_minus_hot_end": [e - he for e in ends],
                          "B1_minus_hot_end": int(r[i, 6]) - he}), flush=True)
