#!/usr/bin/env python3
"""Diagnostic: phase cycles of the culled hot-set sampler (fps_hotcull_kernel, stamped lab
build), B = 16 SA1 clouds, index-exact against the v9 sampler: refreshes, stalls, applied
(cell, centre) pairs, cycles per phase (wave 0 and the mean of the other waves), per-wave
group costs and the per-round event breakdown.

    python tools/stamp_fps_cull.py [--msg] [--json profiles/r2/sa1_cull_stamps.json]

--msg: the MSG SA1 size (B = 8, 16384 -> 512, coordinates read from L2).

--json writes the ScanNet summary bench.py reports as roofline.latency."""
import ctypes, importlib, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from conftest import PKG_NAME  # noqa: E402
pkg = importlib.import_module(PKG_NAME)
L = ctypes.CDLL(os.environ.get("PN2_STAMP_LIB") or os.path.join(ROOT, "tools", "fps_stamp", "libpn2fpsstamp.so"))
for _f in (L.pn2_fps_cull_stamp, L.pn2_fps_cull_stamp_msg):
    _f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
import argparse
ap = argparse.ArgumentParser()
ap.add_argument("--json")
ap.add_argument("--msg", action="store_true")
ARGS = ap.parse_args()
SUMMARY = {}
NAMES = ["cold_async", "tmax", "B_A", "out_count", "B_B", "append", "B_C", "hot_setup"]
dev = torch.device("cuda:0")
lib = pkg._lib.lib()
for kind in ("scannet", "uniform"):
    B, N, M = (8, 16384, 512) if ARGS.msg else (16, 8192, 1024)
    x = torch.from_numpy(pkg.synth.batch(range(B), N, kind)[0]).to(dev)
    idx = torch.empty((B, M), dtype=torch.int32, device=dev)
    buf = np.zeros(16 * 16 * 8, np.uint64)
    stats = np.zeros(16 * 8, np.uint64)
    for _ in range(2):
        rc = (L.pn2_fps_cull_stamp_msg if ARGS.msg else L.pn2_fps_cull_stamp)(
            x.data_ptr(), B, N, M, idx.data_ptr(), buf.ctypes.data, stats.ctypes.data)
        assert rc == 0, rc
    ref = torch.empty((B, M), dtype=torch.int32, device=dev)
    rnx = torch.empty((B, M, 3), dtype=torch.float32, device=dev)
    assert lib.pn2_fps_gather_sched(x.data_ptr(), B, N, M, ref.data_ptr(), rnx.data_ptr(),
                                    pkg._lib.PN2_FPS_BLOCKSCAN,
                                    torch.cuda.current_stream().cuda_stream) == 0
    wv = np.zeros(16 * 16 * 4, np.uint64)
    L.pn2_fps_cull_waves.argtypes = [ctypes.c_void_p]
    assert L.pn2_fps_cull_waves(wv.ctypes.data) == 0
    wv = wv.reshape(16, 16, 4)[:B].astype(np.float64)
    print(json.dumps({"kind": kind, "per_wave_groups": [round(v) for v in wv[:, :, 0].mean(0)],
                      "per_wave_cyc_per_group": [round(v) for v in (wv[:, :, 1] / np.maximum(wv[:, :, 0], 1)).mean(0)],
                      "per_wave_pairs": [round(v) for v in wv[:, :, 2].mean(0)],
                      "per_wave_polls": [round(v) for v in wv[:, :, 3].mean(0)]}), flush=True)
    a = buf.reshape(16, 16, 8)[:B].astype(np.float64)
    st = stats.reshape(16, 8)[:B].astype(np.float64)
    print(json.dumps({
        "kind": kind, "exact_vs_v9": bool(torch.equal(ref, idx)),
        "kernel_cycles": round(st[:, 0].mean()), "refresh": st[:, 1].mean(), "stall": st[:, 2].mean(),
        "pairs_w1": st[:, 3].mean(), "pairs_w2": st[:, 5].mean(), "hot_picks": st[:, 4].mean(), "tail_cycles_w1": st[:, 6].mean(), "tail_groups_w1": st[:, 7].mean(),
        "wave0": {n: round(v) for n, v in zip(NAMES, a[:, 0, :].mean(0))},
        "others": {n: round(v) for n, v in zip(NAMES, a[:, 1:, :].mean((0, 1)))},
    }), flush=True)
# per-round events of cloud 0 (register-buffered, stored after each round's last barrier):
# wave 0: [0] hot phase end; cold waves: [0] async loop end, [1] tail end; all: [2] after B1,
# [3] before B2 (counts), [4] after B2, [5] before B3 (append), [6] after B3
    L.pn2_fps_cull_events.argtypes = [ctypes.c_void_p]
    evb = np.zeros(64 * 16 * 8, np.uint64)
    assert L.pn2_fps_cull_events(evb.ctypes.data) == 0
    E = evb.reshape(64, 16, 8).astype(np.int64)
    rows = []
    for r_ in range(2, 40):
        h_end = E[r_, 0, 0]
        if h_end == 0 or E[r_, 0, 2] == 0:
            continue
        cold_end = E[r_, 1:, 1].max()
        rows.append({"hot_end_to_last_loop_end": int(E[r_, 1:, 0].max() - h_end),
                     "tail_max": int((E[r_, 1:, 1] - E[r_, 1:, 0]).max()),
                     "hot_end_to_last_cold": int(cold_end - h_end),
                     "last_cold_to_B1": int(E[r_, 0, 2] - cold_end),
                     "B1_to_B2": int(E[r_, 0, 4] - E[r_, 0, 2]),
                     "count_max": int((E[r_, 1:, 3] - E[r_, 1:, 2]).max()),
                     "B2_to_B3": int(E[r_, 0, 6] - E[r_, 0, 4]),
                     "append_max": int((E[r_, 1:, 5] - E[r_, 1:, 4]).max()),
                     "B3_to_next_hot_end": int(E[r_ + 1, 0, 0] - E[r_, 0, 6]) if E[r_ + 1, 0, 0] else None})
    # per cold wave: median cycles from the hot phase's end to its loop end / tail end, and how
    # often it is the last to finish (which waves the round's end waits for)
    rr = [r_ for r_ in range(2, 40) if E[r_, 0, 0] and E[r_, 0, 2]]
    print(json.dumps({"kind": kind, "per_wave_loop_end_after_hot": [
        int(np.median([E[r_, w_, 0] - E[r_, 0, 0] for r_ in rr])) for w_ in range(1, 16)],
        "per_wave_tail_end_after_hot": [
        int(np.median([E[r_, w_, 1] - E[r_, 0, 0] for r_ in rr])) for w_ in range(1, 16)],
        "last_wave_counts": np.bincount([int(np.argmax(E[r_, 1:, 1])) + 1 for r_ in rr],
                                        minlength=16).tolist()}), flush=True)
    keys = rows[0].keys()
    med = {k: float(np.median([r[k] for r in rows if r[k] is not None])) for k in keys}
    print(json.dumps({"kind": kind, "median_per_round": med, "rounds": len(rows)}), flush=True)
    if kind == "scannet":
        setup = float(a[:, 1:, 7].mean())  # cold waves' phase 7 = setup only
        hot_total = float(a[:, 0, 7].mean()) - setup
        SUMMARY.update({
            "workload": (f"B={B} ScanNet crops, {N} -> {M} ("
                         + ("cfg5 MSG SA1" if ARGS.msg else "cfg2 SA1") + "), stamped build (tools/fps_stamp)"),
            "kernel_cycles": float(st[:, 0].mean()), "setup_cycles": setup,
            "hot_cycles_per_pick": hot_total / float(st[:, 4].mean()),
            "rounds": float(st[:, 1].mean()), "stalls": float(st[:, 2].mean()),
            "round_cycles": (float(st[:, 0].mean()) - setup - hot_total) / float(st[:, 1].mean()),
            "median_round_events": med})

if ARGS.json:
    with open(ARGS.json, "w") as f:
        json.dump(SUMMARY, f, indent=1)
