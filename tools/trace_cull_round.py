#!/usr/bin/env python3
"""Diagnostic: per-wave timeline of one round (round 23, cloud 0) of the stamped hot-cull
sampler: hot phase start/end/picks; per cold wave the start of every group (cycles from the
hot start, with the centres applied before it and the published count), stop seen, loop end."""
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
L.pn2_fps_cull_round.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
B, N, M = 16, 8192, 1024
x = torch.from_numpy(pkg.synth.batch(range(B), N, "scannet")[0]).to(dev)
idx = torch.empty((B, M), dtype=torch.int32, device=dev)
buf = np.zeros(16 * 16 * 8, np.uint64); st = np.zeros(16 * 8, np.uint64)
for _ in range(2):
    assert L.pn2_fps_cull_stamp(x.data_ptr(), B, N, M, idx.data_ptr(), buf.ctypes.data, st.ctypes.data) == 0
r = np.zeros(16 * 64, np.uint64)
assert L.pn2_fps_cull_round(r.ctypes.data) == 0
r = r.reshape(16, 64)
t0 = int(r[0, 0])
print(json.dumps({"hot": [0, int(r[0, 1]) - t0], "picks": int(r[0, 2])}))
for w in range(1, 16):
    ev = []
    for k in range(2, 62):
        v = int(r[w, k])
        if not v:
            break
        ev.append([(v & ((1 << 48) - 1)) - (t0 & ((1 << 48) - 1)), (v >> 48) & 0xFF, (v >> 56) & 0xFF])
    print(json.dumps({"wave": w, "stop_seen": int(r[w, 0]) - t0, "end": int(r[w, 1]) - t0,
                      "groups[t,applied,avail]": ev}))
