import ctypes, importlib, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from conftest import PKG_NAME
pkg = importlib.import_module(PKG_NAME)
L = ctypes.CDLL(os.environ.get("PN2_STAMP_LIB") or os.path.join(ROOT, "tools", "fps_stamp", "libpn2fpsstamp.so"))
L.pn2_fps_cull_stamp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
L.pn2_fps_cull_events.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
B, N, M = 16, 8192, 1024
x = torch.from_numpy(pkg.synth.batch(range(B), N, "scannet")[0]).to(dev)
idx = torch.empty((B, M), dtype=torch.int32, device=dev)
buf = np.zeros(16 * 16 * 8, np.uint64); stats = np.zeros(16 * 8, np.uint64)
for _ in range(2):
    assert L.pn2_fps_cull_stamp(x.data_ptr(), B, N, M, idx.data_ptr(), buf.ctypes.data, stats.ctypes.data) == 0
evb = np.zeros(64 * 16 * 8, np.uint64)
assert L.pn2_fps_cull_events(evb.ctypes.data) == 0
E = evb.reshape(64, 16, 8).astype(np.int64)
rows = []
for r in range(2, 30):
    h = E[r, 0, 0]
    if h == 0 or E[r, 0, 2] == 0: continue
    lag = (E[r, 1:, 0] - h).tolist()          # cold loop end - hot end, per cold wave
    tail = (E[r, 1:, 1] - E[r, 1:, 0]).tolist()  # end-of-batch refresh per wave
    hot_len = int(h - E[r - 1, 0, 6]) if E[r - 1, 0, 6] else None  # hot phase length (from previous B3)
    rows.append({"round": r, "hot_phase": hot_len, "lag": lag, "tail": tail,
                 "B1_to_B3": int(E[r, 0, 6] - E[r, 0, 2])})
for row in rows: print(json.dumps(row))
lags = np.array([r["lag"] for r in rows])
print(json.dumps({"median_lag_per_wave": np.median(lags, 0).astype(int).tolist(),
                  "median_max_lag": float(np.median(lags.max(1)))}))
