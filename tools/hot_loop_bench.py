#!/usr/bin/env python3
"""Lab: cycles per pick of the hot-set pick loop (tools/fps_lab hot_loop_bench) and of its
variants with pieces removed (1 no ring write, 2 no tie check, 4 no readfirstlane)."""
import ctypes, importlib, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from conftest import PKG_NAME  # noqa: E402
pkg = importlib.import_module(PKG_NAME)
L = ctypes.CDLL(os.path.join(ROOT, "tools", "fps_lab", "libpn2fpslab.so"))
L.pn2_hot_loop_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
x = torch.from_numpy(pkg.synth.batch([0], 8192, "uniform")[0]).to(dev)
out = torch.empty(64, dtype=torch.int32, device=dev)
cyc = torch.zeros(1, dtype=torch.int64, device=dev)
res = {}
for var in (0, 1, 2, 3, 4, 7):
    best = None
    for _ in range(5):
        assert L.pn2_hot_loop_bench(x.data_ptr(), 4000, var, out.data_ptr(), cyc.data_ptr()) == 0
        c = int(cyc.item()) / 4000
        best = c if best is None else min(best, c)
    res[var] = round(best, 1)
print(json.dumps({"cycles_per_pick_by_variant": res}), flush=True)
