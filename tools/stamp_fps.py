#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of the FPS iteration (s_memtime stamps, stamped build)."""
import ctypes, importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "fps_lab", "libpn2fpslab.so"))
L.pn2_fps_stamp.restype = ctypes.c_int
L.pn2_fps_stamp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
names = ["scan", "wave_reduce", "write+barrier", "xwave_reduce", "centre_load", "idx_store"]
# v6 rows (block < 0): scan = active-cell scans, wave_reduce = lane max + wave reduce, idx_store also holds the setup
names9 = ["scan", "wave_max", "ballot+resolve", "write+barrier", "xwave", "centre+store"]
RUNS = [(8192, 1024, 256, 95032), (8192, 1024, 256, 97032), (1024, 256, 256, 95004),
        (1024, 256, 256, 97004)]
for N, M, bl, pp in RUNS:
    x = torch.from_numpy(pkg.synth.batch([0], N, "scannet")[0]).to(dev)
    idx = torch.empty((1, M), dtype=torch.int32, device=dev)
    buf = np.zeros(16 * 8 + 4096, np.uint64)
    for _ in range(2):
        rc = L.pn2_fps_stamp(x.data_ptr(), N, M, idx.data_ptr(), bl, pp, buf.ctypes.data)
    assert rc == 0, rc
    ref = pkg.tf_sampling.farthest_point_sample(M, x)
    assert torch.equal(ref, idx)
    nw = abs(bl) // 64
    a = buf[:128].reshape(16, 8)[:nw, :6].astype(np.float64) / (M - 1)
    if bl < 0:
        it = buf[128:128 + M].astype(np.int64)
        d = np.diff(it[1:M])
        print("   per-iteration cycles (wave 0), iterations 1..:", [int(np.median(d[i:i + 64])) for i in range(0, len(d), 64)])
    nm = names9 if pp >= 90000 else names
    if 97000 <= pp < 98000:
        nm = ["scan+lane_resolve", "wave_max", "ballot+readlane", "atomic+barrier", "read+decode",
              "centre+store"]
    if 95000 <= pp < 96000:
        nm = ["scan+lane_resolve", "wave_max", "ballot+readlane", "write+barrier", "xwave",
              "centre+store"]
    if pp >= 110000:
        nm = ["scan", "wave_max", "resolve+coords", "write+barrier", "xwave+coords", "store"]
    print(f"N={N} M={M} block={bl} ppt={pp}: cycles/iter per phase (mean over {nw} waves):",
          {n: round(v, 1) for n, v in zip(nm, a.mean(0))}, "total", round(a.sum(1).mean(), 1),
          flush=True)
