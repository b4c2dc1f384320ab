#!/usr/bin/env python3
"""Time pn2_grid_build alone at the stack's shapes (HIP events, median of 30): cfg2's SA1 grid
(B = 16, N = 8192, edge 0.1), cfg5's MSG SA1 grid (B = 8, N = 16384, edge 0.2) and FP4's known
grid (B = 16, N = 1024, automatic edge). No checks: phase-split builds can be timed
(PN2HIP_LIB=...)."""
import ctypes
import importlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    L = pkg.lib()
    st = torch.cuda.current_stream().cuda_stream
    res = {"lib": os.path.basename(os.environ.get("PN2HIP_LIB") or "libpn2hip.so")}
    for name, B, N, edge in (("cfg2_sa1", 16, 8192, 0.1), ("cfg5_sa1", 8, 16384, 0.2),
                             ("fp4_known", 16, 1024, 0.0)):
        x = torch.from_numpy(pkg.synth.batch(range(B), N, "scannet")[0]).to(dev)
        nb = L.pn2_grid_size(B, N)
        buf = torch.empty((nb,), dtype=torch.uint8, device=dev)
        fn = lambda: L.pn2_grid_build(x.data_ptr(), B, N, ctypes.c_float(edge), buf.data_ptr(), nb, st)  # noqa: E731
        for _ in range(3):
            fn()
        ts = []
        for _ in range(30):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); fn(); b.record(); b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        res[name + "_us"] = round(statistics.median(ts), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
