#!/usr/bin/env python3
"""Diagnostic: per-workgroup phase cycles of fp_grid_fused_kernel at FP4 size (B = 16, n = 8192
<- m = 1024, C2 = 128), from the stamped build (make -C .../csrc variant VFILE=interp
VNAME=fpgst VFLAGS=-DPN2_FPG_STAMP=1; run with PN2HIP_LIB pointing at it). Phases: header
(bbox + grid_dims), sort (count, scan, scatter), search, write (issue); plus when the
workgroups start and end relative to the first start -- whether they run in lockstep."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    L = pkg.lib()
    L.pn2_fpg_stamps.argtypes = [ctypes.c_void_p]
    B, n, m = 16, 8192, 1024
    t1 = torch.from_numpy(pkg.synth.batch(range(B), n, "scannet")[0]).to(dev)
    _, k = pkg.tf_sampling.farthest_point_sample_and_gather(m, t1)
    ug = pkg.grid.PointGrid(t1, 0.1)
    kg = pkg.grid.PointGrid(k)
    st = torch.cuda.current_stream().cuda_stream
    p2 = torch.rand((B, m, 128), device=dev)
    out = torch.empty((B, n, 128), device=dev)
    res = {}
    for name, known in (("build", None), ("known", kg)):
        buf = np.zeros(4096 * 8, np.uint64)
        for _ in range(3):
            if known is None:
                L.pn2_fp_grid_fused(None, k.data_ptr(), ug.buf.data_ptr(), None, 0, p2.data_ptr(),
                                    128, B, n, m, out.data_ptr(), None, None, st)
            else:
                L.pn2_fp_grid_fused_known(known.buf.data_ptr(), None, k.data_ptr(),
                                          ug.buf.data_ptr(), None, 0, p2.data_ptr(), 128, B, n,
                                          m, out.data_ptr(), None, None, st)
        torch.cuda.synchronize()
        assert L.pn2_fpg_stamps(buf.ctypes.data) == 0
        s = buf.reshape(4096, 8)[:2048].astype(np.int64)
        t0 = s[:, 0].min()
        ph = {"header": s[:, 1] - s[:, 0], "sort": s[:, 2] - s[:, 1], "search": s[:, 3] - s[:, 2],
              "write": s[:, 4] - s[:, 3]}
        if known is not None:
            ph = {"stage": s[:, 2] - s[:, 0], "search": ph["search"], "write": ph["write"]}
        q = lambda v: {"mean": int(v.mean()), "p10": int(np.percentile(v, 10)),  # noqa: E731
                       "p90": int(np.percentile(v, 90))}
        res[name] = {k_: q(v) for k_, v in ph.items()}
        res[name]["start"] = q(s[:, 0] - t0)
        res[name]["end"] = q(s[:, 4] - t0)
        res[name]["span_cycles"] = int(s[:, 4].max() - t0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
