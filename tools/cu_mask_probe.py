#!/usr/bin/env python3
"""How a CU mask (include/pn2plan.h pn2_stream_create_cu_mask) changes a side-lane kernel's
time: the cfg2 SA2-SA4 grouping (pn2_ball_group_layers) and SA1's grid query + grouping
(pn2_ball_group_xyz_grid), alone on a stream masked to K of the 256 CUs with different bit
patterns, HIP events, median of 15.

    python tools/cu_mask_probe.py"""
import ctypes
import importlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    S, PU = pkg.stack, pkg.pointnet_util
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    L = pkg.lib()
    inp = S.make_inputs("cfg2", list(range(16)), dev)
    xyz = [inp["xyz"]]
    for npoint, _, _, _ in S.SSG_SA:
        xyz.append(pkg.tf_sampling.farthest_point_sample_and_gather(npoint, xyz[-1])[1])
    points = [inp["feats"]] + list(inp["sa_out"])
    sa = [(S.SSG_SA[i][1], S.SSG_SA[i][2], xyz[i], points[i], xyz[i + 1]) for i in (1, 2, 3)]
    grid = pkg.tf_grouping.BallGrid(xyz[0], 0.1)
    torch.cuda.synchronize()

    def masked(bits):
        words = (ncu + 31) // 32
        arr = (ctypes.c_uint32 * words)(*[0] * words)
        for i in bits:
            arr[i // 32] |= 1 << (i % 32)
        h = ctypes.c_void_p()
        assert L.pn2_stream_create_cu_mask(arr, words, ctypes.byref(h)) == 0
        return torch.cuda.ExternalStream(h.value, device=dev)

    def timeit(fn, st, reps=15):
        with torch.cuda.stream(st):
            for _ in range(3):
                fn()
            ts = []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st); fn(); b.record(st); b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
        return statistics.median(ts)

    pats = {"all": range(ncu),
            "8_of_32_off (192)": [i for i in range(ncu) if i % 32 >= 8],
            "every_4th_off (192)": [i for i in range(ncu) if i % 4 != 0],
            "16_of_32_off (128)": [i for i in range(ncu) if i % 32 >= 16],
            "first_192": range(192),
            "odd (128)": [i for i in range(ncu) if i % 2]}
    res = {}
    for name, bits in pats.items():
        st = masked(list(bits))
        res[name] = {"sa234_us": round(timeit(lambda: PU.ball_group_layers(sa), st), 1),
                     "sa1_grid_us": round(timeit(lambda: PU.ball_group_xyz(0.1, 32, xyz[0], xyz[1], grid), st), 1)}
    res["unmasked stream"] = {"sa234_us": round(timeit(lambda: PU.ball_group_layers(sa), torch.cuda.Stream()), 1),
                              "sa1_grid_us": round(timeit(lambda: PU.ball_group_xyz(0.1, 32, xyz[0], xyz[1], grid), torch.cuda.Stream()), 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
