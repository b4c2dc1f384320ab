#!/usr/bin/env python3
"""Diagnostic: how much the SA1 sampler (B=16 x 8192 -> 1024) slows when other work runs on
the remaining CUs. The sampler runs on a high-priority stream (its own queue); a background
stream keeps the rest of the chip busy with (a) nothing, (b) a pure-VALU spin kernel,
(c) a streaming HBM copy, (d) the fused MLP kernel of SA2 (matrix cores + LDS), (e) the
LDS-free grouping kernel.
Prints the sampler's mean HIP-event time per case."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    xyz = torch.from_numpy(pkg.synth.batch(range(16), 8192, "scannet")[0]).to(dev)
    idx = torch.empty((16, 1024), dtype=torch.int32, device=dev)
    nx = torch.empty((16, 1024, 3), dtype=torch.float32, device=dev)
    hi = torch.cuda.Stream(device=dev, priority=-1)
    bg = torch.cuda.Stream(device=dev)
    big_a = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    big_b = torch.empty_like(big_a)
    spin = torch.rand(1 << 22, device=dev)
    inp = pkg.stack.make_inputs("cfg2", list(range(16)), dev, model=True)
    mdl = inp["model"]
    x1 = pkg.tf_sampling.farthest_point_sample_and_gather(1024, xyz)[1]
    x2 = pkg.tf_sampling.farthest_point_sample_and_gather(256, x1)[1]
    p1 = torch.rand((16, 1024, 64), device=dev)
    gidx, _ = pkg.tf_grouping.query_ball_point(0.2, 32, x1, x2)
    torch.cuda.synchronize()

    def sampler():
        pkg.tf_sampling.farthest_point_sample_chain([1024], xyz, out=[(idx, nx)])

    loads = {
        "idle": None,
        "valu_spin": lambda: [spin.mul_(1.0000001).add_(1e-7) for _ in range(1)],
        "hbm_copy": lambda: big_b.copy_(big_a),
        "mlp_sa2": lambda: pkg.pointnet_util.group_mlp(x1, p1, x2, gidx, mdl.sa[1], "max"),
        "group_concat": lambda: pkg.pointnet_util.group_concat(x1, p1, x2, gidx,
                                                               want_grouped_xyz=False),
    }
    res = {}
    for name, load in loads.items():
        times = []
        for rep in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if load is not None:
                with torch.cuda.stream(bg):
                    for _ in range(40):
                        load()
            with torch.cuda.stream(hi):
                e0.record(hi)
                sampler()
                e1.record(hi)
            torch.cuda.synchronize()
            if rep >= 2:
                times.append(e0.elapsed_time(e1))
        res[name] = round(sum(times) / len(times), 4)
    print(json.dumps({"sa1_sampler_ms": res, "lib": pkg.LIB_PATH}))


if __name__ == "__main__":
    main()
