#!/usr/bin/env python3
"""Time the fused shared-MLP kernels (csrc/mlp.hip) alone, at the whole-model step's shapes
(stack.SemSegModel, B clouds), one layer at a time on an otherwise idle GPU.

    python tools/bench_mlp.py [--batch 16] [--iters 20] [--lib path/to/libpn2hip.so]

Prints one JSON line per layer: time per launch, the matrix-core FLOPs it does (padded to
the kernel's tiles: 32 output columns, 8 input features) and the fraction of the fp32 MFMA
peak (157.3 TFLOP/s, MI355X_MICROARCH.md).
"""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PEAK_TFLOPS = 157.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3"])
    args = ap.parse_args()
    if args.lib:
        os.environ["PN2HIP_LIB"] = args.lib
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    S, pu = pkg.stack, pkg.pointnet_util
    dev = torch.device("cuda:0")
    B = args.batch
    inp = S.make_inputs(args.config, list(range(B)), dev, model=True)
    mdl = inp["model"]
    xyz = [inp["xyz"]]
    for (m, _, _, _) in S.SSG_SA:
        xyz.append(pkg.tf_sampling.farthest_point_sample_and_gather(m, xyz[-1])[1])
    g = torch.Generator(device=dev)
    g.manual_seed(0)

    def feats(n, c):
        return torch.rand((B, n, c), generator=g, device=dev) * 2 - 1

    def flops(mlp, rows):
        f = 0
        for L in mlp.layers:
            f += 2 * rows * ((L.cin + 7) // 8 * 8) * ((L.cout + 31) // 32 * 32)
        return f

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.iters * 1e3  # us

    rows_out = []
    pts = [inp["feats"]] + [feats(m, c) for (m, _, _, c) in S.SSG_SA]
    for i, (m, r, ns, c) in enumerate(S.SSG_SA):
        idx, _ = pkg.tf_grouping.query_ball_point(r, ns, xyz[i], xyz[i + 1])
        mlp = mdl.sa[i]
        if mdl.attention:
            us = timeit(lambda: pkg.attention_layer.group_mlp_attention(
                xyz[i], pts[i], xyz[i + 1], idx, mlp, mdl.store, f"layer{i + 1}"))
            fl = flops(mlp, B * m * ns) + 2 * 2 * B * m * ns * c * c + 2 * B * m * 32 * c * c
        else:
            us = timeit(lambda: pu.group_mlp(xyz[i], pts[i], xyz[i + 1], idx, mlp, "max"))
            fl = flops(mlp, B * m * ns)
        rows_out.append((f"SA{i + 1}", us, fl))
    p2 = pts[4]
    for k in range(4):
        lvl = 3 - k
        dist, nidx = pkg.tf_interpolate.three_nn(xyz[lvl], xyz[lvl + 1])
        mlp = mdl.fp[k]
        p1 = pts[lvl] if lvl > 0 else inp["feats"]
        us = timeit(lambda: pu.fp_mlp(dist, nidx, p1, p2, mlp))
        rows_out.append((f"FP{k + 1}", us, flops(mlp, B * int(xyz[lvl].shape[1]))))
        p2 = feats(int(xyz[lvl].shape[1]), mlp.cout if k < 3 else 128)
    tot_us = sum(r[1] for r in rows_out)
    for name, us, fl in rows_out:
        print(json.dumps({"layer": name, "us": round(us, 1), "tflops": round(fl / us / 1e6, 1),
                          "frac_fp32_mfma": round(fl / us / 1e6 / PEAK_TFLOPS, 3)}))
    print(json.dumps({"total_us": round(tot_us, 1), "batch": B}))


if __name__ == "__main__":
    main()
