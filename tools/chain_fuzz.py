#!/usr/bin/env python3
"""Diagnostic: the fused sampler chain (pn2_fps_chain) against the stage-by-stage samplers
(farthest_point_sample_and_gather) on many clouds -- the BASELINE crops by id (the pipeline
tests' ids included) and synthetic kinds -- eagerly and with the chain launched repeatedly
back to back. Prints the mismatching (clouds, stage, first differing pick) and saves the
first mismatching cloud's chain input to gpurun_out/chain_fuzz_fail.npy."""
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
    ts = pkg.tf_sampling
    S = pkg.stack
    npts = [256, 64, 16]
    bad = []
    nclouds = 0

    def check(x1, tag):
        nonlocal nclouds
        B = x1.shape[0]
        for rep in range(3):
            outs = ts.farthest_point_sample_chain(npts, x1)
            cur = x1
            for si, ((idx, nx), m) in enumerate(zip(outs, npts)):
                ridx, rnx = ts.farthest_point_sample_and_gather(m, cur)
                if not torch.equal(idx, ridx):
                    a, r = idx.cpu().numpy(), ridx.cpu().numpy()
                    for b in range(B):
                        d = np.nonzero(a[b] != r[b])[0]
                        if len(d):
                            bad.append({"tag": tag, "rep": rep, "b": b, "stage": si,
                                        "first_j": int(d[0]), "ndiff": int(len(d))})
                            if not os.path.exists("gpurun_out/chain_fuzz_fail.npy"):
                                os.makedirs("gpurun_out", exist_ok=True)
                                np.save("gpurun_out/chain_fuzz_fail.npy", x1[b].cpu().numpy())
                    break
                cur = rnx
        nclouds += B

    for base in (0, 100, 116, 132, 200, 300):
        inp = S.make_inputs("cfg2", list(range(base, base + 16)), dev)
        x1 = ts.farthest_point_sample_and_gather(1024, inp["xyz"])[1]
        check(x1, f"cfg2:{base}")
    for kind in ("scannet", "uniform", "grid", "dup"):
        for seed in range(4):
            x = torch.from_numpy(pkg.synth.batch(range(seed * 16, seed * 16 + 16), 8192, kind)[0]
                                 if kind == "scannet" else
                                 np.ascontiguousarray(_synth(pkg, kind, 16, 1024, seed))).to(dev)
            if x.shape[1] > 1024:
                x = ts.farthest_point_sample_and_gather(1024, x)[1]
            check(x, f"{kind}:{seed}")
    print(json.dumps({"clouds": nclouds, "mismatches": len(bad), "first": bad[:20]}))


def _synth(pkg, kind, B, N, seed):
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        return rng.random((B, N, 3), dtype=np.float32)
    if kind == "grid":
        g = np.stack(np.meshgrid(*[np.arange(11)] * 3, indexing="ij"), -1).reshape(-1, 3)
        return np.stack([g[rng.permutation(len(g))[:N]] for _ in range(B)]).astype(np.float32) * 0.1
    base = rng.random((B, N // 4, 3), dtype=np.float32)
    return np.concatenate([base] * 4, axis=1)


if __name__ == "__main__":
    main()
