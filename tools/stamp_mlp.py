#!/usr/bin/env python3
"""Diagnostic: where the fused MLP kernel's time goes, per phase (s_memtime stamps of the
stamped build csrc/build/libpn2hip_stamp.so, `make -C .../csrc stamp`).

For the whole-model layer shapes (SA1..SA4 group + MLP + pool, FP1..FP4 interpolation + MLP)
prints, averaged over the first 4096 workgroups: metadata, gather, each layer, pooling (in
s_memtime ticks and as a share of the workgroup's life). --attention: the cfg3 model's
attention SA layers, with the tail split into query, K/V products and scores/softmax."""
import ctypes
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STAMP_LIB = os.path.join(ROOT, "pointcloud-segmentation-attention_amd", "csrc", "build",
                         "libpn2hip_stamp.so")
os.environ["PN2HIP_LIB"] = STAMP_LIB

import numpy as np  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
S, pu = pkg.stack, pkg.pointnet_util
lib = pkg.lib()
lib.pn2_mlp_set_stamp.argtypes = [ctypes.c_void_p]
lib.pn2_mlp_set_stamp.restype = None
dev = torch.device("cuda:0")
B = 16
ATTN = "--attention" in sys.argv  # cfg3: rgb+normals, attention pooling in every SA
inp = S.make_inputs("cfg3" if ATTN else "cfg2", list(range(B)), dev, model=True)
mdl = inp["model"]
xyz = [inp["xyz"]]
for (m, _, _, _) in S.SSG_SA:
    xyz.append(pkg.tf_sampling.farthest_point_sample_and_gather(m, xyz[-1])[1])
g = torch.Generator(device=dev)
g.manual_seed(0)


def feats(n, c):
    return torch.rand((B, n, c), generator=g, device=dev) * 2 - 1


stamp = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)


def run(name, fn, nl):
    fn()
    torch.cuda.synchronize()
    stamp.zero_()
    lib.pn2_mlp_set_stamp(stamp.data_ptr())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    lib.pn2_mlp_set_stamp(None)
    us = e0.elapsed_time(e1) * 1e3
    t = stamp.cpu().numpy().reshape(4096, 16).astype(np.int64)
    t = t[(t[:, 0] > 0) & (t[:, 15] > 0)]
    life = t[:, 15] - t[:, 0]
    ph = {"meta": t[:, 1] - t[:, 0], "gather": t[:, 2] - t[:, 1]}
    prev = 2
    for l in range(nl):
        ph[f"L{l + 1}"] = t[:, 3 + l] - t[:, prev]
        prev = 3 + l
    if ATTN and name.startswith("SA"):  # attention tail: query, K/V (segment 0), scores
        ph["attn_q"] = t[:, 9] - t[:, prev]
        ph["attn_kv"] = t[:, 13] - t[:, 9]
        ph["attn_scores"] = t[:, 14] - t[:, 13]
        ph["attn_rest"] = t[:, 15] - t[:, 14]
    else:
        ph["pool"] = t[:, 15] - t[:, prev]
    sub = t[(t[:, 10] > 0) & (t[:, 11] > 0) & (t[:, 12] > 0)]
    if len(sub):  # the last layer's first item of wave 0 (stamped builds): MMA, epilogue
        ph["last_item_mma"] = sub[:, 11] - sub[:, 10]
        ph["last_item_epi"] = sub[:, 12] - sub[:, 11]
    # (s_memtime counters of different XCDs are not synchronised: only durations within one
    # workgroup are compared)
    print(json.dumps({"layer": name, "event_us": round(us, 1), "wgs_stamped": int(len(t)),
                      "mean_life_ticks": int(life.mean()),
                      "phase_share": {k: round(float(v.mean() / life.mean()), 3) for k, v in ph.items()},
                      "phase_ticks": {k: int(v.mean()) for k, v in ph.items()}}),
          flush=True)


pts = [inp["feats"]] + [feats(m, c) for (m, _, _, c) in S.SSG_SA]
for i, (m, r, ns, _) in enumerate(S.SSG_SA):
    idx, _ = pkg.tf_grouping.query_ball_point(r, ns, xyz[i], xyz[i + 1])
    if ATTN:
        fn = lambda: pkg.attention_layer.group_mlp_attention(  # noqa: E731
            xyz[i], pts[i], xyz[i + 1], idx, mdl.sa[i], mdl.store, f"layer{i + 1}")
    else:
        fn = lambda: pu.group_mlp(xyz[i], pts[i], xyz[i + 1], idx, mdl.sa[i], "max")  # noqa: E731
    run(f"SA{i + 1}", fn, len(mdl.sa[i].layers))
p2 = pts[4]
for k in range(4 if "--fp" in sys.argv else 0):
    lvl = 3 - k
    dist, nidx = pkg.tf_interpolate.three_nn(xyz[lvl], xyz[lvl + 1])
    p1 = pts[lvl]
    run(f"FP{k + 1}", lambda: pu.fp_mlp(dist, nidx, p1, p2, mdl.fp[k]), len(mdl.fp[k].layers))
    p2 = feats(int(xyz[lvl].shape[1]), mdl.fp[k].cout if k < 3 else 128)
