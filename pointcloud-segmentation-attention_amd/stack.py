"""The SA + FP geometric path of the reference's segmentation models, as the benchmark step.

Layer hyper-parameters are the reference's:
  SSG (cfg2/cfg3)  pointnet2_sem_seg_attention.py:28-53 = pointnet2_sem_seg_features.py:29-50
      SA npoint/radius/nsample/mlp[-1]: 1024/0.1/32/64, 256/0.2/32/128, 64/0.4/32/256,
      16/0.8/32/512; FP mlp[-1]: 256, 256, 128, 128.
  MSG (cfg5)       pointnet2_cls_msg.py:27-28 (as pointnet2_sem_seg_features.py's MSG variant):
      SA1 512, r {0.1,0.2,0.4}, ns {16,32,128}; SA2 128, r {0.2,0.4,0.8}, ns {32,64,128}.

The dense MLPs between the geometric ops are not part of the hot path: their
outputs are replaced by fixed synthetic U[-1,1) tensors of the right shapes, prepared before
the timed region. One "step" runs every geometric op of every layer for the whole batch:
FPS (+gather), ball query, fused group/centre/concat, the attention reduction (cfg3), and
three_nn + IDW + three_interpolate + concat of every FP layer.
"""
import torch

from . import attention_layer, pointnet_util, synth, tf_grouping, tf_sampling

SSG_SA = ((1024, 0.1, 32, 64), (256, 0.2, 32, 128), (64, 0.4, 32, 256), (16, 0.8, 32, 512))
SSG_FP_OUT = (256, 256, 128, 128)
MSG_SA = ((512, (0.1, 0.2, 0.4), (16, 32, 128), (64, 128, 128)),
          (128, (0.2, 0.4, 0.8), (32, 64, 128), (128, 256, 256)))

CONFIGS = {
    # name: (points per cloud, kind, with_features, attention)
    "cfg2": (8192, "ssg", False, False),
    "cfg3": (8192, "ssg", True, True),
    "cfg5": (16384, "msg", False, False),
}


def _rand(gen, shape, device):
    return (torch.rand(shape, generator=gen, device=device, dtype=torch.float32) * 2.0 - 1.0)


def make_inputs(config, cloud_ids, device, seed=1234):
    """Resident inputs of one step: the synthetic ScanNet crops and the stand-in MLP outputs."""
    N, kind, with_feat, attn = CONFIGS[config]
    B = len(cloud_ids)
    xyz, feats = synth.batch(cloud_ids, N, "scannet", with_features=with_feat)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed + int(cloud_ids[0]))
    inp = {"config": config, "B": B, "N": N,
           "xyz": torch.from_numpy(xyz).to(device),
           "feats": torch.from_numpy(feats).to(device) if feats is not None else None}
    if kind == "ssg":
        inp["sa_out"] = [_rand(gen, (B, npt, c), device) for (npt, _, _, c) in SSG_SA]
        n_fp = [SSG_SA[2][0], SSG_SA[1][0], SSG_SA[0][0]]  # FP1..3 output point counts
        inp["fp_out"] = [_rand(gen, (B, n, c), device) for n, c in zip(n_fp, SSG_FP_OUT[:3])]
        if attn:
            inp["attn"] = [(_rand(gen, (B, npt, c), device), _rand(gen, (B, npt, ns, c), device),
                            _rand(gen, (B, npt, ns, c), device)) for (npt, _, ns, c) in SSG_SA]
    else:
        inp["sa_out"] = [_rand(gen, (B, MSG_SA[0][0], sum(MSG_SA[0][3])), device)]
    return inp


def run_ssg(inp, fps_events=None):
    """One step of the SSG SA x4 + FP x4 geometry. fps_events = (start, end) CUDA events
    recorded around the SA1 sampler (the dominant kernel) when given."""
    xyz = [inp["xyz"]]
    points = [inp["feats"]]  # l0_points: None (cfg2) or rgb+normals (cfg3)
    outs = []
    for i, (npoint, radius, nsample, _) in enumerate(SSG_SA):
        if i == 0 and fps_events is not None:
            fps_events[0].record()
        _, new_xyz = tf_sampling.farthest_point_sample_and_gather(npoint, xyz[-1])
        if i == 0 and fps_events is not None:
            fps_events[1].record()
        idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz[-1], new_xyz)
        new_points, _ = pointnet_util.group_concat(xyz[-1], points[-1], new_xyz, idx,
                                                   want_grouped_xyz=False)
        outs.append(new_points)
        if "attn" in inp:  # attention instead of pooling (attention_layer.py:256-261)
            Q, K, V = inp["attn"][i]
            outs.append(attention_layer.attention_reduce(Q, K, V))
        xyz.append(new_xyz)
        points.append(inp["sa_out"][i])  # stand-in for the SA MLP output (l{i+1}_points)
    # FP layers (pointnet2_sem_seg_attention.py:46-53)
    feat = inp["sa_out"][3]  # l4_points
    for k in range(4):
        lvl = 3 - k  # interpolate level lvl+1 -> lvl
        out = pointnet_util.fp_interpolate(xyz[lvl], xyz[lvl + 1], points[lvl], feat)
        outs.append(out)
        feat = inp["fp_out"][k] if k < 3 else None  # stand-in for the FP MLP output
    return outs


def run_msg(inp, fps_events=None):
    """One step of the MSG SA1 + SA2 grouping geometry (cfg5)."""
    xyz, points = inp["xyz"], None
    outs = []
    for i, (npoint, radii, nsamples, _) in enumerate(MSG_SA):
        if i == 0 and fps_events is not None:
            fps_events[0].record()
        _, new_xyz = tf_sampling.farthest_point_sample_and_gather(npoint, xyz)
        if i == 0 and fps_events is not None:
            fps_events[1].record()
        for radius, nsample in zip(radii, nsamples):
            idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz)
            gp, _ = pointnet_util.group_concat(xyz, points, new_xyz, idx, xyz_last=True,
                                               want_grouped_xyz=False)
            outs.append(gp)
        xyz, points = new_xyz, inp["sa_out"][0]
    return outs


def run(inp, fps_events=None):
    kind = CONFIGS[inp["config"]][1]
    return run_ssg(inp, fps_events) if kind == "ssg" else run_msg(inp, fps_events)


def sa_fp_bytes(config, B):
    """Algorithmic HBM bytes of one step (each input read once, each output written once),
    per op as SURVEY.md §8(d) counts them, plus what this step also does: the FP concat of
    points1 and, for cfg3, the attention reduction. Returns {op: bytes}."""
    N, kind, with_feat, attn = CONFIGS[config]
    by = {"fps": 0, "gather": 0, "ball_query": 0, "group": 0, "attention": 0, "three_nn": 0,
          "interpolate": 0, "fp_concat": 0}

    def sa(Nin, M, ns, C):
        by["fps"] += Nin * 12 + M * 4
        by["gather"] += M * 4 + Nin * 12 + M * 12
        by["ball_query"] += Nin * 12 + M * 12 + M * ns * 4 + M * 4
        by["group"] += M * ns * 4 + Nin * (3 + C) * 4 + M * 12 + M * ns * (3 + C) * 4

    if kind == "ssg":
        n_in, c_in = N, (6 if with_feat else 0)
        for (M, _, ns, c_out) in SSG_SA:
            sa(n_in, M, ns, c_in)
            if attn:
                by["attention"] += M * c_out * 4 + 2 * M * ns * c_out * 4 + M * c_out * 4
            n_in, c_in = M, c_out
        levels = [N] + [s[0] for s in SSG_SA]
        chans = [6 if with_feat else 0] + [s[3] for s in SSG_SA]
        c2 = SSG_SA[3][3]
        for k in range(4):
            lvl = 3 - k
            n, m, c1 = levels[lvl], levels[lvl + 1], chans[lvl]
            by["three_nn"] += n * 12 + m * 12 + n * 24
            by["interpolate"] += n * 24 + m * c2 * 4 + n * c2 * 4
            by["fp_concat"] += 2 * n * c1 * 4
            c2 = SSG_FP_OUT[k]
    else:
        n_in, c_in = N, 0
        for (M, radii, nss, couts) in MSG_SA:
            by["fps"] += n_in * 12 + M * 4
            by["gather"] += M * 4 + n_in * 12 + M * 12
            for ns in nss:
                by["ball_query"] += n_in * 12 + M * 12 + M * ns * 4 + M * 4
                by["group"] += M * ns * 4 + n_in * (3 + c_in) * 4 + M * 12 + M * ns * (3 + c_in) * 4
            n_in, c_in = M, sum(couts)
    return {k: v * B for k, v in by.items()}
