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


def _rand_per_cloud(cloud_ids, shape, device, seed, slot):
    """U[-1,1) stand-in tensor (B, *shape) whose row b depends only on the GLOBAL cloud id
    cloud_ids[b] (and the tensor's slot), so a rank's shard of a global batch gets exactly the
    values the same clouds get in a single-process run."""
    rows = []
    for cid in cloud_ids:
        gen = torch.Generator(device=device)
        gen.manual_seed(seed * 1_000_003 + int(cid) * 1009 + slot)
        rows.append(torch.rand(shape, generator=gen, device=device, dtype=torch.float32))
    return torch.stack(rows) * 2.0 - 1.0


def make_inputs(config, cloud_ids, device, seed=1234):
    """Resident inputs of one step: the synthetic ScanNet crops and the stand-in MLP outputs."""
    N, kind, with_feat, attn = CONFIGS[config]
    B = len(cloud_ids)
    xyz, feats = synth.batch(cloud_ids, N, "scannet", with_features=with_feat)
    inp = {"config": config, "B": B, "N": N,
           "xyz": torch.from_numpy(xyz).to(device),
           "feats": torch.from_numpy(feats).to(device) if feats is not None else None}
    r = lambda shape, slot: _rand_per_cloud(cloud_ids, shape, device, seed, slot)  # noqa: E731
    if kind == "ssg":
        inp["sa_out"] = [r((npt, c), i) for i, (npt, _, _, c) in enumerate(SSG_SA)]
        n_fp = [SSG_SA[2][0], SSG_SA[1][0], SSG_SA[0][0]]  # FP1..3 output point counts
        inp["fp_out"] = [r((n, c), 10 + i) for i, (n, c) in enumerate(zip(n_fp, SSG_FP_OUT[:3]))]
        if attn:
            inp["attn"] = [(r((npt, c), 20 + 3 * i), r((npt, ns, c), 21 + 3 * i),
                            r((npt, ns, c), 22 + 3 * i)) for i, (npt, _, ns, c) in enumerate(SSG_SA)]
    else:
        inp["sa_out"] = [r((MSG_SA[0][0], sum(MSG_SA[0][3])), 0)]
    return inp


class Step:
    """One benchmark step, split in two phases so that the dominant kernel (the SA1 sampler)
    can be timed on its own: sampler() runs FPS + gather of the first SA layer, rest() runs
    everything after it and returns the step's outputs. __call__ runs both.

    The samplers of SA2..SA4 form a serial chain (each samples the previous layer's output)
    that keeps only B workgroups busy, so with overlap=True (default) rest() runs that chain
    on the current stream and forks everything that hangs off it onto a side stream:
    layer i's ball query / grouping / attention and the FP layer that interpolates onto
    level i-1 start as soon as sampler i has finished (one event per layer) and run
    concurrently with samplers i+1.. . The side stream joins back before rest() returns, so
    the caller sees one ordered stream (and hipGraph capture records the fork/join).
    Intermediates live on self for the life of the step: nothing made on one stream is freed
    while the other may still read it."""

    def __init__(self, inp, overlap=True):
        self.inp = inp
        self.kind = CONFIGS[inp["config"]][1]
        self.new_xyz1 = None
        self.overlap = overlap and inp["xyz"].is_cuda
        if self.overlap:
            self.side = torch.cuda.Stream(device=inp["xyz"].device)
            self.ready = [torch.cuda.Event() for _ in range(4)]
        self.keep = []

    def sampler(self):
        """SA1 FPS + gather. With overlap, the SA1 ball-query grid over the input cloud is
        built on the side stream meanwhile (it needs only xyz) and joined before returning."""
        npoint = SSG_SA[0][0] if self.kind == "ssg" else MSG_SA[0][0]
        xyz = self.inp["xyz"]
        self.grid1 = None
        build = (self.overlap and self.kind == "ssg"
                 and int(xyz.shape[1]) >= tf_grouping.GRID_MIN_POINTS)
        if build:
            main = torch.cuda.current_stream(xyz.device)
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                self.grid1 = tf_grouping.BallGrid(xyz, SSG_SA[0][1])
        _, self.new_xyz1 = tf_sampling.farthest_point_sample_and_gather(npoint, xyz)
        if build:
            main.wait_stream(self.side)
        return self.new_xyz1

    def rest(self):
        return self._rest_ssg() if self.kind == "ssg" else self._rest_msg()

    def __call__(self):
        self.sampler()
        return self.rest()

    def _fork(self, layer):
        """Context for layer `layer`'s dependent work: the side stream after sampler `layer`."""
        if not self.overlap:
            return _Same()
        main = torch.cuda.current_stream(self.inp["xyz"].device)
        self.ready[layer].record(main)
        self.side.wait_event(self.ready[layer])
        return torch.cuda.stream(self.side)

    def _join(self, outs):
        if self.overlap:
            main = torch.cuda.current_stream(self.inp["xyz"].device)
            main.wait_stream(self.side)
            if not torch.cuda.is_current_stream_capturing():
                for t in outs:  # made on the side stream, consumed on main from here on
                    t.record_stream(main)
        return outs

    def _rest_ssg(self):
        inp = self.inp
        xyz = [inp["xyz"], self.new_xyz1]
        points = [inp["feats"]] + list(inp["sa_out"])  # l0 = None (cfg2) / rgb+normals (cfg3)
        # FP layer k interpolates level lvl+1 onto lvl (pointnet2_sem_seg_attention.py:46-53);
        # level lvl+1's features are the SA4 output (k=0) or the previous FP MLP's stand-in.
        fp_feat = [inp["sa_out"][3]] + list(inp["fp_out"])
        sa_outs, fp_outs = [None] * 4, [None] * 4
        for i, (npoint, radius, nsample, _) in enumerate(SSG_SA):
            if i > 0:
                xyz.append(tf_sampling.farthest_point_sample_and_gather(npoint, xyz[i])[1])
            with self._fork(i):
                new_xyz = xyz[i + 1]
                idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz[i], new_xyz,
                                                      grid=self.grid1 if i == 0 else None)
                new_points, _ = pointnet_util.group_concat(xyz[i], points[i], new_xyz, idx,
                                                           want_grouped_xyz=False)
                sa_outs[i] = [new_points]
                if "attn" in inp:  # attention instead of pooling (attention_layer.py:256-261)
                    Q, K, V = inp["attn"][i]
                    sa_outs[i].append(attention_layer.attention_reduce(Q, K, V))
                k = 3 - i  # the FP layer whose coarse level (i+1) just became available
                # FP4's unknown points are SA1's input cloud: the SA1 grid orders its search
                fp_outs[k] = pointnet_util.fp_interpolate(
                    xyz[i], xyz[i + 1], points[i], fp_feat[k],
                    unknown_grid=self.grid1 if i == 0 else None)
        self.keep = xyz
        return self._join([t for o in sa_outs for t in o] + fp_outs)

    def _rest_msg(self):
        inp = self.inp
        xyz, points, new_xyz = inp["xyz"], None, self.new_xyz1
        outs = []
        kept = [new_xyz]
        for i, (npoint, radii, nsamples, _) in enumerate(MSG_SA):
            if i > 0:
                _, new_xyz = tf_sampling.farthest_point_sample_and_gather(npoint, xyz)
                kept.append(new_xyz)
            with self._fork(i):
                for radius, nsample in zip(radii, nsamples):
                    idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz)
                    gp, _ = pointnet_util.group_concat(xyz, points, new_xyz, idx, xyz_last=True,
                                                       want_grouped_xyz=False)
                    outs.append(gp)
            xyz, points = new_xyz, inp["sa_out"][0]
        self.keep = kept
        return self._join(outs)


class _Same:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def run(inp):
    """One step of the configured SA + FP geometry (eager)."""
    return Step(inp)()


class GraphStep:
    """The step captured as two hipGraphs (sampler, rest) sharing one memory pool; replay()
    launches both on the current stream. Inputs stay resident, outputs are overwritten in
    place at every replay."""

    def __init__(self, inp, warmup=2, overlap=True):
        self.step = Step(inp, overlap=overlap)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.step()
        torch.cuda.current_stream().wait_stream(side)
        self.g_sampler = torch.cuda.CUDAGraph()
        self.g_rest = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_sampler):
            self.step.sampler()
        with torch.cuda.graph(self.g_rest, pool=self.g_sampler.pool()):
            self.outs = self.step.rest()

    def replay(self, sampler_events=None):
        if sampler_events is not None:
            sampler_events[0].record()
        self.g_sampler.replay()
        if sampler_events is not None:
            sampler_events[1].record()
        self.g_rest.replay()
        return self.outs


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
