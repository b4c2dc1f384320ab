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

With model=True (make_inputs) the step is instead the whole inference forward pass of
pointnet2_sem_seg.py:19-61 (cfg3: with rgb+normals and the attention SA layers of
pointnet2_sem_seg_attention.py): every
SA layer as one fused group + MLP + max-pool kernel fed by the previous layer's real output,
every FP layer as one fused interpolation + MLP kernel, and the conv1d head (fc1 with batch
norm, dropout = identity at inference, fc2 to 21 classes) fused into FP4's MLP. Weights are
the reference initialisers (tf_util.ParamStore, fixed seed).
"""
import math
import os
import time

import torch

from . import attention_layer, grid, pointnet_util, synth, tf_grouping, tf_interpolate, \
    tf_sampling, tf_util

SSG_SA = ((1024, 0.1, 32, 64), (256, 0.2, 32, 128), (64, 0.4, 32, 256), (16, 0.8, 32, 512))
SSG_FP_OUT = (256, 256, 128, 128)
MSG_SA = ((512, (0.1, 0.2, 0.4), (16, 32, 128), (64, 128, 128)),
          (128, (0.2, 0.4, 0.8), (32, 64, 128), (128, 256, 256)))
# the full model's MLP widths (pointnet2_sem_seg.py:29-60)
SSG_SA_MLP = ((32, 32, 64), (64, 64, 128), (128, 128, 256), (256, 256, 512))
SSG_FP_MLP = ((256, 256), (256, 256), (256, 128), (128, 128, 128))
NUM_CLASSES = 21  # ScanNet (pointnet2_sem_seg_attention.py:17)
# cell edge of the one grid that serves all of MSG SA1's radii (tools/bench_msg_grid.py)
MSG_GRID_EDGE = 0.2  # 105 us for the three radii vs 110 at 0.1, 122 at 0.4 (profiles/r4/ab2)

# FP4's known points (SA1's picks) gridded once per cloud instead of inside each of FP4's
# workgroups (pn2_fp_grid_fused_known): "lane" = a grid build launch before FP4 on its lane,
# "sampler" = by the SA1 sampler's own workgroups after the last pick (pn2_fps_chain_grid),
# "off" = each FP4 workgroup sorts them in LDS (pn2_fp_grid_fused). None = per config
# (FP4_KNOWN_GRID_BY_CONFIG, else "off"): the 500-step A/B (profiles/r5/kgrid2) gave cfg3
# 60.6-60.8k with "lane" against 57.6-57.7k "off" (58.8k "sampler"), cfg2 87.2-87.4k "lane",
# 87.9-88.4k "sampler", 88.5k "off". Round 6 (FP4 fused 42.4 us alone, 35.5 over a known grid;
# profiles/r6/kg, kg20): cfg2 at 500 steps "sampler" 89.3 / 88.7k against "off" 87.5 / 87.2k,
# the driver's 20-step window 77.5 / 72.0 / 82.4k against 74.4 / 72.7 / 71.1k; cfg3 "lane"
# 58.4 / 57.9 / 58.5k, "sampler" 57.2 / 56.7 / 58.5k, "off" 56.3-56.5k. bench.py
# --fp4-known-grid overrides it.
FP4_KNOWN_GRID = None
FP4_KNOWN_GRID_BY_CONFIG = {"cfg2": "sampler", "cfg3": "lane"}

NSIDE = 4  # side streams of the whole-model step (the geometric steps use 3)
MAX_LANES = 8  # lanes of any step layout (0 = the sampler stream)

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


class SemSegModel:
    """The packed MLPs of pointnet2_sem_seg(_features) (pointnet2_sem_seg.py:29-60) under the
    reference's variable scopes: layer1..4/conv<j>, fa_layer1..4/conv_<j>, fc1, fc2. FP4's
    MLP carries the head: fa_layer4's three layers, then fc1 (128, batch norm, relu) and fc2
    (NUM_CLASSES, no batch norm, no activation) as the 4th and 5th layers of ONE kernel.
    attention=True: the SA layers of pointnet2_sem_seg_attention.py:27-42
    (pointnet_sa_module_attention: attention + batch norm instead of max pooling)."""

    def __init__(self, in_channels, params=None, device="cuda", attention=False):
        self.attention = attention
        self.store = params if params is not None else tf_util.ParamStore(seed=7, device=device)
        st = self.store
        self.sa, c = [], in_channels
        for i, widths in enumerate(SSG_SA_MLP):
            self.sa.append(tf_util.packed_mlp(st, [f"layer{i + 1}/conv{j}" for j in range(3)],
                                              c + 3, widths))
            c = widths[-1]
        levels_c = [in_channels] + [w[-1] for w in SSG_SA_MLP]
        self.fp, c2 = [], SSG_SA_MLP[3][-1]
        for k, widths in enumerate(SSG_FP_MLP):
            cin = c2 + levels_c[3 - k]
            scopes = [f"fa_layer{k + 1}/conv_{j}" for j in range(len(widths))]
            layers = tf_util.packed_mlp(st, scopes, cin, widths).layers
            if k == 3:  # + the conv1d head (pointnet2_sem_seg.py:57-60)
                head1 = tf_util.packed_mlp(st, ["fc1"], widths[-1], [128]).layers
                head2 = tf_util.packed_mlp(st, ["fc2"], 128, [NUM_CLASSES], bn=False,
                                           relu=False).layers
                layers = layers + head1 + head2
            self.fp.append(tf_util.SharedMLP(layers))
            c2 = widths[-1]
        if attention:  # pack the Dense / batch-norm variables up front (not inside a capture)
            for i, widths in enumerate(SSG_SA_MLP):
                C, sc = widths[-1], f"layer{i + 1}"
                for d in attention_layer._attention_scopes(sc):
                    tf_util.packed_dense(st, d, C, C)
                tf_util.bn_affine(st, f"{sc}/{sc}", C, device)


def make_inputs(config, cloud_ids, device, seed=1234, model=False):
    """Resident inputs of one step: the synthetic ScanNet crops and the stand-in MLP outputs
    (or, with model=True, the packed weights of the whole segmentation model)."""
    N, kind, with_feat, attn = CONFIGS[config]
    B = len(cloud_ids)
    xyz, feats = synth.batch(cloud_ids, N, "scannet", with_features=with_feat)
    inp = {"config": config, "B": B, "N": N,
           "xyz": torch.from_numpy(xyz).to(device),
           "feats": torch.from_numpy(feats).to(device) if feats is not None else None}
    if model:
        if kind != "ssg":
            raise NotImplementedError("model=True: the SSG segmentation model (cfg2 / cfg3)")
        inp["model"] = SemSegModel(6 if with_feat else 0, device=device, attention=attn)
        return inp
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


_SIDE = {}
# lane-end events with timing (DIAGNOSTIC: bench.py --timeline sets it before the pipeline)
TIMING_EVENTS = False


def side_stream(dev, lane):
    """The process-wide side stream of `lane` on `dev`: every Step shares them, so the
    sampler chain (the current stream) and the side lanes stay on distinct hardware queues
    (HIP gives each new stream a new hardware queue up to GPU_MAX_HW_QUEUES, then shares the
    least-used ones): the first Step creates lanes 1-3 before any other stream exists."""
    key = (str(dev), lane)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


SIDE_LAYOUTS = ("a", "b", "c", "d")


def side_layout(multi, attention, layout="a"):
    """Side lanes of the SSG geometric step's later SA layers (sa234) and first three FP layers
    (fp123); SA1 (with the grid) stays on lane 1, FP4 on lane 2, the attention reductions of
    the multi-sampler layout on lane 3. Without several sampler streams: lanes 1 and 2.
    With them: a = lanes 1 and 2; b = FP1-3 on a lane of their own; c = SA2-4 on a lane of
    their own; d = both (measured: DESIGN.md §3.6)."""
    if layout not in SIDE_LAYOUTS:
        raise ValueError(f"side layout {layout!r}: one of {SIDE_LAYOUTS}")
    if not multi:
        return {"sa234": 1, "fp123": 2}
    nxt = 4 if attention else 3
    return {"a": {"sa234": 1, "fp123": 2}, "b": {"sa234": 1, "fp123": nxt},
            "c": {"sa234": nxt, "fp123": 2}, "d": {"sa234": nxt, "fp123": nxt + 1}}[layout]


class Task:
    """One piece of a step: `fn` runs on stream `lane` (0 = the sampler chain, 1.. = side
    streams) after the tasks named in `deps` (same-lane order is implicit)."""

    def __init__(self, name, lane, deps, fn, direct=False, chain=None):
        self.name, self.lane, self.deps, self.fn = name, lane, tuple(deps), fn
        # direct: one C launch into fixed buffers; GraphStep launches it as is (a one-kernel
        # graph costs more queue time than the kernel launch itself)
        self.direct = direct
        # chain: (npoints, xyz, outs) of a direct sampler launch (pn2_fps_chain into fixed
        # buffers), so a native plan can record the same launch (Step.emit_plan)
        self.chain = chain


class Step:
    """One benchmark step as a list of tasks over streams.

    The FPS samplers form a serial chain (each samples the previous layer's output) that
    keeps only B workgroups busy. The SA1 sampler (~85 % of the chain) runs on lane 0 with
    nothing else in its way; SA2..SA4's samplers run fused on lane 3, so with pipelining the
    next step's SA1 sampler follows this one back to back. Everything that hangs off sampler
    i -- layer i's ball query / grouping / attention (lane 1) and the FP layer that
    interpolates onto level i-1 (lane 2; MSG: radius 0 on lane 1, the others on lane 2) --
    waits for that sampler only and runs concurrently with the samplers after it and with
    each other. Three side lanes: with the current stream that is one stream per hardware
    queue of the box (GPU_MAX_HW_QUEUES = 4); a fourth side lane shared a queue with lane 1
    and serialised the FPS chain behind cfg3's attention.
    The SA1 ball-query grid needs only the input cloud and is built on lane 1 while SA1 is
    sampled. Lanes join lane 0 at the end of the step.

    With overlap=False every task runs in order on the current stream (lanes collapse).
    run() executes the tasks eagerly; GraphStep captures one hipGraph per task and replays
    them with the same cross-stream events, so the graph executor never reorders the chain
    behind side work. `sampler_events` brackets the SA1 sampler task (bench.py's roofline).
    Intermediates live on self for the life of the step."""

    SAMPLER = "fps1"

    def __init__(self, inp, overlap=True, streams=None, chain_lane=3, layout="a"):
        # chain_lane: the lane of the later samplers (SA2..SA4 / MSG SA2); 0 = behind the SA1
        # sampler on its stream; -1 = a lane of their own after the side lanes (both: several
        # sampler streams, Pipeline); layout: side_layout()
        self.chain_lane = chain_lane if overlap else 0
        self.layout = layout
        self.inp = inp
        self.kind = CONFIGS[inp["config"]][1]
        self.overlap = overlap and inp["xyz"].is_cuda
        self.v = {}  # intermediates by name
        if "model" in inp:
            self.tasks = self._tasks_ssg_model()
        else:
            self.tasks = self._tasks_ssg() if self.kind == "ssg" else self._tasks_msg()
        self.ran = False
        self.synced_inputs = False
        self.nlanes = 1 + max(t.lane for t in self.tasks)
        if self.overlap:
            dev = inp["xyz"].device
            if streams and len(streams) < self.nlanes:
                raise ValueError(f"this step layout uses {self.nlanes} lanes, {len(streams)} "
                                 "streams given")
            self.streams = [None] + (list(streams[1:self.nlanes]) if streams else
                                     [side_stream(dev, lane) for lane in range(1, self.nlanes)])
            # HIP binds a stream to a hardware queue when the stream is first used: use the
            # lanes now, in order, so that they (not the warm-up or capture streams made later)
            # get the queues the current stream does not hold
            main = torch.cuda.current_stream(dev)
            for st in self.streams[1:]:
                st.wait_stream(main)
            self.done = {t.name: torch.cuda.Event() for t in self.tasks}
            # (timing-enabled under bench.py --timeline, which reads their GPU times)
            self.lane_done = [torch.cuda.Event(enable_timing=TIMING_EVENTS)
                              for _ in range(self.nlanes)]

    # ------------------------------------------------------------------ task lists
    def _tasks_ssg(self):
        inp, v = self.inp, self.v
        big = int(inp["xyz"].shape[1]) >= tf_grouping.GRID_MIN_POINTS
        points = [inp["feats"]] + list(inp["sa_out"])  # l0 = None (cfg2) / rgb+normals (cfg3)
        # FP layer k interpolates level lvl+1 onto lvl (pointnet2_sem_seg_attention.py:46-53);
        # level lvl+1's features are the SA4 output (k=0) or the previous FP MLP's stand-in.
        fp_feat = [inp["sa_out"][3]] + list(inp["fp_out"])
        v["xyz"] = [inp["xyz"], None, None, None, None]
        v["sa"], v["fp"], v["att"] = [None] * 4, [None] * 4, [None] * 4
        v["bq"], v["nn"] = [None] * 4, [None] * 4  # kept for the parity tests (intermediates())
        # with the later samplers behind SA1 on its stream (chain_lane 0: several sampler
        # streams), lane 3 is free: the attention reductions (they read only their resident
        # inputs) run there instead of inside lane 1's SA tasks
        multi = self.chain_lane <= 0 and self.overlap
        attn_lane = 3 if (multi and "attn" in inp) else None
        lane = side_layout(multi, attn_lane is not None, self.layout)
        chain_lane = self.chain_lane
        if chain_lane < 0:  # the later samplers on a lane after every side lane (-1: the
            # first such lane, -2: the second, ... -- Pipeline's chain_streams)
            chain_lane = max([2] + list(lane.values()) + ([attn_lane] if attn_lane else [])) \
                - chain_lane
        tasks = []
        if big:  # the SA1 grid over the input cloud (also orders FP4's neighbour search)
            tasks.append(Task("grid1", 1, (), lambda: v.__setitem__(
                "grid1", tf_grouping.BallGrid(inp["xyz"], SSG_SA[0][1]))))

        def fps(i):
            def f():
                v["xyz"][i + 1] = tf_sampling.farthest_point_sample_and_gather(
                    SSG_SA[i][0], v["xyz"][i])[1]
            return f

        def sa(i):
            def f():
                _, radius, nsample, _ = SSG_SA[i]
                xyz, new_xyz = v["xyz"][i], v["xyz"][i + 1]
                if i == 0 and v.get("grid1") is not None:
                    # SA1 (cfg2 xyz only, cfg3 with rgb + normals): query and grouping in one
                    # kernel over the grid
                    idx, _, new_points = pointnet_util.ball_group(radius, nsample, xyz,
                                                                  points[0], new_xyz, v["grid1"])
                else:
                    idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz,
                                                          grid=v.get("grid1") if i == 0 else None)
                    new_points, _ = pointnet_util.group_concat(xyz, points[i], new_xyz, idx,
                                                               want_grouped_xyz=False)
                v["bq"][i] = idx
                v["sa"][i] = new_points
                if "attn" in inp and attn_lane is None:
                    att(i)()
            return f

        def att(i):  # attention instead of pooling (attention_layer.py:256-261)
            def f():
                v["att"][i] = attention_layer.attention_reduce(*inp["attn"][i])
            return f

        def fp(i):
            def f():
                k = 3 - i  # the FP layer whose coarse level (i+1) just became available
                if i == 0 and v.get("kgrid") is not None and v["kgrid_mode"] == "lane":
                    v["kgrid"].rebuild()
                v["fp"][k], v["nn"][k] = pointnet_util.fp_interpolate(
                    v["xyz"][i], v["xyz"][i + 1], points[i], fp_feat[k],
                    known_grid=v.get("kgrid") if i == 0 else None,
                    unknown_grid=v.get("grid1") if i == 0 else None, return_nn=True)
            return f

        npoints = [sa_[0] for sa_ in SSG_SA]
        grid_dep = ("grid1",) if big else ()
        if tf_sampling.chain_supported(int(inp["xyz"].shape[1]), npoints):
            # lane 0: the four samplers as ONE launch (pn2_fps_chain; what bench.py times)
            xyz = inp["xyz"]
            B = int(xyz.shape[0])
            v["chain"] = [(torch.empty((B, m), dtype=torch.int32, device=xyz.device),
                           torch.empty((B, m, 3), dtype=torch.float32, device=xyz.device))
                          for m in npoints]
            for i, (_, nx) in enumerate(v["chain"]):
                v["xyz"][i + 1] = nx
            # FP4's known points (SA1's picks) gridded by the SA1 sampler's own workgroups
            # after the last pick (pn2_fps_chain_grid), not by each FP4 workgroup again
            kgrid = None
            mode = FP4_KNOWN_GRID or FP4_KNOWN_GRID_BY_CONFIG.get(inp["config"], "off")
            v["kgrid_mode"] = mode
            if mode != "off" and big and xyz.is_cuda and tf_interpolate.use_grid(
                    int(xyz.shape[1]), npoints[0]) and npoints[0] <= pointnet_util.FP_GRID_MAX_KNOWN:
                v["kgrid"] = grid.PointGrid(v["chain"][0][1], build=False)
                if mode == "sampler":
                    kgrid = v["kgrid"]

            # lane 0: SA1's sampler alone (bench.py times it); lane 4: SA2..SA4's samplers
            # fused in one launch, so the next step's SA1 sampler follows this one directly.
            # Both are direct launches into fixed buffers.
            tasks.append(Task("fps1", 0, (), lambda: tf_sampling.farthest_point_sample_chain(
                npoints[:1], xyz, out=v["chain"][:1], grid0=kgrid), direct=True,
                chain=(npoints[:1], xyz, v["chain"][:1], kgrid)))
            tasks.append(Task("fps234", chain_lane, ("fps1",), lambda: tf_sampling.farthest_point_sample_chain(
                npoints[1:], v["xyz"][1], out=v["chain"][1:]), direct=True,
                chain=(npoints[1:], v["xyz"][1], v["chain"][1:])))
            sampled = ("fps1", "fps234", "fps234", "fps234")
        else:
            # lane 0: SA1's sampler alone; lane 3: SA2..SA4's samplers as one task
            tasks.append(Task("fps1", 0, (), fps(0)))
            tasks.append(Task("fps234", chain_lane, ("fps1",), lambda: [fps(i)() for i in (1, 2, 3)]))
            sampled = ("fps1", "fps234", "fps234", "fps234")
        tasks.append(Task("sa1", 1, (sampled[0],), sa(0)))
        tasks.append(Task("fp4", 2, (sampled[0],) + grid_dep, fp(0)))
        if npoints[0] <= pointnet_util.BALL_GROUP_MAX_POINTS and sampled[1:] == ("fps234",) * 3:
            # SA2..SA4 wait for the same sampler launch: their three ball queries and groupings
            # run as ONE kernel (pn2_ball_group_layers) instead of six launches on the lane
            def sa234():
                specs = [(SSG_SA[i][1], SSG_SA[i][2], v["xyz"][i], points[i], v["xyz"][i + 1])
                         for i in (1, 2, 3)]
                for i, (idx, _, new_points) in zip((1, 2, 3),
                                                   pointnet_util.ball_group_layers(specs)):
                    v["bq"][i], v["sa"][i] = idx, new_points
                if "attn" in inp and attn_lane is None:
                    for i in (1, 2, 3):
                        att(i)()
            tasks.append(Task("sa234", lane["sa234"], (sampled[1],), sa234))
        else:
            for i in (1, 2, 3):
                tasks.append(Task(f"sa{i + 1}", lane["sa234"], (sampled[i],), sa(i)))
        small = [not tf_interpolate.use_grid(SSG_SA[i - 1][0] if i else int(inp["xyz"].shape[1]),
                                             SSG_SA[i][0]) for i in (1, 2, 3)]
        if all(small) and sampled[1:] == ("fps234",) * 3:
            # FP3, FP2, FP1 wait for the same sampler launch: one kernel (pn2_fp_fused_layers)
            def fp123():
                outs = pointnet_util.fp_interpolate_layers(
                    [(v["xyz"][i], v["xyz"][i + 1], points[i], fp_feat[3 - i]) for i in (1, 2, 3)])
                for i, o in zip((1, 2, 3), outs):
                    v["fp"][3 - i], v["nn"][3 - i] = o, None
            tasks.append(Task("fp123", lane["fp123"], (sampled[1],), fp123))
        else:
            tasks.append(Task("fp3", lane["fp123"], (sampled[1],), fp(1)))
            tasks.append(Task("fp2", lane["fp123"], (sampled[2],), fp(2)))
            tasks.append(Task("fp1", lane["fp123"], (sampled[3],), fp(3)))
        if attn_lane is not None:
            # the four reductions as ONE launch (pn2_attn_reduce_layers): they read only their
            # resident inputs and share nsample
            def att_all():
                for i, o in enumerate(attention_layer.attention_reduce_layers(inp["attn"])):
                    v["att"][i] = o
            tasks.append(Task("att", attn_lane, (), att_all))
        return tasks

    def _tasks_ssg_model(self):
        """The whole inference forward of the SSG segmentation model. Lane 0: SA1's sampler;
        lane 4: SA2..SA4's samplers; lanes 2-3: the FP layers' neighbour searches (they need
        only the sampled coordinates); lane 1: the data-dependent chain SA1 -> SA4 -> FP1 ->
        FP4+head, each layer one fused kernel (plus the ball query before each SA)."""
        inp, v, mdl = self.inp, self.v, self.inp["model"]
        xyz0 = inp["xyz"]
        B = int(xyz0.shape[0])
        npoints = [sa_[0] for sa_ in SSG_SA]
        if not tf_sampling.chain_supported(int(xyz0.shape[1]), npoints):
            raise NotImplementedError("model step: the fused sampler chain's cloud sizes")
        big = int(xyz0.shape[1]) >= tf_grouping.GRID_MIN_POINTS
        v["chain"] = [(torch.empty((B, m), dtype=torch.int32, device=xyz0.device),
                       torch.empty((B, m, 3), dtype=torch.float32, device=xyz0.device))
                      for m in npoints]
        v["xyz"] = [xyz0] + [nx for _, nx in v["chain"]]
        v["pts"] = [inp["feats"], None, None, None, None]
        v["nn"], v["fp"] = [None] * 4, [None] * 4
        tasks = []
        if big:  # on a search lane (lane 1 carries the MLPs only)
            tasks.append(Task("grid1", 2, (), lambda: v.__setitem__(
                "grid1", tf_grouping.BallGrid(xyz0, SSG_SA[0][1]))))
        tasks.append(Task("fps1", 0, (), lambda: tf_sampling.farthest_point_sample_chain(
            npoints[:1], xyz0, out=v["chain"][:1]), direct=True,
            chain=(npoints[:1], xyz0, v["chain"][:1])))
        tasks.append(Task("fps234", 4, ("fps1",), lambda: tf_sampling.farthest_point_sample_chain(
            npoints[1:], v["xyz"][1], out=v["chain"][1:]), direct=True,
            chain=(npoints[1:], v["xyz"][1], v["chain"][1:])))
        sampled = ("fps1", "fps234", "fps234", "fps234")

        def nn(k):  # FP layer k interpolates level 4-k onto level 3-k
            def f():
                lvl = 3 - k
                v["nn"][k] = tf_interpolate.three_nn(
                    v["xyz"][lvl], v["xyz"][lvl + 1],
                    unknown_grid=v.get("grid1") if lvl == 0 else None)
            return f

        v["bq"] = [None] * 4

        def bq(i):  # layer i's ball query: needs only the sampled coordinates
            def f():
                _, radius, nsample, _ = SSG_SA[i]
                v["bq"][i] = tf_grouping.query_ball_point(
                    radius, nsample, v["xyz"][i], v["xyz"][i + 1],
                    grid=v.get("grid1") if i == 0 else None)[0]
            return f

        def sa(i):
            def f():
                xyz, new_xyz, idx = v["xyz"][i], v["xyz"][i + 1], v["bq"][i]
                if mdl.attention:  # attention + batch norm (attention_layer.py:229-276)
                    v["pts"][i + 1] = attention_layer.group_mlp_attention(
                        xyz, v["pts"][i], new_xyz, idx, mdl.sa[i], mdl.store, f"layer{i + 1}")
                else:
                    v["pts"][i + 1] = pointnet_util.group_mlp(xyz, v["pts"][i], new_xyz, idx,
                                                              mdl.sa[i], "max")
            return f

        def fp(k):
            def f():
                lvl = 3 - k
                p2 = v["pts"][4] if k == 0 else v["fp"][k - 1]
                dist, idx = v["nn"][k]
                v["fp"][k] = pointnet_util.fp_mlp(dist, idx, v["pts"][lvl], p2, mdl.fp[k])
            return f

        grid_dep = ("grid1",) if big else ()
        # the searches (ball queries "bq<i>", FP layer k+1's three_nn "nn<k+1>") need only
        # the sampled coordinates: they run on lanes 2-3, so lane 1 carries the MLP kernels
        # alone (with the queries on it they were ~60 us of its ~810 us per step,
        # profiles/r5/model/lanes_model_cfg2.txt)
        tasks.append(Task("bq1", 2, (sampled[0],) + grid_dep, bq(0)))
        tasks.append(Task("nn4", 2, (sampled[0],) + grid_dep, nn(3)))
        for i in (1, 2, 3):
            tasks.append(Task(f"bq{i + 1}", 3, (sampled[i],), bq(i)))
        tasks.append(Task("nn3", 2, (sampled[1],), nn(2)))
        tasks.append(Task("nn2", 3, (sampled[2],), nn(1)))
        tasks.append(Task("nn1", 3, (sampled[3],), nn(0)))
        for i in range(4):
            tasks.append(Task(f"sa{i + 1}", 1, (f"bq{i + 1}",), sa(i)))
        for k in range(4):
            tasks.append(Task(f"fp{k + 1}", 1, (f"nn{k + 1}",), fp(k)))
        return tasks

    def _tasks_msg(self):
        inp, v = self.inp, self.v
        v["xyz"] = [inp["xyz"], None, None]
        v["gp"], v["bq"] = {}, {}
        tasks = []

        xyz0 = inp["xyz"]
        B = int(xyz0.shape[0])
        # the samplers write into fixed buffers (direct launches, no one-kernel graphs)
        v["fps_out"] = [(torch.empty((B, sa_[0]), dtype=torch.int32, device=xyz0.device),
                         torch.empty((B, sa_[0], 3), dtype=torch.float32, device=xyz0.device))
                        for sa_ in MSG_SA]
        for i, (_, nx) in enumerate(v["fps_out"]):
            v["xyz"][i + 1] = nx

        def fps(i):
            def f():
                tf_sampling.farthest_point_sample_chain([MSG_SA[i][0]], v["xyz"][i],
                                                        out=v["fps_out"][i:i + 1])
            return f

        # the xyz-only level (SA1) is grouped with the grid query: ONE grid over the input
        # cloud (built on lane 1 while SA1 is sampled) serves all of its radii -- the query's
        # cell range follows its own radius, whatever the cell edge
        grid_level = int(xyz0.shape[1]) >= tf_grouping.GRID_MIN_POINTS
        if grid_level:
            tasks.append(Task("grid1", 1, (), lambda: v.__setitem__(
                "grid1", tf_grouping.BallGrid(xyz0, MSG_GRID_EDGE))))

        def grp(i, r):
            def f():
                radius, nsample = MSG_SA[i][1][r], MSG_SA[i][2][r]
                points = None if i == 0 else inp["sa_out"][0]
                xyz, new_xyz = v["xyz"][i], v["xyz"][i + 1]
                if i == 0 and grid_level:
                    # xyz-only level (SA1): grid query and grouping in one kernel
                    idx, _, v["gp"][(i, r)] = pointnet_util.ball_group_xyz(
                        radius, nsample, xyz, new_xyz, v["grid1"])
                else:
                    idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz)
                    v["gp"][(i, r)] = pointnet_util.group_concat(xyz, points, new_xyz, idx,
                                                                 xyz_last=True,
                                                                 want_grouped_xyz=False)[0]
                v["bq"][(i, r)] = idx
            return f

        def grp_all(i):
            # every radius of a level whose input fits the multi-layer kernel (N <= 1024: SA2)
            # as ONE launch (pn2_ball_group_layers, MSG [points, xyz] order)
            def f():
                points = inp["sa_out"][0]
                specs = [(MSG_SA[i][1][r], MSG_SA[i][2][r], v["xyz"][i], points, v["xyz"][i + 1])
                         for r in range(len(MSG_SA[i][1]))]
                for r, (idx, _, new_points) in enumerate(
                        pointnet_util.ball_group_layers(specs, xyz_last=True)):
                    v["bq"][(i, r)], v["gp"][(i, r)] = idx, new_points
            return f

        def grp_radii():
            # SA1's radii as ONE launch over the grid (pn2_ball_group_xyz_grid_radii: one walk
            # over the largest radius' cells serves all three)
            def f():
                outs = pointnet_util.ball_group_xyz_radii(MSG_SA[0][1], MSG_SA[0][2], v["xyz"][0],
                                                          v["xyz"][1], v["grid1"])
                for r, (idx, _, gp) in enumerate(outs):
                    v["bq"][(0, r)], v["gp"][(0, r)] = idx, gp
            return f

        for i in range(len(MSG_SA)):
            # lane 0: SA1's sampler only; the later samplers run on lane 3 after it; radius 0's
            # grouping on lane 1, the other radii on lane 2
            spec = ([MSG_SA[i][0]], v["xyz"][i], v["fps_out"][i:i + 1])
            if i == 0:
                tasks.append(Task("fps1", 0, (), fps(0), direct=True, chain=spec))
            else:
                chain_lane = 3 - self.chain_lane if self.chain_lane < 0 else self.chain_lane  # after the radii
                tasks.append(Task(f"fps{i + 1}", chain_lane, (f"fps{i}",), fps(i), direct=True,
                                  chain=spec))
            if i > 0 and MSG_SA[i - 1][0] <= pointnet_util.BALL_GROUP_MAX_POINTS \
                    and max(MSG_SA[i][2]) <= pointnet_util.BALL_GROUP_MAX_NSAMPLE:
                tasks.append(Task(f"sa{i + 1}", 2, (f"fps{i + 1}",), grp_all(i)))
                continue
            if i == 0 and grid_level:
                tasks.append(Task("sa1", 1, ("fps1", "grid1"), grp_radii()))
                continue
            for r in range(len(MSG_SA[i][1])):
                # radius r on lane 1 + r when lane 3 is free (chain_lane 0), else radius 0 on
                # lane 1 and the others on lane 2
                lane = 1 + r if self.chain_lane <= 0 and self.overlap else 1 + min(r, 1)
                deps = (f"fps{i + 1}",) + (("grid1",) if i == 0 and grid_level else ())
                tasks.append(Task(f"sa{i + 1}_{r}", lane, deps, grp(i, r)))
        return tasks

    def outputs(self):
        v = self.v
        if "model" in self.inp:  # logits (B, N, 21), then the SA levels' features
            return [v["fp"][3]] + v["pts"][1:]
        if self.kind == "ssg":
            sa = [[p] + ([a] if "attn" in self.inp else []) for p, a in zip(v["sa"], v["att"])]
            return [t for o in sa for t in o] + list(v["fp"])
        return [v["gp"][k] for k in sorted(v["gp"])]

    def intermediates(self):
        """The index and copy results inside the step, by name (the parity tests compare them
        bit for bit): 'fps<i>.idx' / 'fps<i>.new_xyz' (sampler i + fused gather),
        'bq<i>.idx' (SSG) or 'bq<i>_<r>.idx' (MSG radius r) (ball query), and for FP layers
        whose neighbour search ran as its own kernel 'nn<k>.idx' / 'nn<k>.dist' (k = the
        FP layer, 1..4 = fa_layer1..4). Geometric step only."""
        v, out = self.v, {}
        samp = v.get("chain") or v.get("fps_out") or []
        for i, (idx, nx) in enumerate(samp):
            out[f"fps{i + 1}.idx"], out[f"fps{i + 1}.new_xyz"] = idx, nx
        if self.kind == "ssg":
            for i, idx in enumerate(v.get("bq", [])):
                out[f"bq{i + 1}.idx"] = idx
            for k, nn in enumerate(v.get("nn", [])):
                if nn is not None:
                    out[f"nn{k + 1}.dist"], out[f"nn{k + 1}.idx"] = nn
        else:
            for (i, r), idx in sorted(v.get("bq", {}).items()):
                out[f"bq{i + 1}_{r}.idx"] = idx
        return out

    # ------------------------------------------------------------------ execution
    def _stream(self, lane, main):
        return main if (lane == 0 or not self.overlap) else self.streams[lane]

    def run(self, sampler_events=None, launch=None, join=True):
        """Execute every task: launch(task) (default: its fn) on its lane's stream after its
        cross-lane dependencies; lanes join the current stream at the end unless join=False
        (then call join() before reading the outputs)."""
        main = torch.cuda.current_stream(self.inp["xyz"].device) if self.inp["xyz"].is_cuda \
            else None
        launch = launch or (lambda t: t.fn())
        self.ran = True
        if not self.overlap:
            for t in self.tasks:
                if t.name == self.SAMPLER and sampler_events is not None:
                    sampler_events[0].record()
                launch(t)
                if t.name == self.SAMPLER and sampler_events is not None:
                    sampler_events[1].record()
            return self.outputs()
        lane_of = {t.name: t.lane for t in self.tasks}
        if not self.synced_inputs:  # the resident inputs were written on the current stream
            for lane in range(1, self.nlanes):
                self.streams[lane].wait_stream(main)
            self.synced_inputs = True
        done = dict(self.done)  # this run's release events (the timed sampler's is its end event)
        for t in self.tasks:
            st = self._stream(t.lane, main)
            for d in t.deps:
                if lane_of[d] != t.lane:
                    st.wait_event(done[d])
            timed = t.name == self.SAMPLER and sampler_events is not None
            with torch.cuda.stream(st):
                if timed:
                    sampler_events[0].record(st)
                launch(t)
            if any(t.name in u.deps for u in self.tasks):
                if timed:  # one event both times the sampler and releases its dependents
                    done[t.name] = sampler_events[1]
                done[t.name].record(st)
            elif timed:
                sampler_events[1].record(st)
        # every lane records its own end; the host (Pipeline) and join() wait for all of them
        for lane in range(1, self.nlanes):
            self.lane_done[lane].record(self.streams[lane])
        return self.join() if join else None

    def done_lanes(self):
        """The lanes whose end events mark the end of the step's side work."""
        return list(range(1, self.nlanes))

    def _needed_waits(self, waits):
        """`waits` minus the events another waited task already implies (its own cross-lane
        waits reach them): each wait packet stalls the side queue, so fewer is faster."""
        deps = {t.name: t.deps for t in self.tasks}

        def closure(n, seen):
            for d in deps.get(n, ()):
                if d not in seen:
                    seen.add(d)
                    closure(d, seen)
            return seen
        implied = set()
        for w in waits:
            implied |= closure(w, set())
        return [w for w in waits if w not in implied]

    def restrict(self, only):
        """DIAGNOSTIC (bench.py --diag-only; never a measured step): keep only the samplers
        ("samplers") or only the side-lane work ("side", on the sampled buffers the full
        warm-up steps left), to see which part bounds a pipelined layout."""
        keep = (lambda t: t.direct) if only == "samplers" else (lambda t: not t.direct)
        names = {t.name for t in self.tasks if keep(t)}
        self.tasks = [Task(t.name, t.lane, [d for d in t.deps if d in names], t.fn, t.direct,
                           t.chain) for t in self.tasks if keep(t)]

    def segments(self):
        """The tasks grouped into launch segments for a native plan: consecutive tasks of one
        lane (in list order) share a segment until a task whose result another lane waits for
        (its release must not wait for the tasks after it); a direct task is a segment of its
        own, and so is every task of the whole-model step. A segment waits, up front, for every cross-lane dependency of its tasks -- never
        earlier than a task would have, only later, so a consumer still cannot run before its
        producer -- and releases its tasks' events at its end. Returned in an order in which
        every segment comes after the segments it waits for and after the earlier segments of
        its lane (the host enqueues waits after the records they refer to). A task whose
        cross-lane waits the open segment does not already imply starts a new segment, so no
        task waits for a producer it does not need. On the SSG step the side lanes become
        [grid1], [sa1], [sa2..sa4], [fp4], [fp3..fp1]."""
        lane_of = {t.name: (t.lane if self.overlap else 0) for t in self.tasks}
        xdeps = {t.name: any(t.name in u.deps and lane_of[u.name] != lane_of[t.name]
                             for u in self.tasks) for t in self.tasks}
        segs, open_seg = [], {}
        # the whole-model step keeps one segment per task: its lane-1 chain of SA and FP
        # layers waits for each neighbour search separately, not for all of them up front
        merge = "model" not in self.inp
        deps_of = {t.name: t.deps for t in self.tasks}

        def closure(names):
            seen, todo = set(), list(names)
            while todo:
                n = todo.pop()
                if n not in seen:
                    seen.add(n)
                    todo.extend(deps_of.get(n, ()))
            return seen
        seg_waits = {}  # open segment's lane -> what its up-front waits already imply
        for t in self.tasks:
            lane = lane_of[t.name]
            if t.direct or not merge:
                open_seg.pop(lane, None)
                segs.append([t])
                continue
            cur = open_seg.get(lane)
            xd = {d for d in t.deps if lane_of[d] != lane}
            # a task that would add a wait to the open segment starts its own: otherwise the
            # segment's earlier tasks would wait for it too (SA1's grouping behind the later
            # samplers' chain; profiles/r4/ab4)
            if cur is not None and not xd <= seg_waits[lane]:
                del open_seg[lane]
                cur = None
            if cur is None:
                cur = open_seg[lane] = []
                segs.append(cur)
                seg_waits[lane] = set()
            cur.append(t)
            seg_waits[lane] |= closure(xd)
            if xdeps[t.name]:
                del open_seg[lane]
        seg_of = {t.name: i for i, seg in enumerate(segs) for t in seg}
        prev_same_lane = {}
        preds = []
        for i, seg in enumerate(segs):
            lane = lane_of[seg[0].name]
            p = {seg_of[d] for t in seg for d in t.deps if seg_of[d] != i}
            if lane in prev_same_lane:
                p.add(prev_same_lane[lane])
            prev_same_lane[lane] = i
            preds.append(p)
        order, placed = [], set()
        while len(order) < len(segs):  # topological, earliest segment first
            i = next((i for i in range(len(segs)) if i not in placed and preds[i] <= placed), None)
            if i is None:
                raise RuntimeError("task dependencies form a cycle")
            order.append(segs[i])
            placed.add(i)
        return order

    @staticmethod
    def segment_key(seg):
        return "+".join(t.name for t in seg)

    def emit_plan(self, plan, graphs, main, direct=True):
        """Record the step -- per launch segment (segments()): its cross-lane waits, its
        captured kernels (graphs[segment_key]: launched directly when direct=True and the graph
        is a plain chain of kernels, else as a graph) or direct sampler launch (the task's
        `chain` spec), and the release events other lanes wait for; lane 0 = `main`; then the
        lane ends of run() -- into a native plan (plan.Plan over include/pn2plan.h), so one host
        call enqueues the whole step. The SA1 sampler is the plan's timed operation."""
        assert self.overlap and self.synced_inputs
        lane_of = {t.name: t.lane for t in self.tasks}
        for seg in self.segments():
            lane = seg[0].lane
            st = self._stream(lane, main)
            waits = []
            for t in seg:
                for d in t.deps:
                    if lane_of[d] != lane and d not in waits:
                        waits.append(d)
            for d in self._needed_waits(waits):
                plan.wait(st, self.done[d])
            if seg[0].direct:
                if seg[0].chain is None:
                    raise RuntimeError(f"task {seg[0].name}: a direct task needs its chain spec")
                c = seg[0].chain
                plan.fps_chain(c[0], c[1], c[2], st, c[3] if len(c) > 3 else None)
            elif direct:
                plan.graph_direct(graphs[self.segment_key(seg)], st)
            else:
                plan.graph(graphs[self.segment_key(seg)], st)
            if seg[0].name == self.SAMPLER:
                plan.mark_timed()
            for t in seg:
                if any(t.name in u.deps and u.lane != lane for u in self.tasks):
                    plan.record(self.done[t.name], st)
        for lane in range(1, self.nlanes):  # as run(): each lane records its own end
            plan.record(self.lane_done[lane], self.streams[lane])

    def join(self):
        """Make the current stream wait for every lane; returns the outputs (None before the
        first run)."""
        if not self.ran:
            return None
        outs = self.outputs()
        if self.overlap:
            main = torch.cuda.current_stream(self.inp["xyz"].device)
            for lane in self.done_lanes():
                main.wait_event(self.lane_done[lane])
            if not torch.cuda.is_current_stream_capturing():
                for o in outs:  # made on side streams, consumed on the current stream from here
                    o.record_stream(main)
        return outs

    def __call__(self):
        return self.run()


def run(inp):
    """One step of the configured SA + FP geometry (eager)."""
    return Step(inp)()


class GraphStep:
    """The step with every task captured as its own hipGraph (one shared memory pool), each
    on its lane's stream; replay() relaunches them with the same cross-stream events as the
    eager step. Inputs stay resident, outputs are overwritten in place at every replay."""

    def __init__(self, inp, warmup=2, overlap=True, streams=None, chain_lane=3, segments=False,
                 only=None, layout="a"):
        # segments: capture one graph per launch segment (Step.segments(), for a native plan:
        # replay_plan) instead of one per task (replay)
        self.step = Step(inp, overlap=overlap, streams=streams, chain_lane=chain_lane,
                         layout=layout)
        self.segmented = segments and self.step.overlap
        dev = inp["xyz"].device
        warm = side_stream(dev, "warm")
        warm.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(warm):
            for _ in range(warmup):
                self.step.run()
        torch.cuda.current_stream(dev).wait_stream(warm)
        torch.cuda.synchronize(dev)
        if only:
            self.step.restrict(only)
        # One memory pool PER LANE: graphs of one lane replay in capture order on one stream,
        # so a block one of them frees may be reused by a later one; graphs of different
        # lanes replay concurrently and must never share a block. (Tensors passed between
        # lanes live in self.step.v and are never freed.)
        pools = {}
        self.graphs = {}
        cap = side_stream(dev, "capture")

        def capture_tasks(ts, lane, key):
            # keep_graph: the plan reads the captured nodes (pn2_plan_graph_direct)
            g = torch.cuda.CUDAGraph(keep_graph=True)
            st = torch.cuda.current_stream(dev)
            cap.wait_stream(st)
            if lane not in pools:
                pools[lane] = torch.cuda.graph_pool_handle()
            with torch.cuda.graph(g, pool=pools[lane], stream=cap):
                for t in ts:
                    t.fn()
            g.instantiate()
            st.wait_stream(cap)
            self.graphs[key] = g

        def capture(t):
            if not t.direct:
                capture_tasks([t], t.lane if self.step.overlap else 0, t.name)

        if self.segmented:
            # each segment's tasks as one graph, in segment order, on the segment's lane pool
            # (the warm-up runs above made the direct samplers' outputs and synced the lanes)
            for seg in self.step.segments():
                if not seg[0].direct:
                    capture_tasks(seg, seg[0].lane, Step.segment_key(seg))
        else:
            self.step.run(launch=capture)
        torch.cuda.synchronize(dev)
        self.outs = self.step.outputs()

    def replay(self, sampler_events=None, join=True):
        if self.segmented:
            raise RuntimeError("a segmented GraphStep replays through replay_plan()")
        self.step.run(sampler_events, join=join,
                      launch=lambda t: t.fn() if t.direct else self.graphs[t.name].replay())
        return self.outs

    def plan_for(self, main, direct=True):
        """The native plan of this step with `main` as lane 0, recorded at the first request
        (Pipeline records every (set, sampler stream) pair it will use up front, so no plan is
        built inside a timed region). direct: the side segments' kernels launched directly
        (pn2_plan_graph_direct) instead of as graph launches."""
        if not hasattr(self, "plans"):
            self.plans = {}
        p = self.plans.get((main.cuda_stream, direct))
        if p is None:
            from .plan import Plan
            p = Plan()
            self.step.emit_plan(p, self.graphs, main, direct)
            self.plans[(main.cuda_stream, direct)] = p
        return p

    def replay_plan(self, sampler_events=None, direct=True):
        """replay(join=False) through a native plan (one host call for the whole step) for the
        current stream as lane 0."""
        main = torch.cuda.current_stream(self.step.inp["xyz"].device)
        self.plan_for(main, direct).launch(sampler_events)
        self.step.ran = True
        return self.outs

    def join(self):
        self.step.join()
        return self.outs

    def intermediates(self):
        return self.step.intermediates()


class Pipeline:
    """Consecutive steps software-pipelined over `nsets` buffer sets: step k runs on set
    k % nsets, its side-lane work (the later samplers, ball query, grouping, attention, FP)
    finishing while the following steps' SA1 samplers already run on the shared lane-0
    stream. Before a set is reused (step k + nsets) the HOST waits for that set's side lanes,
    so no buffer is overwritten while read and lane 0 carries no wait packet between
    samplers; with 3 sets the side work of a step has two sampler periods to finish. Every
    step still does all of its work; run(k) returns after enqueueing, join() waits.

    sampler_lanes > 1 (geometric steps): step k's samplers (SA1, then the later ones behind it
    on the same stream) run on sampler stream k % sampler_lanes, so the samplers of
    consecutive steps run at the same time on different CUs -- one sampler launch keeps B CUs
    busy and the rest of the chip waits on its pick chain. The side lanes (1: ball query /
    grouping / attention, 2: FP) are shared. Each stream is its own hardware queue:
    1 + 2 + (sampler_lanes - 1) <= GPU_MAX_HW_QUEUES."""

    def __init__(self, inp, graphs=True, overlap=True, nsets=3, private_streams=False,
                 sampler_lanes=1, native_plan=True, only=None, layout="a", chain_own=False,
                 set_inputs=None, chain_streams=1, direct=True):
        # chain_streams (with chain_own): the later samplers of set i run on chain stream
        # i % chain_streams, so consecutive steps' chains can overlap (one shared chain stream
        # runs one chain per step back to back: its launch time bounds the step)
        # set_inputs: one make_inputs() dict per buffer set (distinct clouds per set: the
        # steps of a pipelined run then sample different clouds); None = every set reads `inp`
        # private_streams: every buffer set gets its own side streams, so the side lanes of
        # consecutive steps overlap each other too (the whole-model step, whose lane-1 chain
        # of SA/FP layers is longer than a sampler period; the geometric step once its
        # samplers run on several streams and the shared side lanes set the pace); otherwise
        # the sets share them
        dev = inp["xyz"].device
        nsets = max(2, nsets)
        private = private_streams and overlap and inp["xyz"].is_cuda

        def streams(i):  # set 0 keeps the process-wide side streams
            if i == 0 or not private:
                return None
            # every lane a step of any layout can use (side lanes, attention, the later
            # samplers' own lane); a stream takes a hardware queue only when first used
            return [None] + [side_stream(dev, (i, lane)) for lane in range(1, MAX_LANES)]

        multi = sampler_lanes > 1 and overlap and inp["xyz"].is_cuda
        # chain_own: the later samplers on a stream of their own instead of behind SA1
        chain_lane = (-1 if chain_own else 0) if multi else 3
        self.lane0 = [None]
        if multi:
            # queues go to streams in order of first use: the extra sampler streams now, then
            # each set's side lanes when its Step is built (Step.__init__ touches them in
            # order), all before the sets' warm-up and capture streams
            cur = torch.cuda.current_stream(dev)
            for i in range(1, sampler_lanes):
                st = side_stream(dev, ("sampler", i))
                st.wait_stream(cur)
                self.lane0.append(st)
        # native_plan: a graph step is enqueued by ONE call into the C++ executor
        # (include/pn2plan.h), its side lanes as a few segment graphs, instead of the per-task
        # Python loop
        self.native_plan = native_plan and graphs and overlap and inp["xyz"].is_cuda
        # direct: the plans launch the side segments' captured kernels directly
        # (pn2_plan_graph_direct) instead of as one graph launch each
        self.direct = direct
        # only: DIAGNOSTIC restriction of every step to its samplers or its side work
        if set_inputs is not None and len(set_inputs) != nsets:
            raise ValueError(f"set_inputs: {len(set_inputs)} input dicts for {nsets} sets")
        inps = list(set_inputs) if set_inputs is not None else [inp] * nsets
        cl = (lambda i: chain_lane - (i % max(1, chain_streams)) if chain_lane < 0
              else chain_lane)
        mk = (lambda i: GraphStep(inps[i], overlap=overlap, streams=streams(i),
                                  chain_lane=cl(i), segments=self.native_plan, only=only,
                                  layout=layout)) \
            if graphs else (lambda i: Step(inps[i], overlap=overlap, streams=streams(i),
                                           chain_lane=cl(i), layout=layout))
        self.sets = [mk(i) for i in range(nsets)]
        self.inputs = inps
        self.k = 0
        self.host_wait_s = self.host_launch_s = 0.0  # host wait for a set / enqueue time
        if self.native_plan:
            # every (set, sampler stream) pair the rotation will meet gets its plan now, not at
            # its first replay (which could fall inside a timed region)
            nl = len(self.lane0)
            for k in range(nsets * nl // math.gcd(nsets, nl)):
                st = self.lane0[k % nl] or torch.cuda.current_stream(dev)
                self.sets[k % nsets].plan_for(st, self.direct)

    def prime(self):
        """Run every (buffer set, sampler stream) pair's step once and wait for it: the first
        launch of a set's plan and kernels, its events and buffers then happen here, outside
        any timed region (at the driver's 5 warm-up steps, 4 of cfg2's 9 sets were first used
        inside the 20 timed steps: 71.6k median against 77.1k with 20 warm-up steps,
        profiles/r5/warm). Returns the number of steps run; the rotation starts again at set 0."""
        nl = len(self.lane0)
        n = len(self.sets) * nl // math.gcd(len(self.sets), nl)
        for _ in range(n):
            self.run()
        self.join()
        self.k = 0
        self.host_wait_s = self.host_launch_s = 0.0
        return n

    def run(self, sampler_events=None):
        st = self.lane0[self.k % len(self.lane0)]
        if st is not None:
            with torch.cuda.stream(st):
                return self._run(sampler_events)
        return self._run(sampler_events)

    def start_trace(self):
        """DIAGNOSTIC (bench.py --timeline): from now on every step records its host times
        (wait for the set, enqueue) and, once its set is reused (or at finish_trace), the GPU
        times of its lane ends relative to a base event; sampler events passed to run() are
        read the same way. No cost when not started."""
        self.trace = []
        self.trace_base = torch.cuda.Event(enable_timing=True)
        self.trace_base.record()
        self.trace_t0 = time.perf_counter()
        self._last_of_set = {}

    def _trace_done(self, si):
        # the set's previous step: its lane-end events are complete (synchronised or joined)
        j = self._last_of_set.get(si)
        if j is None:
            return
        st = self.sets[si].step if isinstance(self.sets[si], GraphStep) else self.sets[si]
        rec = self.trace[j]
        rec["lane_end_ms"] = {lane: self.trace_base.elapsed_time(st.lane_done[lane])
                              for lane in st.done_lanes()}
        ev = rec.pop("_events", None)
        if ev is not None:
            rec["sampler_ms"] = [self.trace_base.elapsed_time(ev[0]),
                                 self.trace_base.elapsed_time(ev[1])]

    def finish_trace(self):
        """Synchronise and complete the records of the last steps; returns the list."""
        torch.cuda.synchronize()
        for si in range(len(self.sets)):
            self._trace_done(si)
        out, self.trace = self.trace, None
        return out

    def _run(self, sampler_events):
        si = self.k % len(self.sets)
        s = self.sets[si]
        self.k += 1
        t0 = time.perf_counter()
        tr = getattr(self, "trace", None)
        try:
            if isinstance(s, GraphStep):
                if s.step.ran and s.step.overlap:
                    for lane in s.step.done_lanes():  # this set's previous side work
                        s.step.lane_done[lane].synchronize()
                else:
                    s.step.join()
                t1 = time.perf_counter()
                self.host_wait_s += t1 - t0
                if tr is not None:
                    self._trace_done(si)
                    tr.append({"k": self.k - 1, "set": si,
                               "host_ms": [(t0 - self.trace_t0) * 1e3, (t1 - self.trace_t0) * 1e3],
                               "_events": sampler_events})
                    self._last_of_set[si] = len(tr) - 1
                t0 = t1
                if self.native_plan:
                    return s.replay_plan(sampler_events, self.direct)
                return s.replay(sampler_events, join=False)
            s.join()
            return s.run(sampler_events, join=False)
        finally:  # host time of the enqueue (bench.py reports both per step)
            t2 = time.perf_counter()
            self.host_launch_s += t2 - t0
            if tr is not None and tr and "host_ms" in tr[-1] and len(tr[-1]["host_ms"]) == 2:
                tr[-1]["host_ms"].append((t2 - self.trace_t0) * 1e3)

    def join(self):
        """Wait for everything enqueued; returns the outputs of the last step run. Raises
        RuntimeError if a sampler launch that has already completed stored a fault (the host
        sees the fault word once the launch is done; check_faults() synchronises first)."""
        for s in self.sets:
            s.join()
        out = self.sets[(self.k - 1) % len(self.sets)].join()
        _raise_fault(_lib_fault_status(clear=True))
        return out

    def check_faults(self):
        """Synchronise with every set's enqueued work, then return the sampler fault word
        (include/pn2hip.h pn2_fault_status; 0 = no fault) and clear it, raising RuntimeError
        when it is set (Pn2RuntimeError): the indices of the step whose sampler faulted are not
        to be trusted."""
        for s in self.sets:
            st = s.step if isinstance(s, GraphStep) else s
            if st.ran and st.overlap:
                for lane in range(1, st.nlanes):
                    st.lane_done[lane].synchronize()
        torch.cuda.synchronize(self.inputs[0]["xyz"].device)
        code = _lib_fault_status(clear=True)
        _raise_fault(code)
        return code

    def outputs_by_set(self):
        """(inputs, outputs, intermediates) of every set's last step, after join()."""
        res = []
        for s, inp in zip(self.sets, self.inputs):
            st = s.step if isinstance(s, GraphStep) else s
            if st.ran:
                res.append((inp, st.outputs(), st.intermediates()))
        return res


def _lib_fault_status(clear):
    from ._lib import lib
    return int(lib().pn2_fault_status(1 if clear else 0))


def _raise_fault(code):
    if code:
        from ._lib import Pn2RuntimeError
        raise Pn2RuntimeError(f"sampler fault {code} (pn2_fault_status; PN2_FAULT_FPS_POLL = 1: a "
                              "culled sampler's cold waves ran past their poll bound): the "
                              "indices of the step it sampled are not valid")


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
