"""The hot-path geometry of pointnet2_tensorflow/utils/pointnet_util.py on gfx950.

sample_and_group / sample_and_group_all keep the reference signatures and return values.
The geometric halves of the SA / FP layers:

  sample_and_group          pointnet_util.py:16-58    FPS + gather + ball query + fused group
  sample_and_group_all      pointnet_util.py:61-87
  sample_and_group_msg      pointnet_util.py:180-193  one FPS, several (radius, nsample) scales
  ball_group_layers         several layers' query_ball_point + group_concat, one launch
  group_pool                pointnet_util.py:130-145  max / avg / weighted_avg / max_and_avg
  fp_interpolate            pointnet_util.py:218-228  three_nn + IDW + interpolate + concat
  fp_interpolate_layers     several FP layers' fp_interpolate, one launch

The whole layers, shared MLP included (tf_util.py for the parameters):

  pointnet_sa_module        pointnet_util.py:90-163   group + MLP + pooling in one kernel
  pointnet_sa_module_msg    pointnet_util.py:166-201  one fused kernel per scale
  pointnet_fp_module        pointnet_util.py:204-238  interpolation + MLP in one kernel

Without autograd the fused kernels run (fewest launches, one pass over HBM); when a gradient
is required, the composition of differentiable ops (gather_point, group_point,
three_interpolate) is used instead so that backward reaches xyz and points like the
reference's registered gradients.
"""
import ctypes

import torch

from . import tf_grouping, tf_interpolate, tf_sampling, tf_util
from ._lib import (POOL_MODES, PN2_BQ_MAX_RADII, PN2_ENOTSUP, PN2_FP_MAX_LAYERS, PN2_POOL_NONE,
                   PN2_SA_MAX_LAYERS, PN2_USE_XYZ, PN2_XYZ_LAST, FpLayer, InvalidArgumentError,
                   SaLayer, check, device_tensor, lib, ptr, stream_of)


def _is_empty_points(points):
    # pointnet_util.py:41: points with the shape of tf.zeros([0]) mean "no features"
    return points is None or (points.dim() == 1 and points.shape[0] == 0)


def _needs_grad(*ts):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


def group_concat(xyz, points, new_xyz, idx, use_xyz=True, xyz_last=False, want_grouped_xyz=True):
    """Fused group_point(xyz) - new_xyz, group_point(points) and concat
    (pointnet_util.py:39-56 SSG order [xyz, points]; xyz_last=True gives the MSG order
    [points, xyz] of :191). Returns (new_points, grouped_xyz or None)."""
    B, N = int(xyz.shape[0]), int(xyz.shape[1])
    M, ns = int(idx.shape[1]), int(idx.shape[2])
    if _is_empty_points(points):
        points, C, Cout = None, 0, 3
    else:
        points = device_tensor(points, "points", torch.float32)
        C = int(points.shape[2])
        Cout = C + 3 if use_xyz else C
    if _needs_grad(xyz, points, new_xyz):
        grouped_xyz = tf_grouping.group_point(xyz, idx) - new_xyz.unsqueeze(2)
        if points is None:
            return grouped_xyz, grouped_xyz
        gp = tf_grouping.group_point(points, idx)
        if not use_xyz:
            return gp, grouped_xyz
        parts = [gp, grouped_xyz] if xyz_last else [grouped_xyz, gp]
        return torch.cat(parts, dim=-1), grouped_xyz
    flags = (PN2_USE_XYZ if use_xyz else 0) | (PN2_XYZ_LAST if xyz_last else 0)
    new_points = torch.empty((B, M, ns, Cout), dtype=torch.float32, device=xyz.device)
    grouped_xyz = torch.empty((B, M, ns, 3), dtype=torch.float32, device=xyz.device) \
        if (want_grouped_xyz and points is not None) else None
    check(lib().pn2_group_concat(ptr(xyz), ptr(points), ptr(new_xyz), ptr(idx), B, N, C, M, ns,
                                 flags, ptr(grouped_xyz), ptr(new_points), stream_of(xyz)),
          "group_concat")
    if points is None and want_grouped_xyz:
        grouped_xyz = new_points  # identical values (pointnet_util.py:56)
    return new_points, grouped_xyz


def ball_group_xyz(radius, nsample, xyz, new_xyz, grid):
    """query_ball_point over `grid` (a tf_grouping.BallGrid built over xyz) and the grouping of
    an xyz-only layer (group_concat with points None: xyz[idx] - new_xyz, pointnet_util.py:
    39-40, 55-56) in ONE kernel (pn2_ball_group_xyz_grid). Returns (idx, pts_cnt, grouped)."""
    xyz = device_tensor(xyz, "xyz", torch.float32)
    new_xyz = device_tensor(new_xyz, "new_xyz", torch.float32)
    if not grid.matches(xyz):
        raise InvalidArgumentError("ball_group_xyz: the grid was built over a different xyz")
    B, N, M, ns = int(xyz.shape[0]), int(xyz.shape[1]), int(new_xyz.shape[1]), int(nsample)
    if int(new_xyz.shape[0]) != B:
        raise InvalidArgumentError("ball_group_xyz: xyz and new_xyz need the same batch")
    idx = torch.empty((B, M, ns), dtype=torch.int32, device=xyz.device)
    cnt = torch.empty((B, M), dtype=torch.int32, device=xyz.device)
    grouped = torch.empty((B, M, ns, 3), dtype=torch.float32, device=xyz.device)
    check(lib().pn2_ball_group_xyz_grid(ptr(grid.buf), ptr(xyz), ptr(new_xyz), B, N, M,
                                        float(radius), ns, ptr(idx), ptr(cnt), ptr(grouped),
                                        stream_of(xyz)), "ball_group_xyz")
    return idx, cnt, grouped


def ball_group(radius, nsample, xyz, points, new_xyz, grid, xyz_last=False):
    """query_ball_point over `grid` (a tf_grouping.BallGrid built over xyz) and the grouping +
    centring + concat of sample_and_group (pointnet_util.py:38-52; xyz_last: the MSG order
    :186-191) in ONE kernel (pn2_ball_group_grid). points None: ball_group_xyz. Returns (idx,
    pts_cnt, new_points), bit-identical to query_ball_point + group_concat."""
    if points is None:
        return ball_group_xyz(radius, nsample, xyz, new_xyz, grid)
    xyz = device_tensor(xyz, "xyz", torch.float32)
    points = device_tensor(points, "points", torch.float32)
    new_xyz = device_tensor(new_xyz, "new_xyz", torch.float32)
    if not grid.matches(xyz):
        raise InvalidArgumentError("ball_group: the grid was built over a different xyz")
    B, N, M, ns = int(xyz.shape[0]), int(xyz.shape[1]), int(new_xyz.shape[1]), int(nsample)
    if int(new_xyz.shape[0]) != B or tuple(points.shape[:2]) != (B, N):
        raise InvalidArgumentError("ball_group: xyz (B,N,3), points (B,N,C), new_xyz (B,M,3)")
    C = int(points.shape[2])
    idx = torch.empty((B, M, ns), dtype=torch.int32, device=xyz.device)
    cnt = torch.empty((B, M), dtype=torch.int32, device=xyz.device)
    new_points = torch.empty((B, M, ns, C + 3), dtype=torch.float32, device=xyz.device)
    flags = PN2_USE_XYZ | (PN2_XYZ_LAST if xyz_last else 0)
    check(lib().pn2_ball_group_grid(ptr(grid.buf), ptr(xyz), ptr(points), C, flags,
                                    ptr(new_xyz), B, N, M, float(radius), ns, ptr(idx),
                                    ptr(cnt), ptr(new_points), stream_of(xyz)), "ball_group")
    return idx, cnt, new_points


def ball_group_xyz_radii(radii, nsamples, xyz, new_xyz, grid):
    """ball_group_xyz for several radii of the same queries (MSG's SA1 radius loop,
    pointnet_util.py:162-203) in ONE kernel (pn2_ball_group_xyz_grid_radii: one walk over the
    largest radius' cells). Returns [(idx, pts_cnt, grouped)] per radius, each bit-identical
    to ball_group_xyz(radius, nsample, ...)."""
    xyz = device_tensor(xyz, "xyz", torch.float32)
    new_xyz = device_tensor(new_xyz, "new_xyz", torch.float32)
    nr = len(radii)
    if not 1 <= nr <= PN2_BQ_MAX_RADII or len(nsamples) != nr:
        raise InvalidArgumentError(f"ball_group_xyz_radii: 1..{PN2_BQ_MAX_RADII} radii, one "
                                   "nsample each")
    if not grid.matches(xyz):
        raise InvalidArgumentError("ball_group_xyz_radii: the grid was built over a different xyz")
    B, N, M = int(xyz.shape[0]), int(xyz.shape[1]), int(new_xyz.shape[1])
    if int(new_xyz.shape[0]) != B:
        raise InvalidArgumentError("ball_group_xyz_radii: xyz and new_xyz need the same batch")
    if nr * ((N + 31) // 32) > 4096:
        # the bitmasks' LDS bound (grid.hip ball_query_grid: 4 waves x nr x words x 4 B <= 64 KB;
        # the xyz-only path keeps no hit lists): one launch per radius
        return [ball_group_xyz(r, ns, xyz, new_xyz, grid) for r, ns in zip(radii, nsamples)]
    outs = []
    for ns in nsamples:
        ns = int(ns)
        outs.append((torch.empty((B, M, ns), dtype=torch.int32, device=xyz.device),
                     torch.empty((B, M), dtype=torch.int32, device=xyz.device),
                     torch.empty((B, M, ns, 3), dtype=torch.float32, device=xyz.device)))
    rad = (ctypes.c_float * nr)(*[float(r) for r in radii])
    nsa = (ctypes.c_int * nr)(*[int(n) for n in nsamples])
    ids = (ctypes.c_void_p * nr)(*[ptr(o[0]) for o in outs])
    cnts = (ctypes.c_void_p * nr)(*[ptr(o[1]) for o in outs])
    grps = (ctypes.c_void_p * nr)(*[ptr(o[2]) for o in outs])
    check(lib().pn2_ball_group_xyz_grid_radii(ptr(grid.buf), ptr(xyz), ptr(new_xyz), B, N, M, nr,
                                              rad, nsa, ids, cnts, grps, stream_of(xyz)),
          "ball_group_xyz_radii")
    return outs


BALL_GROUP_MAX_POINTS = 1024  # pn2_ball_group_layers stages each cloud in LDS
BALL_GROUP_MAX_NSAMPLE = 128


def ball_group_layers(layers, use_xyz=True, xyz_last=False, want_grouped_xyz=False):
    """query_ball_point followed by group_concat for several layers in ONE launch
    (pn2_ball_group_layers): layers = [(radius, nsample, xyz, points, new_xyz)], every cloud at
    most BALL_GROUP_MAX_POINTS points. Returns [(idx, pts_cnt, new_points)], plus grouped_xyz
    (B, M, nsample, 3) as a 4th element with want_grouped_xyz, bit-identical to the separate
    ops (tf_grouping_g.cu:3-57, pointnet_util.py:38-58)."""
    if not 1 <= len(layers) <= PN2_SA_MAX_LAYERS:
        raise InvalidArgumentError(f"ball_group_layers: 1..{PN2_SA_MAX_LAYERS} layers")
    flags = (PN2_USE_XYZ if use_xyz else 0) | (PN2_XYZ_LAST if xyz_last else 0)
    arr = (SaLayer * len(layers))()
    outs, keep, B = [], [], None
    for a, (radius, nsample, xyz, points, new_xyz) in zip(arr, layers):
        xyz = device_tensor(xyz, "xyz", torch.float32)
        new_xyz = device_tensor(new_xyz, "new_xyz", torch.float32)
        if B is None:
            B = int(xyz.shape[0])
        N, M, ns = int(xyz.shape[1]), int(new_xyz.shape[1]), int(nsample)
        if int(xyz.shape[0]) != B or int(new_xyz.shape[0]) != B:
            raise InvalidArgumentError("ball_group_layers: every layer needs the same batch")
        if N > BALL_GROUP_MAX_POINTS or not 0 < ns <= BALL_GROUP_MAX_NSAMPLE or not radius > 0:
            raise InvalidArgumentError("ball_group_layers: N <= 1024, 0 < nsample <= 128, "
                                       "radius > 0")
        if _is_empty_points(points):
            points, C, Cout = None, 0, 3
        else:
            points = device_tensor(points, "points", torch.float32)
            if tuple(points.shape[:2]) != (B, N):
                raise InvalidArgumentError("ball_group_layers: points (B,N,C) for xyz (B,N,3)")
            C = int(points.shape[2])
            Cout = C + 3 if use_xyz else C
        idx = torch.empty((B, M, ns), dtype=torch.int32, device=xyz.device)
        cnt = torch.empty((B, M), dtype=torch.int32, device=xyz.device)
        new_points = torch.empty((B, M, ns, Cout), dtype=torch.float32, device=xyz.device)
        gxyz = (torch.empty((B, M, ns, 3), dtype=torch.float32, device=xyz.device)
                if want_grouped_xyz else None)
        a.xyz, a.points, a.new_xyz = ptr(xyz), ptr(points), ptr(new_xyz)
        a.N, a.C, a.M, a.nsample, a.radius, a.flags = N, C, M, ns, float(radius), flags
        a.idx, a.pts_cnt, a.grouped_xyz, a.new_points = ptr(idx), ptr(cnt), ptr(gxyz), ptr(new_points)
        keep += [xyz, points, new_xyz]
        outs.append((idx, cnt, new_points) + ((gxyz,) if want_grouped_xyz else ()))
    check(lib().pn2_ball_group_layers(arr, len(layers), B, stream_of(keep[0])),
          "ball_group_layers")
    return outs


def sample_and_group(npoint, radius, nsample, xyz, points, knn=False, use_xyz=True):
    """pointnet_util.py:16-58.

    Output:
        new_xyz: (batch_size, npoint, 3)
        new_points: (batch_size, npoint, nsample, 3+channel)
        idx: (batch_size, npoint, nsample) int32
        grouped_xyz: (batch_size, npoint, nsample, 3), centred on new_xyz
    """
    xyz = device_tensor(xyz, "xyz", torch.float32)
    if _needs_grad(xyz):
        fps_idx = tf_sampling.farthest_point_sample(npoint, xyz)
        new_xyz = tf_sampling.gather_point(xyz, fps_idx)
    else:
        _, new_xyz = tf_sampling.farthest_point_sample_and_gather(npoint, xyz)
    if knn:  # pointnet_util.py:35-36
        _, idx = tf_grouping.knn_point(nsample, xyz, new_xyz.detach())
    else:
        idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz.detach())
    new_points, grouped_xyz = group_concat(xyz, points, new_xyz, idx, use_xyz=use_xyz)
    return new_xyz, new_points, idx, grouped_xyz


def sample_and_group_all(xyz, points, use_xyz=True):
    """pointnet_util.py:61-87: one group per cloud holding every point, centroid (0,0,0)."""
    xyz = device_tensor(xyz, "xyz", torch.float32)
    B, N = int(xyz.shape[0]), int(xyz.shape[1])
    new_xyz = torch.zeros((B, 1, 3), dtype=torch.float32, device=xyz.device)
    idx = torch.arange(N, dtype=torch.int32, device=xyz.device).reshape(1, 1, N).expand(
        B, 1, N).contiguous()
    grouped_xyz = xyz.reshape(B, 1, N, 3)
    if _is_empty_points(points):
        return new_xyz, grouped_xyz, idx, grouped_xyz
    new_points = torch.cat([xyz, points], dim=2) if use_xyz else points
    return new_xyz, new_points.unsqueeze(1), idx, grouped_xyz


def sample_and_group_msg(npoint, radius_list, nsample_list, xyz, points, use_xyz=True):
    """Grouping half of pointnet_sa_module_msg (pointnet_util.py:180-193): one FPS, then per
    scale a ball query and the fused group with the MSG concat order [points, xyz].
    Returns (new_xyz, [grouped_points per scale])."""
    xyz = device_tensor(xyz, "xyz", torch.float32)
    if _needs_grad(xyz):
        new_xyz = tf_sampling.gather_point(xyz, tf_sampling.farthest_point_sample(npoint, xyz))
    else:
        _, new_xyz = tf_sampling.farthest_point_sample_and_gather(npoint, xyz)
    out = []
    for radius, nsample in zip(radius_list, nsample_list):
        idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz.detach())
        gp, _ = group_concat(xyz, points, new_xyz, idx, use_xyz=use_xyz, xyz_last=True,
                             want_grouped_xyz=False)
        out.append(gp)
    return new_xyz, out


def group_pool(new_points, pooling="max", grouped_xyz=None):
    """Per-region pooling of pointnet_sa_module (pointnet_util.py:130-145), keep_dims=True:
    (B, M, ns, C) -> (B, M, 1, C), or (B, M, 1, 2C) = [avg, max] for 'max_and_avg'."""
    if pooling not in POOL_MODES:
        raise InvalidArgumentError(f"unknown pooling {pooling!r}")
    if new_points.dim() != 4:
        raise InvalidArgumentError("group_pool expects (batch_size, npoint, nsample, channel)")
    x = device_tensor(new_points, "new_points", torch.float32)
    B, M, ns, C = (int(s) for s in x.shape)
    g = None
    if pooling == "weighted_avg":
        if grouped_xyz is None or tuple(grouped_xyz.shape) != (B, M, ns, 3):
            raise InvalidArgumentError("weighted_avg pooling needs grouped_xyz (B, M, ns, 3)")
        g = device_tensor(grouped_xyz, "grouped_xyz", torch.float32)
    Cout = 2 * C if pooling == "max_and_avg" else C
    out = torch.empty((B, M, 1, Cout), dtype=torch.float32, device=x.device)
    check(lib().pn2_group_pool(ptr(x), ptr(g), B, M, ns, C, POOL_MODES[pooling], ptr(out),
                               stream_of(x)), "group_pool")
    return out


FP_GRID_MAX_KNOWN = 4096  # pn2_fp_grid_fused's LDS bound on m


def fp_interpolate(xyz1, xyz2, points1, points2, known_grid=None, unknown_grid=None,
                   return_nn=False):
    """Geometry of pointnet_fp_module (pointnet_util.py:218-228), before its MLP:
    three_nn, IDW weights, three_interpolate and concat [interpolated, points1].
    Returns (B, n, C2 + C1). known_grid / unknown_grid: optional grid.PointGrid over xyz2 /
    xyz1 for the neighbour search. A large search without a known grid (FP4) is ONE launch,
    pn2_fp_grid_fused, whose workgroups grid the known points in LDS themselves.
    return_nn: also return the three_nn (dist, idx) the layer used, or None when the search
    ran fused inside the interpolation kernel (pn2_fp_fused keeps them in registers)."""
    xyz1 = device_tensor(xyz1, "xyz1", torch.float32)
    xyz2 = device_tensor(xyz2, "xyz2", torch.float32)
    points2 = device_tensor(points2, "points2", torch.float32)
    if _needs_grad(points1, points2):
        dist, idx = tf_interpolate.three_nn(xyz1, xyz2, known_grid, unknown_grid)
        weight = tf_interpolate.idw_weights(dist)
        interp = tf_interpolate.three_interpolate(points2, idx, weight)
        out = interp if points1 is None else torch.cat([interp, points1], dim=2)
        return (out, (dist, idx)) if return_nn else out
    B, n, m = int(xyz1.shape[0]), int(xyz1.shape[1]), int(xyz2.shape[1])
    C2 = int(points2.shape[2])
    if points1 is not None:
        points1 = device_tensor(points1, "points1", torch.float32)
        C1 = int(points1.shape[2])
    else:
        C1 = 0
    nn = None
    if known_grid is not None and known_grid.cell_edge <= 0 and m <= FP_GRID_MAX_KNOWN \
            and C1 + C2 > 0 and tf_interpolate.use_grid(n, m):
        # one launch over the known points' prebuilt grid (pn2_fp_grid_fused_known: the SA1
        # sampler built it, pn2_fps_chain_grid), staged into each workgroup's LDS
        if not known_grid.matches(xyz2) or (unknown_grid is not None
                                            and not unknown_grid.matches(xyz1)):
            raise InvalidArgumentError("fp_interpolate: a grid was built over other points")
        out = torch.empty((B, n, C2 + C1), dtype=torch.float32, device=xyz1.device)
        if return_nn:
            nn = (torch.empty((B, n, 3), dtype=torch.float32, device=xyz1.device),
                  torch.empty((B, n, 3), dtype=torch.int32, device=xyz1.device))
        rc = lib().pn2_fp_grid_fused_known(
            ptr(known_grid.buf), ptr(xyz1), ptr(xyz2),
            None if unknown_grid is None else ptr(unknown_grid.buf),
            ptr(points1), C1, ptr(points2), C2, B, n, m, ptr(out),
            ptr(nn[0]) if nn else None, ptr(nn[1]) if nn else None, stream_of(xyz1))
        if rc == PN2_ENOTSUP:
            # (the known grid does not fit this device's LDS per workgroup; any other code,
            # PN2_EINVAL included, is an argument error and raises below)
            nn = tf_interpolate.three_nn(xyz1, xyz2, known_grid, unknown_grid)
            out = fp_apply(nn, points1, points2, unknown_grid)
        else:
            check(rc, "fp_interpolate")
    elif known_grid is None and tf_interpolate.use_grid(n, m) and m <= FP_GRID_MAX_KNOWN \
            and C1 + C2 > 0:
        # one launch: each workgroup grids the known points in LDS, searches, writes its rows
        if unknown_grid is not None and not unknown_grid.matches(xyz1):
            raise InvalidArgumentError("fp_interpolate: the unknown grid was built over other points")
        out = torch.empty((B, n, C2 + C1), dtype=torch.float32, device=xyz1.device)
        if return_nn:
            nn = (torch.empty((B, n, 3), dtype=torch.float32, device=xyz1.device),
                  torch.empty((B, n, 3), dtype=torch.int32, device=xyz1.device))
        rc = lib().pn2_fp_grid_fused(ptr(xyz1), ptr(xyz2),
                                     None if unknown_grid is None else ptr(unknown_grid.buf),
                                     ptr(points1), C1, ptr(points2), C2, B, n, m, ptr(out),
                                     ptr(nn[0]) if nn else None, ptr(nn[1]) if nn else None,
                                     stream_of(xyz1))
        if rc == PN2_ENOTSUP:
            # (the known grid does not fit this device's LDS per workgroup; any other code,
            # PN2_EINVAL included, is an argument error and raises below)
            nn = tf_interpolate.three_nn(xyz1, xyz2, None, unknown_grid)
            out = fp_apply(nn, points1, points2, unknown_grid)
        else:
            check(rc, "fp_interpolate")
    elif known_grid is not None or tf_interpolate.use_grid(n, m):
        nn = tf_interpolate.three_nn(xyz1, xyz2, known_grid, unknown_grid)
        out = fp_apply(nn, points1, points2, unknown_grid)
    else:
        out = torch.empty((B, n, C2 + C1), dtype=torch.float32, device=xyz1.device)
        check(lib().pn2_fp_fused(ptr(xyz1), ptr(xyz2), ptr(points1), C1, ptr(points2), C2, B, n,
                                 m, ptr(out), stream_of(xyz1)), "fp_interpolate")
    return (out, nn) if return_nn else out


def fp_apply(nn, points1, points2, unknown_grid=None):
    """The second half of fp_interpolate's grid path (pn2_fp_apply): IDW weights from the
    three_nn distances, three_interpolate and concat [interpolated, points1] -- nn = (dist, idx)
    of tf_interpolate.three_nn over the same points (unknown_grid: the grid that search took
    its unknowns' order from; rows are written in that order). Returns (B, n, C2 + C1)."""
    dist, idx = nn
    points2 = device_tensor(points2, "points2", torch.float32)
    B, n, m, C2 = int(dist.shape[0]), int(dist.shape[1]), int(points2.shape[1]), int(points2.shape[2])
    if tuple(idx.shape) != (B, n, 3) or tuple(dist.shape) != (B, n, 3) or int(points2.shape[0]) != B:
        raise InvalidArgumentError("fp_apply: dist / idx (B,n,3), points2 (B,m,C2)")
    if points1 is not None:
        points1 = device_tensor(points1, "points1", torch.float32)
        if tuple(points1.shape[:2]) != (B, n):
            raise InvalidArgumentError("fp_apply: points1 (B,n,C1)")
        C1 = int(points1.shape[2])
    else:
        C1 = 0
    if unknown_grid is not None and int(unknown_grid.N) != n:
        raise InvalidArgumentError("fp_apply: the unknown grid was built over other points")
    out = torch.empty((B, n, C2 + C1), dtype=torch.float32, device=dist.device)
    check(lib().pn2_fp_apply(ptr(dist), ptr(idx),
                             None if unknown_grid is None else ptr(unknown_grid.buf),
                             ptr(points1), C1, ptr(points2), C2, B, n, m, ptr(out),
                             stream_of(dist)), "fp_apply")
    return out


def fp_interpolate_layers(layers):
    """fp_interpolate (fused search path, no grid) of several FP layers in ONE launch
    (pn2_fp_fused_layers): layers = [(xyz1, xyz2, points1, points2)] with the same batch.
    Returns [out (B, n, C2 + C1)], bit-identical to fp_interpolate per layer."""
    if not 1 <= len(layers) <= PN2_FP_MAX_LAYERS:
        raise InvalidArgumentError(f"fp_interpolate_layers: 1..{PN2_FP_MAX_LAYERS} layers")
    arr = (FpLayer * len(layers))()
    outs, keep, B = [], [], None
    for a, (xyz1, xyz2, points1, points2) in zip(arr, layers):
        xyz1 = device_tensor(xyz1, "xyz1", torch.float32)
        xyz2 = device_tensor(xyz2, "xyz2", torch.float32)
        points2 = device_tensor(points2, "points2", torch.float32)
        if B is None:
            B = int(xyz1.shape[0])
        n, m, C2 = int(xyz1.shape[1]), int(xyz2.shape[1]), int(points2.shape[2])
        if int(xyz1.shape[0]) != B or int(xyz2.shape[0]) != B or tuple(points2.shape[:2]) != (B, m):
            raise InvalidArgumentError("fp_interpolate_layers: xyz1 (B,n,3), xyz2 (B,m,3), "
                                       "points2 (B,m,C2) with one batch size")
        C1 = 0
        if points1 is not None:
            points1 = device_tensor(points1, "points1", torch.float32)
            if tuple(points1.shape[:2]) != (B, n):
                raise InvalidArgumentError("fp_interpolate_layers: points1 (B,n,C1)")
            C1 = int(points1.shape[2])
        out = torch.empty((B, n, C2 + C1), dtype=torch.float32, device=xyz1.device)
        a.xyz1, a.xyz2, a.points1, a.points2 = ptr(xyz1), ptr(xyz2), ptr(points1), ptr(points2)
        a.C1, a.C2, a.n, a.m, a.out = C1, C2, n, m, ptr(out)
        keep += [xyz1, xyz2, points1, points2]
        outs.append(out)
    check(lib().pn2_fp_fused_layers(arr, len(layers), B, stream_of(keep[0])),
          "fp_interpolate_layers")
    return outs


# ---------------------------------------------------------------- whole SA / FP layers -----

def group_mlp(xyz, points, new_xyz, idx, mlp, pooling="max", use_xyz=True, xyz_last=False):
    """Fused group + centre + concat (as group_concat) -> shared MLP `mlp` (a
    tf_util.SharedMLP) -> pooling over nsample (pn2_group_mlp). pooling: 'max', 'avg',
    'weighted_avg', 'max_and_avg' -> (B, M, C') or None -> per-point (B, M, ns, C)."""
    xyz = device_tensor(xyz, "xyz", torch.float32)
    new_xyz = device_tensor(new_xyz, "new_xyz", torch.float32)
    idx = device_tensor(idx, "idx", torch.int32)
    B, N = int(xyz.shape[0]), int(xyz.shape[1])
    M, ns = int(idx.shape[1]), int(idx.shape[2])
    if _is_empty_points(points):
        points, C = None, 0
    else:
        points = device_tensor(points, "points", torch.float32)
        C = int(points.shape[2])
    if pooling is not None and pooling not in POOL_MODES:
        raise InvalidArgumentError(f"unknown pooling {pooling!r}")
    mode = PN2_POOL_NONE if pooling is None else POOL_MODES[pooling]
    cout = mlp.cout
    if pooling is None:
        shape = (B, M, ns, cout)
    else:
        shape = (B, M, 2 * cout if pooling == "max_and_avg" else cout)
    out = torch.empty(shape, dtype=torch.float32, device=xyz.device)
    flags = (PN2_USE_XYZ if use_xyz else 0) | (PN2_XYZ_LAST if xyz_last else 0)
    tab, n = mlp.table()
    check(lib().pn2_group_mlp(ptr(xyz), ptr(points), ptr(new_xyz), ptr(idx), B, N, C, M, ns,
                              flags, n, tab, mode, ptr(out), stream_of(xyz)), "group_mlp")
    return out


def _pool_torch(x, pooling, grouped_xyz):
    # pointnet_util.py:130-145 (keep_dims=False)
    if pooling == "max":
        return x.max(dim=2).values
    if pooling == "avg":
        return x.mean(dim=2)
    if pooling == "weighted_avg":
        e = torch.exp(-torch.linalg.norm(grouped_xyz, dim=-1, keepdim=True) * 5)
        return (x * (e / e.sum(dim=2, keepdim=True))).sum(dim=2)
    if pooling == "max_and_avg":
        return torch.cat([x.mean(dim=2), x.max(dim=2).values], dim=-1)
    raise InvalidArgumentError(f"unknown pooling {pooling!r}")


def pointnet_sa_module(xyz, points, npoint, radius, nsample, mlp, mlp2, group_all, is_training,
                       bn_decay, scope, bn=True, pooling='max', knn=False, use_xyz=True,
                       use_nchw=False, params=None):
    """pointnet_util.py:90-163. Returns (new_xyz (B,npoint,3), new_points (B,npoint,mlp[-1] or
    mlp2[-1]), idx (B,npoint,nsample)). Variables come from `params` (tf_util.ParamStore,
    default tf_util.default_store()) under '<scope>/conv<i>/...' and '<scope>/conv_post_<i>/...'.

    Inference (is_training False, no autograd): FPS + ball query, then ONE kernel for group,
    MLP and pooling (pn2_group_mlp), and mlp2 as a per-point MLP. Training: the same ops
    composed from differentiable torch ops (batch-statistics batch norm)."""
    store = params if params is not None else tf_util.default_store()
    xyz = device_tensor(xyz, "xyz", torch.float32)
    scopes = [f"{scope}/conv{i}" for i in range(len(mlp))]
    post = [f"{scope}/conv_post_{i}" for i in range(len(mlp2 or []))]
    if group_all:
        new_xyz, new_points, idx, grouped_xyz = sample_and_group_all(xyz, points, use_xyz)
    elif is_training or _needs_grad(xyz, points) or knn:
        new_xyz, new_points, idx, grouped_xyz = sample_and_group(npoint, radius, nsample, xyz,
                                                                 points, knn, use_xyz)
    else:
        _, new_xyz = tf_sampling.farthest_point_sample_and_gather(npoint, xyz)
        idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz)
        new_points = None
    cin = (0 if _is_empty_points(points) else int(points.shape[2])) + (
        3 if (use_xyz or _is_empty_points(points)) else 0)
    if is_training or _needs_grad(xyz, points):
        layers = tf_util.torch_layers(store, scopes, cin, mlp, bn=bn)
        x = tf_util.mlp_torch(new_points, layers, is_training, bn_decay)
        x = _pool_torch(x, pooling, grouped_xyz)
        if mlp2:
            c = int(x.shape[-1])
            x = tf_util.mlp_torch(x, tf_util.torch_layers(store, post, c, mlp2, bn=bn),
                                  is_training, bn_decay)
        return new_xyz, x, idx
    fused = tf_util.packed_mlp(store, scopes, cin, mlp, bn=bn)
    # group_all: one group of all N points centred on (0,0,0) (pointnet_util.py:72-87)
    x = group_mlp(xyz, points, new_xyz, idx, fused, pooling, use_xyz=use_xyz)
    if mlp2:
        c = int(x.shape[-1])
        x = tf_util.packed_mlp(store, post, c, mlp2, bn=bn)(x)
    return new_xyz, x, idx


def pointnet_sa_module_msg(xyz, points, npoint, radius_list, nsample_list, mlp_list,
                           is_training, bn_decay, scope, bn=True, use_xyz=True, use_nchw=False,
                           params=None):
    """pointnet_util.py:166-201: one FPS, then per scale i a ball query and the fused
    group ([points, xyz] order, :191) + MLP ('<scope>/conv<i>_<j>') + max pool; the scales'
    features are concatenated. Returns (new_xyz, new_points_concat)."""
    store = params if params is not None else tf_util.default_store()
    xyz = device_tensor(xyz, "xyz", torch.float32)
    training = is_training or _needs_grad(xyz, points)
    if training:
        new_xyz = tf_sampling.gather_point(xyz, tf_sampling.farthest_point_sample(npoint, xyz))
    else:
        _, new_xyz = tf_sampling.farthest_point_sample_and_gather(npoint, xyz)
    C = 0 if _is_empty_points(points) else int(points.shape[2])
    cin = C + (3 if (use_xyz or C == 0) else 0)
    outs = []
    for i, (radius, nsample) in enumerate(zip(radius_list, nsample_list)):
        scopes = [f"{scope}/conv{i}_{j}" for j in range(len(mlp_list[i]))]
        idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz.detach())
        if training:
            gp, _ = group_concat(xyz, points, new_xyz, idx, use_xyz=use_xyz, xyz_last=True)
            layers = tf_util.torch_layers(store, scopes, cin, mlp_list[i], bn=bn)
            outs.append(tf_util.mlp_torch(gp, layers, is_training, bn_decay).max(dim=2).values)
        else:
            fused = tf_util.packed_mlp(store, scopes, cin, mlp_list[i], bn=bn)
            outs.append(group_mlp(xyz, points, new_xyz, idx, fused, "max", use_xyz=use_xyz,
                                  xyz_last=True))
    return new_xyz, torch.cat(outs, dim=-1)


def pointnet_fp_module(xyz1, xyz2, points1, points2, mlp, is_training, bn_decay, scope, bn=True,
                       params=None, known_grid=None, unknown_grid=None):
    """pointnet_util.py:204-238: three_nn, IDW weights, three_interpolate, concat
    [interp, points1], MLP ('<scope>/conv_<i>'). Inference: three_nn (grid search when large)
    then ONE kernel for weights + interpolation + concat + MLP (pn2_fp_mlp)."""
    store = params if params is not None else tf_util.default_store()
    xyz1 = device_tensor(xyz1, "xyz1", torch.float32)
    xyz2 = device_tensor(xyz2, "xyz2", torch.float32)
    points2 = device_tensor(points2, "points2", torch.float32)
    scopes = [f"{scope}/conv_{i}" for i in range(len(mlp))]
    C1 = 0 if points1 is None else int(points1.shape[2])
    C2 = int(points2.shape[2])
    if is_training or _needs_grad(points1, points2):
        x = fp_interpolate(xyz1, xyz2, points1, points2, known_grid, unknown_grid)
        layers = tf_util.torch_layers(store, scopes, C1 + C2, mlp, bn=bn)
        return tf_util.mlp_torch(x, layers, is_training, bn_decay)
    fused = tf_util.packed_mlp(store, scopes, C1 + C2, mlp, bn=bn)
    dist, idx = tf_interpolate.three_nn(xyz1, xyz2, known_grid, unknown_grid)
    return fp_mlp(dist, idx, points1, points2, fused)


def fp_mlp(dist, idx, points1, points2, mlp):
    """pointnet_fp_module after three_nn: IDW weights of dist (B,n,3), interpolation of
    points2 (B,m,C2) at idx, concat [interp, points1 (B,n,C1) or None], then the fused MLP
    `mlp` (tf_util.SharedMLP) -> (B, n, mlp.cout) (pn2_fp_mlp, one kernel)."""
    dist = device_tensor(dist, "dist", torch.float32)
    idx = device_tensor(idx, "idx", torch.int32)
    points2 = device_tensor(points2, "points2", torch.float32)
    B, n, m, C2 = int(dist.shape[0]), int(dist.shape[1]), int(points2.shape[1]), int(points2.shape[2])
    if points1 is not None:
        points1 = device_tensor(points1, "points1", torch.float32)
    C1 = 0 if points1 is None else int(points1.shape[2])
    out = torch.empty((B, n, mlp.cout), dtype=torch.float32, device=dist.device)
    tab, nl = mlp.table()
    check(lib().pn2_fp_mlp(ptr(dist), ptr(idx), ptr(points1), C1, ptr(points2), C2, B, n, m, nl,
                           tab, ptr(out), stream_of(dist)), "fp_mlp")
    return out
