"""Python front of the oracle — TEST INFRASTRUCTURE ONLY.

Loads
  oracle/liboracle.so          our C restatement (pn2_oracle.c), numpy in / numpy out
  oracle/_ref/libref_cpu.so    the reference's own CPU code (query_ball_point.cpp,
                               interpolate.cpp, tf_interpolate.cpp:57-103), compiled unchanged
  oracle/_ref/libref_gpu.so    the reference's own CUDA kernels (tf_sampling_g.cu,
                               tf_grouping_g.cu) compiled unchanged for gfx950 (GPU box only)
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker / CPU baseline. The product never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_CPU_SO = os.path.join(HERE, "_ref", "libref_cpu.so")
REF_GPU_SO = os.path.join(HERE, "_ref", "libref_gpu.so")

_P, _I, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float

_ORACLE_SIGS = {
    "pn2o_selection_sort": [_P, _I, _I, _I, _I, _P, _P],
    "pn2o_knn_point": [_P, _P, _I, _I, _I, _I, _I, _P, _P],
    "pn2o_prob_sample": [_P, _P, _I, _I, _I, _P],
    "pn2o_set_threads": [_I],
    "pn2o_fps": [_P, _I, _I, _I, _P],
    "pn2o_gather_point": [_P, _P, _I, _I, _I, _P],
    "pn2o_gather_point_grad": [_P, _P, _I, _I, _I, _P],
    "pn2o_ball_query": [_P, _P, _I, _I, _I, _F, _I, _P, _P],
    "pn2o_group_point": [_P, _P, _I, _I, _I, _I, _I, _P],
    "pn2o_group_point_grad": [_P, _P, _I, _I, _I, _I, _I, _P],
    "pn2o_group_concat": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P],
    "pn2o_three_nn": [_P, _P, _I, _I, _I, _P, _P],
    "pn2o_three_interpolate": [_P, _P, _P, _I, _I, _I, _I, _P],
    "pn2o_three_interpolate_grad": [_P, _P, _P, _I, _I, _I, _I, _P],
    "pn2o_idw_weights": [_P, _I, _I, _P],
    "pn2o_fp_fused": [_P, _P, _P, _I, _P, _I, _I, _I, _I, _P],
    "pn2o_attn_reduce": [_P, _P, _P, _I, _I, _I, _I, _P],
    "pn2o_group_pool": [_P, _P, _I, _I, _I, _I, _I, _P],
}
_REF_CPU_SIGS = {
    "pn2ref_query_ball_point": [_I, _I, _I, _F, _I, _P, _P, _P],
    "pn2ref_group_point": [_I, _I, _I, _I, _I, _P, _P, _P],
    "pn2ref_group_point_grad": [_I, _I, _I, _I, _I, _P, _P, _P],
    "pn2ref_three_nn": [_I, _I, _I, _P, _P, _P, _P],
    "pn2ref_three_interpolate": [_I, _I, _I, _I, _P, _P, _P, _P],
    "pn2ref_three_interpolate_grad": [_I, _I, _I, _I, _P, _P, _P, _P],
}
_REF_GPU_SIGS = {
    "pn2ref_selection_sort": [_P, _I, _I, _I, _I, _P, _P],
    "pn2ref_fps": [_P, _I, _I, _I, _P],
    "pn2ref_prob_sample": [_P, _P, _I, _I, _I, _P],
    "pn2ref_gather_point": [_P, _P, _I, _I, _I, _P],
    "pn2ref_query_ball_point": [_P, _P, _I, _I, _I, _F, _I, _P, _P],
    "pn2ref_group_point": [_P, _P, _I, _I, _I, _I, _I, _P],
}

_cache = {}


def build(ref=False):
    """make -C oracle (and the _ref targets when /root/reference is present and ref=True)."""
    targets = ["all"]
    if ref and os.path.isdir("/root/reference"):
        targets.append("ref")
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def _load(path, sigs, restype=None):
    if path not in _cache:
        if not os.path.exists(path):
            if path == ORACLE_SO:
                build()
            else:
                raise FileNotFoundError(f"{path} not built (make -C oracle ref, needs /root/reference)")
        lib = ctypes.CDLL(path)
        for name, args in sigs.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = restype
        _cache[path] = lib
    return _cache[path]


def olib():
    return _load(ORACLE_SO, _ORACLE_SIGS)


def ref_cpu():
    return _load(REF_CPU_SO, _REF_CPU_SIGS)


def ref_gpu():
    return _load(REF_GPU_SO, _REF_GPU_SIGS, restype=_I)


def have_ref_cpu():
    return os.path.exists(REF_CPU_SO)


def have_ref_gpu():
    return os.path.exists(REF_GPU_SO)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _p(a):
    return None if a is None else a.ctypes.data


def set_threads(n):
    olib().pn2o_set_threads(int(n))


# ---------------------------------------------------------------- restatement (numpy API)

def fps(xyz, npoint):
    xyz = _f32(xyz)
    B, N = xyz.shape[:2]
    idx = np.zeros((B, npoint), np.int32)
    olib().pn2o_fps(_p(xyz), B, N, npoint, _p(idx))
    return idx


def gather_point(inp, idx):
    inp, idx = _f32(inp), _i32(idx)
    B, N = inp.shape[:2]
    M = idx.shape[1]
    out = np.zeros((B, M, 3), np.float32)
    olib().pn2o_gather_point(_p(inp), _p(idx), B, N, M, _p(out))
    return out


def gather_point_grad(N, idx, out_g):
    idx, out_g = _i32(idx), _f32(out_g)
    B, M = idx.shape
    g = np.zeros((B, N, 3), np.float32)
    olib().pn2o_gather_point_grad(_p(out_g), _p(idx), B, N, M, _p(g))
    return g


def ball_query(xyz1, xyz2, radius, nsample):
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    B, N = xyz1.shape[:2]
    M = xyz2.shape[1]
    idx = np.zeros((B, M, nsample), np.int32)
    cnt = np.zeros((B, M), np.int32)
    olib().pn2o_ball_query(_p(xyz1), _p(xyz2), B, N, M, float(radius), nsample, _p(idx), _p(cnt))
    return idx, cnt


def group_point(points, idx):
    points, idx = _f32(points), _i32(idx)
    B, N, C = points.shape
    M, ns = idx.shape[1:]
    out = np.zeros((B, M, ns, C), np.float32)
    olib().pn2o_group_point(_p(points), _p(idx), B, N, C, M, ns, _p(out))
    return out


def group_point_grad(N, idx, grad_out):
    idx, grad_out = _i32(idx), _f32(grad_out)
    B, M, ns, C = grad_out.shape
    g = np.zeros((B, N, C), np.float32)
    olib().pn2o_group_point_grad(_p(grad_out), _p(idx), B, N, C, M, ns, _p(g))
    return g


def group_concat(xyz, points, new_xyz, idx, use_xyz=True, xyz_last=False):
    xyz, new_xyz, idx = _f32(xyz), _f32(new_xyz), _i32(idx)
    B, N = xyz.shape[:2]
    M, ns = idx.shape[1:]
    if points is None:
        C, Cout = 0, 3
    else:
        points = _f32(points)
        C = points.shape[2]
        Cout = C + 3 if use_xyz else C
    gx = np.zeros((B, M, ns, 3), np.float32)
    out = np.zeros((B, M, ns, Cout), np.float32)
    flags = (1 if use_xyz else 0) | (2 if xyz_last else 0)
    olib().pn2o_group_concat(_p(xyz), _p(points), _p(new_xyz), _p(idx), B, N, C, M, ns, flags,
                             _p(gx), _p(out))
    return out, gx


def three_nn(xyz1, xyz2):
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    B, n = xyz1.shape[:2]
    m = xyz2.shape[1]
    dist = np.zeros((B, n, 3), np.float32)
    idx = np.zeros((B, n, 3), np.int32)
    olib().pn2o_three_nn(_p(xyz1), _p(xyz2), B, n, m, _p(dist), _p(idx))
    return dist, idx


def three_interpolate(points, idx, weight):
    points, idx, weight = _f32(points), _i32(idx), _f32(weight)
    B, m, C = points.shape
    n = idx.shape[1]
    out = np.zeros((B, n, C), np.float32)
    olib().pn2o_three_interpolate(_p(points), _p(idx), _p(weight), B, m, C, n, _p(out))
    return out


def three_interpolate_grad(m, idx, weight, grad_out):
    idx, weight, grad_out = _i32(idx), _f32(weight), _f32(grad_out)
    B, n, C = grad_out.shape
    g = np.zeros((B, m, C), np.float32)
    olib().pn2o_three_interpolate_grad(_p(grad_out), _p(idx), _p(weight), B, n, C, m, _p(g))
    return g


def idw_weights(dist):
    dist = _f32(dist)
    B, n = dist.shape[:2]
    w = np.zeros_like(dist)
    olib().pn2o_idw_weights(_p(dist), B, n, _p(w))
    return w


def fp_fused(xyz1, xyz2, points1, points2):
    xyz1, xyz2, points2 = _f32(xyz1), _f32(xyz2), _f32(points2)
    B, n = xyz1.shape[:2]
    m, C2 = xyz2.shape[1], points2.shape[2]
    C1 = 0 if points1 is None else points1.shape[2]
    if points1 is not None:
        points1 = _f32(points1)
    out = np.zeros((B, n, C1 + C2), np.float32)
    olib().pn2o_fp_fused(_p(xyz1), _p(xyz2), _p(points1), C1, _p(points2), C2, B, n, m, _p(out))
    return out


def attn_reduce(Q, K, V):
    Q, K, V = _f32(Q), _f32(K), _f32(V)
    B, M, ns, C = K.shape
    out = np.zeros((B, M, C), np.float32)
    olib().pn2o_attn_reduce(_p(Q), _p(K), _p(V), B, M, ns, C, _p(out))
    return out


def group_pool(x, grouped_xyz, mode):
    modes = {"max": 0, "avg": 1, "weighted_avg": 2, "max_and_avg": 3}
    x = _f32(x)
    B, M, ns, C = x.shape
    g = _f32(grouped_xyz) if grouped_xyz is not None else None
    Cout = 2 * C if mode == "max_and_avg" else C
    out = np.zeros((B, M, 1, Cout), np.float32)
    olib().pn2o_group_pool(_p(x), _p(g), B, M, ns, C, modes[mode], _p(out))
    return out


# ---------------------------------------------------------------- shared MLP (float64)
# The dense half of pointnet_sa_module / pointnet_fp_module restated in numpy float64: the bar
# for the fp32 matrix-core kernels of csrc/mlp.hip (floating point: within a tolerance, stated
# in tests/test_gpu_mlp.py).

BN_EPSILON = 1e-3  # tf.contrib.layers.batch_norm default (tf_util.py:527-531)


def mlp_f64(x, layers):
    """tf_util.conv2d 1x1 in inference mode, layer by layer (tf_util.py:165-185):
    y = act(((x W) + b - moving_mean) * gamma / sqrt(moving_variance + eps) + beta).
    layers: dicts with weights (cin,cout) [, biases, gamma, beta, moving_mean,
    moving_variance], relu (bool)."""
    y = np.asarray(x, np.float64)
    for L in layers:
        y = y @ np.asarray(L["weights"], np.float64)
        if L.get("biases") is not None:
            y = y + np.asarray(L["biases"], np.float64)
        if L.get("gamma") is not None:
            g = np.asarray(L["gamma"], np.float64)
            mean = np.asarray(L["moving_mean"], np.float64)
            var = np.asarray(L["moving_variance"], np.float64)
            y = (y - mean) * (g / np.sqrt(var + BN_EPSILON)) + np.asarray(L["beta"], np.float64)
        if L.get("relu", True):
            y = np.maximum(y, 0.0)
    return y


def pool_f64(x, grouped_xyz, mode):
    """Pooling over nsample (pointnet_util.py:130-145), x (B,M,ns,C) -> (B,M,C')."""
    x = np.asarray(x, np.float64)
    if mode == "max":
        return x.max(axis=2)
    if mode == "avg":
        return x.mean(axis=2)
    if mode == "weighted_avg":
        d = np.sqrt((np.asarray(grouped_xyz, np.float64) ** 2).sum(-1, keepdims=True))
        e = np.exp(-d * 5)
        return (x * (e / e.sum(axis=2, keepdims=True))).sum(axis=2)
    if mode == "max_and_avg":
        return np.concatenate([x.mean(axis=2), x.max(axis=2)], axis=-1)
    raise ValueError(mode)


# ---------------------------------------------------------------- reference CPU code

def ref_ball_query(xyz1, xyz2, radius, nsample, fill=-1):
    """query_ball_point_cpu (query_ball_point.cpp:19-47). idx rows of queries with no hit keep
    `fill` (the reference leaves them uninitialised)."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    B, N = xyz1.shape[:2]
    M = xyz2.shape[1]
    idx = np.full((B, M, nsample), fill, np.int32)
    ref_cpu().pn2ref_query_ball_point(B, N, M, float(radius), nsample, _p(xyz1), _p(xyz2), _p(idx))
    return idx


def ref_group_point(points, idx):
    points, idx = _f32(points), _i32(idx)
    B, N, C = points.shape
    M, ns = idx.shape[1:]
    out = np.zeros((B, M, ns, C), np.float32)
    ref_cpu().pn2ref_group_point(B, N, C, M, ns, _p(points), _p(idx), _p(out))
    return out


def ref_group_point_grad(N, idx, grad_out):
    idx, grad_out = _i32(idx), _f32(grad_out)
    B, M, ns, C = grad_out.shape
    g = np.zeros((B, N, C), np.float32)  # the CPU twin accumulates into caller memory
    ref_cpu().pn2ref_group_point_grad(B, N, C, M, ns, _p(grad_out), _p(idx), _p(g))
    return g


def ref_three_nn(xyz1, xyz2):
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    B, n = xyz1.shape[:2]
    m = xyz2.shape[1]
    dist = np.zeros((B, n, 3), np.float32)
    idx = np.zeros((B, n, 3), np.int32)
    ref_cpu().pn2ref_three_nn(B, n, m, _p(xyz1), _p(xyz2), _p(dist), _p(idx))
    return dist, idx


def ref_three_interpolate(points, idx, weight):
    points, idx, weight = _f32(points), _i32(idx), _f32(weight)
    B, m, C = points.shape
    n = idx.shape[1]
    out = np.zeros((B, n, C), np.float32)
    ref_cpu().pn2ref_three_interpolate(B, m, C, n, _p(points), _p(idx), _p(weight), _p(out))
    return out


def ref_three_interpolate_grad(m, idx, weight, grad_out):
    idx, weight, grad_out = _i32(idx), _f32(weight), _f32(grad_out)
    B, n, C = grad_out.shape
    g = np.zeros((B, m, C), np.float32)
    ref_cpu().pn2ref_three_interpolate_grad(B, n, C, m, _p(grad_out), _p(idx), _p(weight), _p(g))
    return g


# ---------------------------------------------------------------- the geometric stack on CPU

def selection_sort(dist, k):
    """select_top_k(k, dist) -> (outi, out), both (B,m,n) (tf_grouping.py:22-31)."""
    dist = _f32(dist)
    B, m, n = dist.shape
    outi = np.zeros((B, m, n), np.int32)
    out = np.zeros((B, m, n), np.float32)
    olib().pn2o_selection_sort(_p(dist), B, m, n, int(k), _p(outi), _p(out))
    return outi, out


def knn_point(k, xyz1, xyz2):
    """knn_point(k, xyz1, xyz2) -> (val, idx), (B,m,k) (tf_grouping.py:48-73)."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    B, n, c = xyz1.shape
    m = xyz2.shape[1]
    val = np.zeros((B, m, k), np.float32)
    idx = np.zeros((B, m, k), np.int32)
    olib().pn2o_knn_point(_p(xyz1), _p(xyz2), B, n, m, c, int(k), _p(val), _p(idx))
    return val, idx


def prob_sample(inp, inpr):
    """prob_sample(inp (B,n), inpr (B,m)) -> (B,m) int32 (tf_sampling.py:14-23)."""
    inp, inpr = _f32(inp), _f32(inpr)
    B, n = inp.shape
    m = inpr.shape[1]
    out = np.zeros((B, m), np.int32)
    if B and m:
        olib().pn2o_prob_sample(_p(inp), _p(inpr), B, n, m, _p(out))
    return out


def run_stack_cpu(inp_np, config, intermediates=False):
    """The same step as stack.run(), on the CPU restatement (numpy inputs).

    intermediates=True returns (outs, labels, inter): labels[k] names outs[k] and says how it
    is compared -- ("sa<i>.new_points", None) and ("sa<i>_<r>.new_points", None) are copies
    (bit-exact), ("sa<i>.attn", "tol") floating point, ("fp<k>.out", C2) the FP output whose
    first C2 columns are interpolated (1e-5) and the rest a copy of points1 (bit-exact);
    inter holds the step's index results by Step.intermediates() names."""
    import importlib
    stack = importlib.import_module("pointcloud-segmentation-attention_amd.stack")
    kind = stack.CONFIGS[config][1]
    outs, labels, inter = [], [], {}
    if kind == "ssg":
        xyz, points = [inp_np["xyz"]], [inp_np["feats"]]
        for i, (npoint, radius, nsample, _) in enumerate(stack.SSG_SA):
            idx = fps(xyz[-1], npoint)
            new_xyz = gather_point(xyz[-1], idx)
            gidx, _ = ball_query(xyz[-1], new_xyz, radius, nsample)
            inter[f"fps{i + 1}.idx"], inter[f"fps{i + 1}.new_xyz"] = idx, new_xyz
            inter[f"bq{i + 1}.idx"] = gidx
            new_points, _ = group_concat(xyz[-1], points[-1], new_xyz, gidx)
            outs.append(new_points)
            labels.append((f"sa{i + 1}.new_points", None))
            if "attn" in inp_np:
                outs.append(attn_reduce(*inp_np["attn"][i]))
                labels.append((f"sa{i + 1}.attn", "tol"))
            xyz.append(new_xyz)
            points.append(inp_np["sa_out"][i])
        feat = inp_np["sa_out"][3]
        for k in range(4):
            lvl = 3 - k
            d, ni = three_nn(xyz[lvl], xyz[lvl + 1])
            inter[f"nn{k + 1}.dist"], inter[f"nn{k + 1}.idx"] = d, ni
            outs.append(fp_fused(xyz[lvl], xyz[lvl + 1], points[lvl], feat))
            labels.append((f"fp{k + 1}.out", int(feat.shape[-1])))
            feat = inp_np["fp_out"][k] if k < 3 else None
    else:
        xyz, points = inp_np["xyz"], None
        for i, (npoint, radii, nsamples, _) in enumerate(stack.MSG_SA):
            idx = fps(xyz, npoint)
            new_xyz = gather_point(xyz, idx)
            inter[f"fps{i + 1}.idx"], inter[f"fps{i + 1}.new_xyz"] = idx, new_xyz
            for r, (radius, nsample) in enumerate(zip(radii, nsamples)):
                gidx, _ = ball_query(xyz, new_xyz, radius, nsample)
                inter[f"bq{i + 1}_{r}.idx"] = gidx
                outs.append(group_concat(xyz, points, new_xyz, gidx, xyz_last=True)[0])
                labels.append((f"sa{i + 1}_{r}.new_points", None))
            xyz, points = new_xyz, inp_np["sa_out"][0]
    return (outs, labels, inter) if intermediates else outs


def _bits32(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def compare_stack(inp_np, config, outs, inter, rtol=1e-5, atol=1e-5):
    """The CHECKER of a step (tests/, bench.py's `verified` field): every output and index
    intermediate of one step (numpy arrays, Step.outputs() / Step.intermediates() order and
    names) against run_stack_cpu on the same inputs, each with the bar north_star sets --
    bit-exact for indices and copies, rtol = atol = 1e-5 for the interpolated FP columns and the
    attention reduction. Returns a list of failure strings (empty = parity)."""
    ref, labels, rinter = run_stack_cpu(inp_np, config, intermediates=True)
    bad = []
    if len(outs) != len(ref):
        return [f"{len(outs)} outputs, oracle has {len(ref)}"]

    def exact(name, g, r):
        if g.shape != r.shape:
            bad.append(f"{name}: shape {g.shape} vs {r.shape}")
            return
        d = (g != r) if (g.dtype == np.int32 or r.dtype == np.int32) else (_bits32(g) != _bits32(r))
        if d.any():
            bad.append(f"{name}: {int(d.sum())} of {d.size} values differ (bit-exact bar)")

    def close(name, g, r):
        if g.shape != r.shape:
            bad.append(f"{name}: shape {g.shape} vs {r.shape}")
        elif not np.allclose(g, r, rtol=rtol, atol=atol):
            err = np.abs(g.astype(np.float64) - r) - atol - rtol * np.abs(r)
            bad.append(f"{name}: {int((err > 0).sum())} values outside rtol=atol=1e-5")

    for g, r, (name, how) in zip(outs, ref, labels):
        if how is None:
            exact(name, g, r)
        elif how == "tol":
            close(name, g, r)
        else:  # FP output: [interpolated (C2 columns), points1 copy]
            close(name + "[:C2] interpolated", g[..., :how], r[..., :how])
            exact(name + "[C2:] points1 copy", g[..., how:], r[..., how:])
    if not inter:
        bad.append("the step recorded no intermediates")
    for name, t in inter.items():
        exact(name, t, rinter[name])
    for name in rinter:
        if name.startswith(("fps", "bq")) and name not in inter:
            bad.append(f"{name} missing from the step's intermediates")
    return bad


# ---------------------------------------------------------------- scene crops (numpy)
# data_transformation.py:70-154 (get_subset) restated in numpy with TF's float32 semantics, for
# caller-supplied random draws (test infrastructure: the crop sampler kernels' bar). TensorFlow
# is not importable here, so this restatement is "parity unpinned" beyond its own reading of the
# reference text; the scene CHUNKER (complete_scene_loader.py) is pinned to the reference
# function itself through tests/golden/scene_chunks_*.npz.

GET_SUBSET_LABEL_WEIGHTS = [0, 2.743064592944318, 3.0830506790927132, 4.785754459526457,
                            4.9963745147506184, 4.372710774561782, 5.039124880965811,
                            4.86451825464344, 4.717751595568025, 4.809412839311939,
                            5.052097251455304, 5.389129668645318, 5.390614085649042,
                            5.127458225110977, 5.086056870814752, 5.3831185190895265,
                            5.422684124268539, 5.422955391988761, 5.433705358072363,
                            5.417426773812747, 4.870172044153657]  # data_transformation.py:82-86


def crop_sample(points, labels, colors, normals, centres, u, label_weights=None):
    """One crop: centres (T,) point indices of the tries, u (K,) uniform draws.
    Returns points, labels, colors, normals, sample_weight, chosen try, stats (T,3)."""
    f32 = np.float32
    p = np.asarray(points, f32)
    lw = np.asarray(GET_SUBSET_LABEL_WEIGHTS if label_weights is None else label_weights, f32)
    mn, mx = p.min(0), p.max(0)  # :90-91
    T = len(centres)
    chosen, stats = T - 1, []

    def area(t):
        c = p[centres[t]]
        lo = np.array([c[0] - f32(0.75), c[1] - f32(0.75), mn[2]], f32)  # :98-103
        hi = np.array([c[0] + f32(0.75), c[1] + f32(0.75), mx[2]], f32)
        return lo, hi

    for t in range(T):
        lo, hi = area(t)
        inarea = np.all((p >= lo - f32(0.2)) & (hi + f32(0.2) > p), axis=1)  # :105-106
        cur = p[inarea]
        n = len(cur)
        lab = int((np.asarray(labels)[inarea] > 0).sum())
        m = np.all((cur >= lo - f32(0.01)) & (hi + f32(0.01) > cur), axis=1)  # :114-117
        v = np.ceil(((cur[m] - lo) / (hi - lo)) * np.array([31, 31, 62], f32))  # :119-120
        key = (v[:, 0] * f32(31.0)) * f32(62.0) + v[:, 1] * f32(62) + v[:, 2]   # :121
        occ = len(np.unique(key))
        stats.append((n, lab, occ))
        cur_len = f32(3 * n)  # reduce_sum(ones_like((n,3) cur_points)) (:113)
        with np.errstate(invalid="ignore", divide="ignore"):
            valid = (f32(lab) / cur_len >= f32(0.7)) and \
                (f32(f32(f32(f32(occ) / f32(31.0)) / f32(31.0)) / f32(62.0)) >= f32(0.02))
        if valid:
            chosen = t
            break
    lo, hi = area(chosen)
    inarea = np.all((p >= lo - f32(0.2)) & (hi + f32(0.2) > p), axis=1)
    sel = np.nonzero(inarea)[0]
    n = len(sel)
    mask = np.all((p[sel] >= lo - f32(0.01)) & (hi + f32(0.01) > p[sel]), axis=1)
    k = (np.asarray(u, f32) * f32(n)).astype(np.int64)  # random_uniform(0, cur_len) -> int32
    k = np.clip(k, 0, n - 1)
    idx = sel[k]
    lab = np.asarray(labels)[idx]
    w = lw[lab] * mask[k].astype(f32)  # :152-153
    return (p[idx], lab, None if colors is None else np.asarray(colors)[idx],
            None if normals is None else np.asarray(normals)[idx], w, chosen,
            np.array(stats + [(0, 0, 0)] * (T - len(stats)), np.int64))
