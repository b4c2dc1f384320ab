"""GPU parity of the fused shared-MLP kernels (csrc/mlp.hip) through the C ABI.

The MLP is floating-point work (fp32 products and sums on the matrix cores), so it is held to
a tolerance against the float64 restatement oracle.mlp_f64 / pool_f64 (tf_util.py:165-185,
pointnet_util.py:130-145) applied to the oracle's bit-exact grouping / interpolation:

    max |gpu - f64|  <=  max(4 * max |numpy_fp32 - f64|,  1e-6 * (1 + max |f64|))

i.e. no worse than 4x the error of a plain fp32 evaluation of the same layers on the CPU
(numpy sgemm), with a floor of 1e-6 relative. The grouped / interpolated inputs themselves are
bit-identical to pn2_group_concat / pn2_fp_apply (tested in test_gpu_parity.py).
"""
import importlib

import numpy as np
import pytest

from conftest import PKG_NAME, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


@pytest.fixture(scope="module")
def env():
    import torch

    from oracle import oracle as O
    O.set_threads(16)
    pkg = importlib.import_module(PKG_NAME)
    return pkg, O, torch, torch.device("cuda:0")


def make_layers(rng, cin, widths, bn=True, relu=True, last_relu=None, last_bn=None):
    layers, c = [], cin
    for i, w in enumerate(widths):
        last = i == len(widths) - 1
        use_bn = bn if not (last and last_bn is not None) else last_bn
        use_relu = relu if not (last and last_relu is not None) else last_relu
        lim = np.sqrt(6.0 / (c + w))
        L = {"weights": rng.uniform(-lim, lim, (c, w)).astype(np.float32),
             "biases": rng.uniform(-0.1, 0.1, w).astype(np.float32), "relu": use_relu}
        if use_bn:
            L.update(gamma=rng.uniform(0.5, 1.5, w).astype(np.float32),
                     beta=rng.uniform(-0.2, 0.2, w).astype(np.float32),
                     moving_mean=rng.uniform(-0.1, 0.1, w).astype(np.float32),
                     moving_variance=rng.uniform(0.5, 2.0, w).astype(np.float32))
        layers.append(L)
        c = w
    return layers


def fused(pkg, layers):
    tu = pkg.tf_util
    return tu.SharedMLP([tu.PackedLayer(L["weights"], L["biases"], L.get("gamma"), L.get("beta"),
                                        L.get("moving_mean"), L.get("moving_variance"),
                                        relu=L["relu"]) for L in layers])


def mlp_f32(x, layers):
    """The same layers in numpy float32 (the error yardstick of the tolerance)."""
    y = np.asarray(x, np.float32)
    for L in layers:
        y = y @ L["weights"] + L["biases"]
        if L.get("gamma") is not None:
            s = (L["gamma"].astype(np.float64) / np.sqrt(L["moving_variance"].astype(np.float64)
                                                         + 1e-3))
            t = L["beta"] - L["moving_mean"] * s
            y = (y * s.astype(np.float32) + t.astype(np.float32)).astype(np.float32)
        if L["relu"]:
            y = np.maximum(y, 0)
    return y


def assert_close(got, ref64, ref32, what):
    got = np.asarray(got, np.float64)
    err = np.abs(got - ref64).max() if got.size else 0.0
    err32 = np.abs(np.asarray(ref32, np.float64) - ref64).max() if got.size else 0.0
    tol = max(4 * err32, 1e-6 * (1 + np.abs(ref64).max() if got.size else 1.0))
    assert got.shape == ref64.shape, (got.shape, ref64.shape)
    assert np.isfinite(got).all(), f"{what}: non-finite outputs"
    assert err <= tol, f"{what}: max err {err:.3g} > tol {tol:.3g} (fp32 numpy err {err32:.3g})"


MLP_CASES = [
    (1000, 3, [32, 32, 64], {}),                       # SA1 widths, ragged rows
    (77, 259, [256, 256, 512], {}),                    # SA4 widths
    (4099, 128, [128, 128, 128, 128, 21],              # FP4 + fc1 + fc2 head (no BN/relu)
     dict(last_relu=False, last_bn=False)),
    (64, 768, [256, 256], {}),                         # FP1
    (33, 9, [64], {}),
    (5, 1030, [1024], dict(bn=False)),
    (300, 67, [64, 96, 128], dict(relu=False)),
]


@pytest.mark.parametrize("rows,cin,widths,kw", MLP_CASES)
def test_shared_mlp_vs_f64(env, rows, cin, widths, kw):
    pkg, O, torch, dev = env
    rng = np.random.default_rng(rows * 31 + cin)
    layers = make_layers(rng, cin, widths, **kw)
    x = rng.uniform(-1, 1, (rows, cin)).astype(np.float32)
    got = fused(pkg, layers)(torch.from_numpy(x).to(dev)).cpu().numpy()
    assert_close(got, O.mlp_f64(x, layers), mlp_f32(x, layers), "shared_mlp")


def _sa_inputs(pkg, O, B, N, M, C, radius, ns, seed):
    xyz, feats = pkg.synth.batch(range(seed, seed + B), N, "scannet", with_features=True)
    rng = np.random.default_rng(seed)
    if C == 6:
        points = feats
    elif C > 0:
        points = rng.uniform(-1, 1, (B, N, C)).astype(np.float32)
    else:
        points = None
    fidx = O.fps(xyz, M)
    new_xyz = O.gather_point(xyz, fidx)
    idx, _ = O.ball_query(xyz, new_xyz, radius, ns)
    return xyz, points, new_xyz, idx


GROUP_CASES = [
    # (C, ns, pooling, use_xyz, xyz_last, widths)
    (0, 32, "max", True, False, [32, 32, 64]),         # SSG SA1 (xyz only)
    (6, 32, "max", True, False, [32, 32, 64]),         # cfg3 SA1 (rgb + normals)
    (64, 32, "max", True, False, [64, 64, 128]),       # SA2
    (64, 16, "max", True, True, [32, 32, 64]),         # MSG order, ns 16 (two groups per tile)
    (64, 64, "max", True, True, [64, 64, 128]),        # ns 64 (a group spans two tiles)
    (64, 128, "max", True, True, [64, 96, 128]),       # ns 128
    (32, 5, "max", True, False, [32, 64]),             # ns 5 (padded to 8)
    (32, 24, "avg", True, False, [32, 64]),            # ns 24 (padded to 32)
    (32, 32, "avg", True, False, [64, 64]),
    (32, 32, "weighted_avg", True, False, [64, 64]),
    (32, 128, "weighted_avg", True, False, [64, 64]),  # weights over a multi-pass group
    (32, 32, "max_and_avg", True, False, [64, 64]),
    (32, 16, "max", False, False, [64, 64]),           # use_xyz=False
    (16, 32, None, True, False, [32, 32, 64]),         # per-point output (attention input)
    (16, 128, None, True, True, [64]),
]


@pytest.mark.parametrize("C,ns,pooling,use_xyz,xyz_last,widths", GROUP_CASES)
def test_group_mlp_vs_f64(env, C, ns, pooling, use_xyz, xyz_last, widths):
    pkg, O, torch, dev = env
    B, N, M, radius = 2, 2048, 96, 0.2
    xyz, points, new_xyz, idx = _sa_inputs(pkg, O, B, N, M, C, radius, ns, seed=ns + C)
    grouped, gxyz = O.group_concat(xyz, points, new_xyz, idx, use_xyz=use_xyz,
                                   xyz_last=xyz_last)
    rng = np.random.default_rng(7 * ns + C)
    layers = make_layers(rng, grouped.shape[-1], widths)
    T = lambda a: None if a is None else torch.from_numpy(a).to(dev)
    got = pkg.pointnet_util.group_mlp(T(xyz), T(points), T(new_xyz), T(idx), fused(pkg, layers),
                                      pooling, use_xyz=use_xyz, xyz_last=xyz_last).cpu().numpy()
    y64, y32 = O.mlp_f64(grouped, layers), mlp_f32(grouped, layers)
    if pooling is None:
        ref64, ref32 = y64, y32
    else:
        ref64 = O.pool_f64(y64, gxyz, pooling)
        ref32 = O.pool_f64(y32, gxyz, pooling)  # pooled in f64 from the fp32 activations
    assert_close(got, ref64, ref32, f"group_mlp {pooling}")


FP_CASES = [
    # (n, m, C1, C2, widths)
    (2048, 256, 0, 128, [128, 128, 128]),   # FP4 (grid three_nn path)
    (2048, 256, 6, 128, [128, 128, 128]),   # FP4 of the features model (+6 skip channels)
    (256, 64, 128, 256, [256, 256]),         # FP2
    (64, 16, 256, 512, [256, 256]),          # FP1
    (1000, 3, 64, 32, [64]),                  # m = 3
]


@pytest.mark.parametrize("n,m,C1,C2,widths", FP_CASES)
def test_fp_mlp_vs_f64(env, n, m, C1, C2, widths):
    pkg, O, torch, dev = env
    B = 2
    rng = np.random.default_rng(n + m + C1)
    xyz1 = pkg.synth.batch(range(3, 3 + B), n, "scannet")[0]
    xyz2 = xyz1[:, rng.choice(n, m, replace=False)].copy()
    p1 = rng.uniform(-1, 1, (B, n, C1)).astype(np.float32) if C1 else None
    p2 = rng.uniform(-1, 1, (B, m, C2)).astype(np.float32)
    layers = make_layers(rng, C1 + C2, widths)
    store = pkg.tf_util.ParamStore()
    for i, L in enumerate(layers):
        s = f"fa/conv_{i}"
        store[f"{s}/weights"] = torch.from_numpy(L["weights"])
        store[f"{s}/biases"] = torch.from_numpy(L["biases"])
        for k in ("gamma", "beta", "moving_mean", "moving_variance"):
            store[f"{s}/bn/{k}"] = torch.from_numpy(L[k])
    T = lambda a: None if a is None else torch.from_numpy(a).to(dev)
    got = pkg.pointnet_util.pointnet_fp_module(T(xyz1), T(xyz2), T(p1), T(p2), widths, False,
                                               None, "fa", params=store).cpu().numpy()
    x = O.fp_fused(xyz1, xyz2, p1, p2)  # bit-exact interpolation + concat
    assert_close(got, O.mlp_f64(x, layers), mlp_f32(x, layers), "fp_mlp")


def test_sa_module_inference_matches_torch_composition(env):
    """pointnet_sa_module's fused inference path vs its own differentiable torch path
    (is_training=False: moving statistics), SSG and MSG."""
    pkg, O, torch, dev = env
    pu, tu = pkg.pointnet_util, pkg.tf_util
    xyz_np, feats_np = pkg.synth.batch([0, 1], 4096, "scannet", with_features=True)
    xyz, feats = torch.from_numpy(xyz_np).to(dev), torch.from_numpy(feats_np).to(dev)
    store = tu.ParamStore(seed=3)
    # non-trivial batch-norm statistics
    g = np.random.default_rng(5)
    for i, w in enumerate([32, 32, 64]):
        store[f"l1/conv{i}/bn/moving_mean"] = torch.from_numpy(g.uniform(-.1, .1, w).astype(np.float32))
        store[f"l1/conv{i}/bn/moving_variance"] = torch.from_numpy(g.uniform(.5, 2, w).astype(np.float32))
    with torch.no_grad():
        new_xyz, got, idx = pu.pointnet_sa_module(xyz, feats, 512, 0.1, 32, [32, 32, 64], None,
                                                  False, False, None, "l1", params=store)
        x, _ = pu.group_concat(xyz, feats, new_xyz, idx)
        layers = tu.torch_layers(store, [f"l1/conv{i}" for i in range(3)], 9, [32, 32, 64])
        ref = tu.mlp_torch(x, layers, False).max(dim=2).values
    assert got.shape == (2, 512, 64)
    np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-4, atol=1e-5)
    with torch.no_grad():
        nx, got = pu.pointnet_sa_module_msg(xyz, feats, 256, [0.1, 0.2], [16, 32],
                                            [[16, 32], [32, 64]], False, None, "msg",
                                            params=store)
    assert got.shape == (2, 256, 96)
    assert np.array_equal(nx.cpu().numpy(), O.gather_point(xyz_np, O.fps(xyz_np, 256)))


def test_group_all_and_mlp2(env):
    pkg, O, torch, dev = env
    pu, tu = pkg.pointnet_util, pkg.tf_util
    xyz_np, _ = pkg.synth.batch([4, 5], 128, "uniform")
    pts_np = np.random.default_rng(1).uniform(-1, 1, (2, 128, 32)).astype(np.float32)
    xyz, pts = torch.from_numpy(xyz_np).to(dev), torch.from_numpy(pts_np).to(dev)
    store = tu.ParamStore(seed=9)
    with torch.no_grad():
        nx, got, _ = pu.pointnet_sa_module(xyz, pts, None, None, None, [64, 128], [96], True,
                                           False, None, "ga", params=store)
    assert got.shape == (2, 1, 96)
    x = np.concatenate([xyz_np, pts_np], axis=2)
    cv = lambda s, c, w: {**{k: v.numpy() for k, v in store.conv(s, c, w).items()}, "relu": True}
    layers = [cv("ga/conv0", 35, 64), cv("ga/conv1", 64, 128)]
    y = O.mlp_f64(x, layers).max(axis=1, keepdims=True)
    ref = O.mlp_f64(y, [cv("ga/conv_post_0", 128, 96)])
    np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("and_pooling", [False, True])
def test_attention_sa_module_matches_torch_composition(env, and_pooling):
    """pointnet_sa_module_attention(_and_pooling) (attention_layer.py:229-338): the fused
    inference path (group + MLP kernel, packed Dense layers, reduction kernel, batch norm)
    against its differentiable torch composition on the same variables (grad-enabled inputs
    take that path; is_training=False keeps the moving statistics)."""
    pkg, O, torch, dev = env
    al, tu = pkg.attention_layer, pkg.tf_util
    xyz_np, feats_np = pkg.synth.batch([2, 3], 2048, "scannet", with_features=True)
    xyz, feats = torch.from_numpy(xyz_np).to(dev), torch.from_numpy(feats_np).to(dev)
    store = tu.ParamStore(seed=11)
    g = np.random.default_rng(2)
    for k in ("moving_mean", "moving_variance", "gamma", "beta"):
        lo, hi = {"moving_mean": (-.1, .1), "moving_variance": (.5, 2), "gamma": (.5, 1.5),
                  "beta": (-.2, .2)}[k]
        store[f"att/att/{k}"] = torch.from_numpy(g.uniform(lo, hi, 64).astype(np.float32))
    fn = al.pointnet_sa_module_attention_and_pooling if and_pooling else \
        al.pointnet_sa_module_attention
    with torch.no_grad():
        nx, got, idx = fn(xyz, feats, 256, 0.2, 32, [32, 64], None, False, False, None, "att",
                          params=store)
    assert got.shape == (2, 256, 64)
    ref = fn(xyz.clone().requires_grad_(True), feats, 256, 0.2, 32, [32, 64], None, False,
             False, None, "att", params=store)[1].detach()
    np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("widths,ns,add_max", [
    ([32, 64], 32, False),     # C = 64 < 4 ns: heads span whole rows (one segment)
    ([64, 128], 32, True),     # C = 4 ns
    ([128, 256], 32, False),   # C = 8 ns: 2 column segments
    ([256, 512], 32, True),    # SA4 widths: 4 column segments
    ([32, 64], 16, False),     # 2 groups per row tile
    ([64, 128], 64, True),     # a group spans 2 row tiles
])
def test_fused_attention_matches_unfused(env, widths, ns, add_max):
    """pn2_group_mlp_attention (one kernel: group + MLP + Dense q/k/v + heads + batch norm
    [+ max pool]) against the same layer run unfused (per-point group_mlp output, packed Dense
    layers, attention_reduce kernel, batch norm, group_pool), rtol 1e-4 / atol 2e-5."""
    pkg, O, torch, dev = env
    al, tu, pu = pkg.attention_layer, pkg.tf_util, pkg.pointnet_util
    xyz_np, _ = pkg.synth.batch([5, 6], 2048, "scannet")
    pts_np = np.random.default_rng(ns).uniform(-1, 1, (2, 2048, 16)).astype(np.float32)
    xyz, pts = torch.from_numpy(xyz_np).to(dev), torch.from_numpy(pts_np).to(dev)
    store = tu.ParamStore(seed=ns + widths[-1])
    C = widths[-1]
    g = np.random.default_rng(C)
    for k, (lo, hi) in {"moving_mean": (-.1, .1), "moving_variance": (.5, 2), "gamma": (.5, 1.5),
                        "beta": (-.2, .2)}.items():
        store[f"s/s/{k}"] = torch.from_numpy(g.uniform(lo, hi, C).astype(np.float32))
    for d in al._attention_scopes("s"):  # non-zero Dense biases
        store[f"{d}/bias"] = torch.from_numpy(g.uniform(-.1, .1, C).astype(np.float32))
    with torch.no_grad():
        new_xyz = pkg.tf_sampling.farthest_point_sample_and_gather(128, xyz)[1]
        idx, _ = pkg.tf_grouping.query_ball_point(0.2, ns, xyz, new_xyz)
        mlp = tu.packed_mlp(store, [f"s/conv{i}" for i in range(len(widths))], 19, widths)
        got = al.group_mlp_attention(xyz, pts, new_xyz, idx, mlp, store, "s", add_max)
        X = pu.group_mlp(xyz, pts, new_xyz, idx, mlp, None)
        ref = al.sa_attention_tail(X, store, "s", C, add_max)
    assert got.shape == (2, 128, C)
    np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-4, atol=2e-5)


def test_multi_tile_workgroups_full_batch(env):
    """The whole-batch launches of the model (B = 16 clouds of 8,192 points) are the only ones
    large enough for several tiles per workgroup (csrc/mlp.hip launch_one: tpw doubles while
    the grid keeps >= 4 rounds of 2 workgroups on each of the 256 CUs): SA1 (4,096 tiles of
    128 rows -> 2 tiles per workgroup, weights staged in LDS) and SA2 (4,096 tiles of 32 rows).
    Same f64 bar as above."""
    pkg, O, torch, dev = env
    B, N = 16, 8192
    xyz, _ = pkg.synth.batch(range(40, 40 + B), N, "scannet")
    rng = np.random.default_rng(16)
    T = lambda a: None if a is None else torch.from_numpy(a).to(dev)  # noqa: E731
    x1 = O.gather_point(xyz, O.fps(xyz, 1024))
    for (src, nxt, M, r, C, widths) in [(xyz, x1, 1024, 0.1, 0, [32, 32, 64]),
                                        (x1, None, 256, 0.2, 64, [64, 64, 128])]:
        new_xyz = nxt if nxt is not None else O.gather_point(src, O.fps(src, M))
        idx, _ = O.ball_query(src, new_xyz, r, 32)
        points = rng.uniform(-1, 1, (B, src.shape[1], C)).astype(np.float32) if C else None
        grouped, gxyz = O.group_concat(src, points, new_xyz, idx)
        layers = make_layers(rng, grouped.shape[-1], widths)
        got = pkg.pointnet_util.group_mlp(T(src), T(points), T(new_xyz), T(idx),
                                          fused(pkg, layers), "max").cpu().numpy()
        ref64 = O.pool_f64(O.mlp_f64(grouped, layers), gxyz, "max")
        ref32 = O.pool_f64(mlp_f32(grouped, layers), gxyz, "max")
        assert_close(got, ref64, ref32, f"group_mlp B=16 M={M}")


def test_multi_tile_attention_full_batch(env):
    """The cfg3 SA1 attention launch (B = 16, 8,192 tiles of 64 rows -> 4 tiles per workgroup)
    against the unfused composition, as test_fused_attention_matches_unfused."""
    pkg, O, torch, dev = env
    al, tu, pu = pkg.attention_layer, pkg.tf_util, pkg.pointnet_util
    xyz_np, feats_np = pkg.synth.batch(range(60, 76), 8192, "scannet", with_features=True)
    xyz, pts = torch.from_numpy(xyz_np).to(dev), torch.from_numpy(feats_np).to(dev)
    store = tu.ParamStore(seed=23)
    g = np.random.default_rng(64)
    for k, (lo, hi) in {"moving_mean": (-.1, .1), "moving_variance": (.5, 2), "gamma": (.5, 1.5),
                        "beta": (-.2, .2)}.items():
        store[f"s/s/{k}"] = torch.from_numpy(g.uniform(lo, hi, 64).astype(np.float32))
    with torch.no_grad():
        new_xyz = pkg.tf_sampling.farthest_point_sample_and_gather(1024, xyz)[1]
        idx, _ = pkg.tf_grouping.query_ball_point(0.1, 32, xyz, new_xyz)
        mlp = tu.packed_mlp(store, [f"s/conv{i}" for i in range(3)], 9, [32, 32, 64])
        got = al.group_mlp_attention(xyz, pts, new_xyz, idx, mlp, store, "s", False)
        X = pu.group_mlp(xyz, pts, new_xyz, idx, mlp, None)
        ref = al.sa_attention_tail(X, store, "s", 64, False)
    assert got.shape == (16, 1024, 64)
    np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-4, atol=2e-5)
