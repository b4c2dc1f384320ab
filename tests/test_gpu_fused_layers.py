"""GPU parity of the multi-layer launches against the oracle, bit for bit:

* pointnet_util.ball_group_layers (pn2_ball_group_layers): several layers' query_ball_point +
  group_concat in one kernel == oracle.ball_query + oracle.group_concat per layer
  (tf_grouping_g.cu:3-57, pointnet_util.py:38-56 / :186-193);
* pointnet_util.fp_interpolate_layers (pn2_fp_fused_layers): several FP layers' three_nn +
  IDW + three_interpolate + concat in one kernel == pointnet_util.fp_interpolate per layer
  (itself pinned to the oracle in test_gpu_parity.py::test_fp_fused).
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


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def _layer(pkg, O, kind, B, N, M, C, seed):
    if kind == "grid":  # integer lattice: exact distances on the radius
        g = np.stack(np.meshgrid(*[np.arange(8)] * 3, indexing="ij"), -1).reshape(-1, 3)
        rng = np.random.default_rng(seed)
        x = np.stack([g[rng.integers(0, len(g), N)] for _ in range(B)]).astype(np.float32)
        q = x[:, :M].copy()
    else:
        x = pkg.synth.batch(range(seed, seed + B), N, kind)[0]
        q = O.gather_point(x, O.fps(x, M))
    q[:, :1] = 50.0  # a query with no hit at all (idx 0, pts_cnt 0)
    pts = pkg.synth.features_uniform(seed + 7, (B, N, C)) if C else None
    return x, pts, q


# (kind, N, M, C, radius, nsample) per layer; one list = one launch
LAUNCHES = [
    # the SSG stack's SA2..SA4 at cfg2 shapes
    [("scannet", 1024, 256, 64, 0.2, 32), ("scannet", 256, 64, 128, 0.4, 32),
     ("scannet", 64, 16, 256, 0.8, 32)],
    # cfg3 features (C = 9 at SA1-like widths), and an odd Cout (scalar stores)
    [("scannet", 1000, 100, 9, 0.2, 32), ("uniform", 300, 50, 2, 0.05, 3)],
    # MSG level-2 radii (ns up to 128), no features, a lattice
    [("scannet", 512, 128, 0, 0.2, 32), ("scannet", 512, 128, 0, 0.4, 64),
     ("scannet", 512, 128, 0, 0.8, 128), ("grid", 700, 90, 5, 1.0, 16)],
    # one layer, one point per cloud
    [("uniform", 1, 4, 3, 0.5, 8)],
]


@pytest.mark.parametrize("li", range(len(LAUNCHES)))
@pytest.mark.parametrize("use_xyz,xyz_last", [(True, False), (True, True), (False, False)])
@pytest.mark.parametrize("want_gx", [False, True])
def test_ball_group_layers(env, li, use_xyz, xyz_last, want_gx):
    """Every layout (SSG [xyz, points], MSG [points, xyz], points only, xyz only), with and
    without the grouped_xyz output (written in every layout, as pn2_group_concat does)."""
    pkg, O, torch, dev = env
    B = 3
    t = lambda a: None if a is None else torch.from_numpy(a).to(dev)  # noqa: E731
    specs, refs = [], []
    for j, (kind, N, M, C, r, ns) in enumerate(LAUNCHES[li]):
        if not use_xyz and C == 0:
            C = 4  # points only needs points
        x, pts, q = _layer(pkg, O, kind, B, N, M, C, 10 * li + j)
        specs.append((r, ns, t(x), t(pts), t(q)))
        ridx, rcnt = O.ball_query(x, q, r, ns)
        rnp, rgx = O.group_concat(x, pts, q, ridx, use_xyz=use_xyz, xyz_last=xyz_last)
        refs.append((ridx, rcnt, rnp, rgx))
    got = pkg.pointnet_util.ball_group_layers(specs, use_xyz=use_xyz, xyz_last=xyz_last,
                                              want_grouped_xyz=want_gx)
    for out, (ridx, rcnt, rnp, rgx) in zip(got, refs):
        idx, cnt, new_points = out[:3]
        assert np.array_equal(cnt.cpu().numpy(), rcnt)
        assert np.array_equal(idx.cpu().numpy(), ridx)
        assert np.array_equal(_bits(new_points.cpu().numpy()), _bits(rnp))
        if want_gx:
            assert np.array_equal(_bits(out[3].cpu().numpy()), _bits(rgx)), "grouped_xyz"


def test_ball_group_layers_rejects(env):
    pkg, O, torch, dev = env
    x = torch.zeros((2, 2000, 3), device=dev)
    q = torch.zeros((2, 10, 3), device=dev)
    with pytest.raises(pkg.tf_grouping.InvalidArgumentError):
        pkg.pointnet_util.ball_group_layers([(0.1, 8, x, None, q)])  # N > 1024
    x = torch.zeros((2, 100, 3), device=dev)
    with pytest.raises(pkg.tf_grouping.InvalidArgumentError):
        pkg.pointnet_util.ball_group_layers([(0.1, 129, x, None, q)])  # nsample > 128
    with pytest.raises(pkg.tf_grouping.InvalidArgumentError):
        pkg.pointnet_util.ball_group_layers([(0.1, 8, x, None, q[:1])])  # batch mismatch


FP_LAUNCHES = [
    # the SSG stack's FP3, FP2, FP1 at cfg2 shapes: (n, m, C1, C2)
    [(1024, 256, 64, 256), (256, 64, 128, 256), (64, 16, 256, 512)],
    # no points1, odd widths (scalar columns: another kernel variant, its own launch), m < 3
    [(500, 100, 0, 32), (300, 37, 5, 7), (40, 2, 4, 8)],
    [(1, 1, 4, 4)],
]


@pytest.mark.parametrize("li", range(len(FP_LAUNCHES)))
def test_fp_interpolate_layers(env, li):
    pkg, O, torch, dev = env
    B = 3
    t = lambda a: None if a is None else torch.from_numpy(a).to(dev)  # noqa: E731
    layers = []
    for j, (n, m, C1, C2) in enumerate(FP_LAUNCHES[li]):
        x1 = pkg.synth.batch(range(j, j + B), n, "scannet")[0]
        x2 = x1[:, :m].copy() + np.float32(1e-3)
        p1 = pkg.synth.features_uniform(40 + j, (B, n, C1)) if C1 else None
        p2 = pkg.synth.features_uniform(50 + j, (B, m, C2))
        layers.append((t(x1), t(x2), t(p1), t(p2)))
    got = pkg.pointnet_util.fp_interpolate_layers(layers)
    for out, (x1, x2, p1, p2) in zip(got, layers):
        ref = pkg.pointnet_util.fp_interpolate(x1, x2, p1, p2)
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32))



GROUP_XYZ_CASES = [
    ("scannet", 2, 8192, 1024, 0.1, 32),   # cfg2 SA1
    ("scannet", 1, 16384, 512, 0.4, 128),  # cfg5 SA1, largest radius
    ("scannet", 1, 16384, 512, 0.1, 16),
    ("grid", 2, 4096, 500, 1.0, 16),       # exact lattice distances at the radius
]


@pytest.mark.parametrize("kind,B,N,M,r,ns", GROUP_XYZ_CASES)
def test_ball_group_xyz(env, kind, B, N, M, r, ns):
    """pointnet_util.ball_group_xyz (pn2_ball_group_xyz_grid) == oracle ball_query +
    group_concat of an xyz-only layer, bit for bit, including a query with no hit."""
    pkg, O, torch, dev = env
    x, _, q = _layer(pkg, O, kind, B, N, M, 0, 3)
    xt, qt = torch.from_numpy(x).to(dev), torch.from_numpy(q).to(dev)
    grid = pkg.tf_grouping.BallGrid(xt, r)
    idx, cnt, grouped = pkg.pointnet_util.ball_group_xyz(r, ns, xt, qt, grid)
    ridx, rcnt = O.ball_query(x, q, r, ns)
    rg, _ = O.group_concat(x, None, q, ridx)
    assert np.array_equal(cnt.cpu().numpy(), rcnt)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert np.array_equal(_bits(grouped.cpu().numpy()), _bits(rg))


GROUP_RADII_CASES = [
    ("scannet", 2, 16384, 512, (0.1, 0.2, 0.4), (16, 32, 128), 0.2),  # cfg5 SA1 (its grid)
    ("scannet", 2, 8192, 1024, (0.4, 0.1), (8, 64), 0.1),             # unsorted, grid at r_min
    ("grid", 2, 4096, 500, (1.0, 2.0, 1.5), (16, 8, 32), 1.0),        # lattice ties at radii
    ("scannet", 1, 3000, 300, (0.3,), (40,), 0.5),                    # one radius
    ("uniform", 1, 50000, 200, (0.03, 0.05, 0.08), (8, 16, 32), 0.05),  # beyond the LDS
    # bound of one launch (3 x 1563 bitmask words): the wrapper's launch per radius
]


@pytest.mark.parametrize("kind,B,N,M,radii,nss,edge", GROUP_RADII_CASES)
def test_ball_group_xyz_radii(env, kind, B, N, M, radii, nss, edge):
    """pointnet_util.ball_group_xyz_radii (pn2_ball_group_xyz_grid_radii: one walk over the
    largest radius' cells for all radii) == the oracle's ball_query + group_concat per radius,
    bit for bit, and == ball_group_xyz radius by radius."""
    pkg, O, torch, dev = env
    x, _, q = _layer(pkg, O, kind, B, N, M, 0, 3)
    xt, qt = torch.from_numpy(x).to(dev), torch.from_numpy(q).to(dev)
    grid = pkg.tf_grouping.BallGrid(xt, edge)
    outs = pkg.pointnet_util.ball_group_xyz_radii(radii, nss, xt, qt, grid)
    for (idx, cnt, grouped), r, ns in zip(outs, radii, nss):
        ridx, rcnt = O.ball_query(x, q, r, ns)
        rg, _ = O.group_concat(x, None, q, ridx)
        assert np.array_equal(cnt.cpu().numpy(), rcnt)
        assert np.array_equal(idx.cpu().numpy(), ridx)
        assert np.array_equal(_bits(grouped.cpu().numpy()), _bits(rg))
        one = pkg.pointnet_util.ball_group_xyz(r, ns, xt, qt, grid)
        assert torch.equal(one[0], idx) and torch.equal(one[1], cnt)
        assert torch.equal(one[2].view(torch.int32), grouped.view(torch.int32))


GROUP_FEAT_CASES = [
    # kind, B, N, M, C, r, ns, xyz_last
    ("scannet", 2, 8192, 1024, 6, 0.1, 32, False),   # cfg3 SA1: rgb + normals
    ("scannet", 2, 8192, 1024, 6, 0.1, 32, True),    # the MSG order
    ("grid", 2, 4096, 500, 9, 1.0, 16, False),       # lattice ties at the radius
    ("uniform", 1, 3000, 300, 64, 0.3, 40, True),    # wide rows, queries short of ns
    ("scannet", 1, 16384, 512, 1, 0.4, 128, False),  # ns 128, one channel
    ("uniform", 1, 5, 7, 3, 0.5, 8, False),          # tiny cloud
]


@pytest.mark.parametrize("kind,B,N,M,C,r,ns,xyz_last", GROUP_FEAT_CASES)
def test_ball_group_features(env, kind, B, N, M, C, r, ns, xyz_last):
    """pointnet_util.ball_group (pn2_ball_group_grid: grid query + grouping with features in
    one kernel) == the oracle's ball_query + group_concat ([xyz - new_xyz, points], or the MSG
    order), bit for bit, including a query with no hit; C = 0 is ball_group_xyz."""
    pkg, O, torch, dev = env
    x, p, q = _layer(pkg, O, kind, B, N, M, C, 5)
    xt, pt, qt = (torch.from_numpy(a).to(dev) for a in (x, p, q))
    grid = pkg.tf_grouping.BallGrid(xt, r)
    idx, cnt, new_points = pkg.pointnet_util.ball_group(r, ns, xt, pt, qt, grid,
                                                        xyz_last=xyz_last)
    ridx, rcnt = O.ball_query(x, q, r, ns)
    rnp, _ = O.group_concat(x, p, q, ridx, use_xyz=True, xyz_last=xyz_last)
    assert np.array_equal(cnt.cpu().numpy(), rcnt)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert np.array_equal(_bits(new_points.cpu().numpy()), _bits(rnp))
    i0, c0, g0 = pkg.pointnet_util.ball_group(r, ns, xt, None, qt, grid)
    rg, _ = O.group_concat(x, None, q, ridx)
    assert torch.equal(i0, idx) and np.array_equal(_bits(g0.cpu().numpy()), _bits(rg))


def test_ball_group_rejects(env):
    """PN2_EINVAL (InvalidArgumentError) for features without use_xyz, a negative C, or
    features with no pointer -- never a silent fallback."""
    pkg, O, torch, dev = env
    L = pkg._lib
    x, p, q = _layer(pkg, O, "uniform", 1, 100, 10, 4, 1)
    xt, pt, qt = (torch.from_numpy(a).to(dev) for a in (x, p, q))
    grid = pkg.tf_grouping.BallGrid(xt, 0.2)
    idx = torch.empty((1, 10, 8), dtype=torch.int32, device=dev)
    cnt = torch.empty((1, 10), dtype=torch.int32, device=dev)
    out = torch.empty((1, 10, 8, 7), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    lib = L.lib()
    args = lambda C, flags, pts: (grid.buf.data_ptr(), xt.data_ptr(), pts, C, flags,  # noqa: E731
                                  qt.data_ptr(), 1, 100, 10, 0.2, 8, idx.data_ptr(),
                                  cnt.data_ptr(), out.data_ptr(), st)
    assert lib.pn2_ball_group_grid(*args(4, 0, pt.data_ptr())) == L.PN2_EINVAL
    assert lib.pn2_ball_group_grid(*args(-1, L.PN2_USE_XYZ, pt.data_ptr())) == L.PN2_EINVAL
    assert lib.pn2_ball_group_grid(*args(4, L.PN2_USE_XYZ, None)) == L.PN2_EINVAL
    assert lib.pn2_ball_group_grid(*args(4, L.PN2_USE_XYZ, pt.data_ptr())) == 0


@pytest.mark.parametrize("shapes", [
    # the SSG stack's four attention SA layers at cfg3 (ns 32, C = 64 .. 512), B = 2
    [(1024, 32, 64), (256, 32, 128), (64, 32, 256), (16, 32, 512)],
    [(100, 8, 4), (7, 8, 12)],          # few heads, odd group counts
    [(33, 128, 32)],                    # one layer, ns 128
    [(50, 20, 16), (9, 20, 8)],         # an nsample without a layers-kernel instance: per layer
])
def test_attention_reduce_layers(env, shapes):
    """attention_layer.attention_reduce_layers (pn2_attn_reduce_layers: several layers' attention
    reductions in one launch) == attention_reduce per layer, bit for bit (the same kernel body),
    and within 1e-5 of the oracle's restatement of attention_layer.py:35-42."""
    pkg, O, torch, dev = env
    B = 2
    qkvs = []
    for i, (M, ns, C) in enumerate(shapes):
        g = torch.Generator(device=dev)
        g.manual_seed(100 + i)
        qkvs.append((torch.rand((B, M, C), generator=g, device=dev) * 2 - 1,
                     torch.rand((B, M, ns, C), generator=g, device=dev) * 2 - 1,
                     torch.rand((B, M, ns, C), generator=g, device=dev) * 2 - 1))
    outs = pkg.attention_layer.attention_reduce_layers(qkvs)
    for (Q, K, V), o in zip(qkvs, outs):
        ref = pkg.attention_layer.attention_reduce(Q, K, V)
        assert torch.equal(o.view(torch.int32), ref.view(torch.int32))
        np.testing.assert_allclose(o.cpu().numpy(), O.attn_reduce(Q.cpu().numpy(), K.cpu().numpy(),
                                                                  V.cpu().numpy()),
                                   rtol=1e-5, atol=1e-5)


def test_attention_reduce_layers_rejects(env):
    """Layers of different nsample in one launch: PN2_EINVAL, never a silent fallback."""
    pkg, O, torch, dev = env
    a = (torch.zeros((1, 4, 8), device=dev), torch.zeros((1, 4, 8, 8), device=dev),
         torch.zeros((1, 4, 8, 8), device=dev))
    b = (torch.zeros((1, 4, 8), device=dev), torch.zeros((1, 4, 16, 8), device=dev),
         torch.zeros((1, 4, 16, 8), device=dev))
    with pytest.raises(pkg._lib.InvalidArgumentError):
        pkg.attention_layer.attention_reduce_layers([a, b])
