"""GPU parity: the HIP path (through the C ABI) against the oracle on identical inputs.

Bars (BASELINE.json north_star): indices (FPS, ball query, three_nn idx, gather, group) and
copies are BIT-EXACT; three_nn distances and three_interpolate are bit-exact too (same fp32
expression order, no FMA); IDW weights, attention and pooling are within 1e-5 (rtol=atol=1e-5,
written in each assert). Float-atomic gradients are within 1e-5 as well (order not fixed).
The oracle is pinned to the reference's own code in test_oracle_golden.py and, on this box,
against the reference's own CUDA kernels compiled for gfx950 (the *_vs_reference tests).
"""
import glob
import importlib
import json
import os

import numpy as np
import pytest

from conftest import PKG_NAME, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

TOL = dict(rtol=1e-5, atol=1e-5)


@pytest.fixture(scope="module")
def env():
    import torch

    from oracle import oracle as O
    O.set_threads(16)
    pkg = importlib.import_module(PKG_NAME)
    return pkg, O, torch, torch.device("cuda:0")


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def _cloud(pkg, kind, B, N, seed=0):
    if kind == "scannet":
        return pkg.synth.batch(range(seed, seed + B), N, "scannet")[0]
    if kind == "uniform":
        return pkg.synth.batch(range(seed, seed + B), N, "uniform")[0]
    if kind == "dup":  # every point the same: all distances tie
        x = np.tile(np.array([[0.25, 0.5, 0.75]], np.float32), (B, N, 1))
        return x.reshape(B, N, 3)
    if kind == "grid":  # integer lattice: massive exact ties
        g = np.stack(np.meshgrid(*[np.arange(16)] * 3, indexing="ij"), -1).reshape(-1, 3)
        rng = np.random.default_rng(seed)
        return np.stack([g[rng.integers(0, len(g), N)] for _ in range(B)]).astype(np.float32)
    if kind == "fewuniq":  # 300 distinct points drawn with replacement: npoint > #unique
        rng = np.random.default_rng(seed)
        u = rng.random((300, 3)).astype(np.float32)
        return np.stack([u[rng.integers(0, 300, N)] for _ in range(B)])
    raise ValueError(kind)


FPS_CASES = [
    ("uniform", 1, 1024, 256),   # cfg1
    ("scannet", 2, 8192, 1024),  # SSG SA1 (duplicates)
    ("scannet", 2, 1024, 256),   # SA2
    ("scannet", 3, 256, 64),     # SA3
    ("scannet", 3, 64, 16),      # SA4
    ("scannet", 2, 16384, 512),  # MSG SA1 (global-coordinate path)
    ("scannet", 2, 3000, 300),
    ("uniform", 2, 100, 37),
    ("uniform", 1, 1, 5),        # N = 1
    ("uniform", 2, 50, 80),      # npoint > N
    ("dup", 2, 700, 40),         # all-duplicate cloud
    ("grid", 2, 4096, 512),      # tie-heavy lattice
    ("grid", 2, 600, 100),
    ("scannet", 1, 20000, 64),   # workspace path (N > 16384)
]


@pytest.mark.parametrize("kind,B,N,M", FPS_CASES)
def test_fps_vs_oracle(env, kind, B, N, M):
    pkg, O, torch, dev = env
    x = _cloud(pkg, kind, B, N)
    idx, new_xyz = pkg.tf_sampling.farthest_point_sample_and_gather(M, torch.from_numpy(x).to(dev))
    ref = O.fps(x, M)
    got = idx.cpu().numpy()
    assert np.array_equal(got, ref), f"{(got != ref).sum()} FPS indices differ"
    assert np.array_equal(_bits(new_xyz.cpu().numpy()), _bits(O.gather_point(x, ref)))
    only = pkg.tf_sampling.farthest_point_sample(M, torch.from_numpy(x).to(dev))
    assert np.array_equal(only.cpu().numpy(), ref)


# (the per-schedule sampler cases, the full-size steps and the FPS golden vectors run first:
# tests/test_gpu_a_fullsize.py)


@pytest.mark.parametrize("kind,B,N,M", [c for c in FPS_CASES if c[2] <= 16384])
def test_fps_vs_reference_kernel(env, kind, B, N, M):
    """The reference's own farthestpointsamplingKernel (tf_sampling_g.cu:105-170) run on this
    GPU pins the oracle and the HIP sampler to the reference's behaviour, ties included."""
    pkg, O, torch, dev = env
    if not O.have_ref_gpu():
        pytest.skip("oracle/_ref/libref_gpu.so not built")
    x = _cloud(pkg, kind, B, N)
    xt = torch.from_numpy(x).to(dev)
    ref_out = torch.zeros((B, M), dtype=torch.int32, device=dev)
    assert O.ref_gpu().pn2ref_fps(xt.data_ptr(), B, N, M, ref_out.data_ptr()) == 0
    ref = ref_out.cpu().numpy()
    assert np.array_equal(O.fps(x, M), ref), "oracle FPS differs from the reference kernel"
    got = pkg.tf_sampling.farthest_point_sample(M, xt).cpu().numpy()
    assert np.array_equal(got, ref), f"{(got != ref).sum()} FPS indices differ from reference"


PROB_CASES = [  # (B, n, m, weights)
    (3, 1003, 200, "uniform"),
    (2, 8192, 512, "skewed"),      # exactly one chunk
    (2, 50001, 1000, "uniform"),   # 7 chunks, Kahan carry, partial last quad
    (4, 37, 300, "zeros"),         # zero weights: flat prefix sums, ties
    (1, 1, 5, "uniform"),
]


def _prob_inputs(B, n, m, kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "skewed":
        w = rng.exponential(1.0, (B, n)) ** 6
    else:
        w = rng.random((B, n))
    if kind == "zeros":
        w[:, rng.random(n) < 0.5] = 0.0
        w[:, 0] = 0.0
    r = rng.random((B, m))
    r[:, 0] = 0.0
    return np.ascontiguousarray(w, np.float32), np.ascontiguousarray(r, np.float32)


@pytest.mark.parametrize("B,n,m,kind", PROB_CASES)
def test_prob_sample_vs_oracle_and_reference(env, B, n, m, kind):
    """ProbSample (tf_sampling_g.cu:7-104): indices bit-exact against the oracle and against the
    reference's own cumsumKernel + binarysearchKernel run on this GPU."""
    pkg, O, torch, dev = env
    w, r = _prob_inputs(B, n, m, kind, seed=n + m)
    got = pkg.tf_sampling.prob_sample(torch.from_numpy(w).to(dev),
                                      torch.from_numpy(r).to(dev)).cpu().numpy()
    assert np.array_equal(got, O.prob_sample(w, r)), "prob_sample differs from the oracle"
    if O.have_ref_gpu():
        out = torch.full((B, m), -1, dtype=torch.int32, device=dev)
        wt, rt = torch.from_numpy(w).to(dev), torch.from_numpy(r).to(dev)
        assert O.ref_gpu().pn2ref_prob_sample(wt.data_ptr(), rt.data_ptr(), B, n, m,
                                              out.data_ptr()) == 0
        assert np.array_equal(got, out.cpu().numpy()), "prob_sample differs from the reference"


def test_prob_sample_errors(env):
    pkg, O, torch, dev = env
    ts = pkg.tf_sampling
    with pytest.raises(pkg._lib.InvalidArgumentError, match="num_choices"):
        ts.prob_sample(torch.zeros(2, 3, 4, device=dev), torch.zeros(2, 5, device=dev))
    with pytest.raises(pkg._lib.InvalidArgumentError, match="num_points"):
        ts.prob_sample(torch.zeros(2, 3, device=dev), torch.zeros(3, 5, device=dev))
    with pytest.raises(pkg._lib.InvalidArgumentError):  # n = 0 (the reference reads cum[-1])
        ts.prob_sample(torch.zeros(2, 0, device=dev), torch.zeros(2, 5, device=dev))
    assert ts.prob_sample(torch.ones(2, 3, device=dev), torch.zeros(2, 0, device=dev)).shape == (2, 0)


def test_gather_point(env):
    pkg, O, torch, dev = env
    x = _cloud(pkg, "scannet", 3, 2048)
    idx = np.random.default_rng(1).integers(0, 2048, (3, 300)).astype(np.int32)
    got = pkg.tf_sampling.gather_point(torch.from_numpy(x).to(dev), torch.from_numpy(idx).to(dev))
    assert np.array_equal(_bits(got.cpu().numpy()), _bits(O.gather_point(x, idx)))
    if O.have_ref_gpu():
        out = torch.zeros((3, 300, 3), device=dev)
        xt, it = torch.from_numpy(x).to(dev), torch.from_numpy(idx).to(dev)
        assert O.ref_gpu().pn2ref_gather_point(xt.data_ptr(), it.data_ptr(), 3, 2048, 300,
                                               out.data_ptr()) == 0
        assert np.array_equal(_bits(out.cpu().numpy()), _bits(got.cpu().numpy()))


BQ_CASES = [
    ("uniform", 1, 1024, 256, 0.2, 32),   # cfg1
    ("scannet", 2, 8192, 1024, 0.1, 32),  # SA1
    ("scannet", 2, 1024, 256, 0.2, 32),   # SA2
    ("scannet", 2, 256, 64, 0.4, 32),     # SA3
    ("scannet", 2, 64, 16, 0.8, 32),      # SA4
    ("scannet", 1, 16384, 512, 0.4, 128),  # MSG, global path
    ("scannet", 1, 16384, 512, 0.1, 16),
    ("scannet", 2, 4096, 512, 0.2, 64),
    ("grid", 2, 2000, 100, 1.0, 16),      # exact lattice distances at the radius
    ("uniform", 2, 300, 50, 0.05, 8),     # sparse: many cnt < ns
]


@pytest.mark.parametrize("kind,B,N,M,r,ns", BQ_CASES)
def test_ball_query_vs_oracle(env, kind, B, N, M, r, ns):
    pkg, O, torch, dev = env
    x = _cloud(pkg, kind, B, N)
    q = O.gather_point(x, O.fps(x, M)) if kind != "grid" else x[:, :M].copy()
    idx, cnt = pkg.tf_grouping.query_ball_point(r, ns, torch.from_numpy(x).to(dev),
                                                torch.from_numpy(q).to(dev))
    ridx, rcnt = O.ball_query(x, q, r, ns)
    assert np.array_equal(cnt.cpu().numpy(), rcnt)
    assert np.array_equal(idx.cpu().numpy(), ridx)


def test_ball_query_no_hit_and_boundary(env):
    """Queries far from every point (reference leaves idx uninitialised; defined as 0 here,
    pts_cnt 0) and points whose sqrt rounds exactly onto the radius."""
    pkg, O, torch, dev = env
    r = np.float32(0.3)
    xs = (r * (1.0 + np.arange(-40, 41, dtype=np.float64) * 2e-8)).astype(np.float32)
    pts = np.zeros((1, len(xs), 3), np.float32)
    pts[0, :, 0] = xs
    q = np.array([[[0, 0, 0], [100, 100, 100], [0.0, 1e-7, 0]]], np.float32)
    idx, cnt = pkg.tf_grouping.query_ball_point(float(r), 64, torch.from_numpy(pts).to(dev),
                                                torch.from_numpy(q).to(dev))
    ridx, rcnt = O.ball_query(pts, q, float(r), 64)
    assert np.array_equal(cnt.cpu().numpy(), rcnt)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert rcnt[0, 1] == 0 and (idx.cpu().numpy()[0, 1] == 0).all()
    assert 0 < rcnt[0, 0] < len(xs)


GRID_CASES = [
    ("scannet", 2, 8192, 1024, 0.1, 32),   # SA1 (what the stack runs on the grid)
    ("scannet", 1, 16384, 512, 0.4, 128),  # MSG
    ("scannet", 2, 3000, 300, 0.2, 64),    # N not a multiple of 32
    ("uniform", 2, 700, 200, 0.05, 8),
    ("dup", 2, 2048, 64, 0.1, 16),         # zero extent: one cell
    ("grid", 2, 4096, 500, 1.0, 16),       # exact lattice distances at the radius
    ("scannet", 1, 4096, 256, 0.004, 8),   # tiny radius: cell edge grows to fit the cell cap
    ("scannet", 1, 2048, 128, 5.0, 64),    # ball covers the cloud
]


@pytest.mark.parametrize("kind,B,N,M,r,ns", GRID_CASES)
def test_ball_query_grid_equals_scan(env, kind, B, N, M, r, ns):
    """The spatial-grid path (ball_grid.hip) returns exactly the in-order scan's idx and
    pts_cnt, and the oracle's; queries also far outside the cloud's bounding box."""
    pkg, O, torch, dev = env
    x = _cloud(pkg, kind, B, N)
    q = O.gather_point(x, O.fps(x, M)) if kind != "grid" else x[:, :M].copy()
    q[:, :3] = np.array([[50.0, 50.0, 50.0], [-3.0, 0.5, 0.5], [0.5, 0.5, 9.0]], np.float32)
    xt, qt = torch.from_numpy(x).to(dev), torch.from_numpy(q).to(dev)
    grid = pkg.tf_grouping.BallGrid(xt, r)
    gi, gc = pkg.tf_grouping.query_ball_point(r, ns, xt, qt, grid=grid)
    ri, rc = O.ball_query(x, q, r, ns)
    assert np.array_equal(gc.cpu().numpy(), rc)
    assert np.array_equal(gi.cpu().numpy(), ri)
    # the same grid serves another radius exactly
    gi2, gc2 = pkg.tf_grouping.query_ball_point(2 * r, ns, xt, qt, grid=grid)
    ri2, rc2 = O.ball_query(x, q, 2 * r, ns)
    assert np.array_equal(gc2.cpu().numpy(), rc2) and np.array_equal(gi2.cpu().numpy(), ri2)
    # and the in-order scan agrees
    L = pkg.lib()
    si = torch.empty_like(gi)
    sc = torch.empty_like(gc)
    assert L.pn2_ball_query(xt.data_ptr(), qt.data_ptr(), B, N, M, r, ns, si.data_ptr(),
                            sc.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    assert torch.equal(si, gi) and torch.equal(sc, gc)


@pytest.mark.parametrize("kind,B,N,M,r,ns", BQ_CASES[:6])
def test_ball_query_vs_reference_kernel(env, kind, B, N, M, r, ns):
    """query_ball_point_gpu (tf_grouping_g.cu:3-36) itself, on this GPU."""
    pkg, O, torch, dev = env
    if not O.have_ref_gpu():
        pytest.skip("oracle/_ref/libref_gpu.so not built")
    x = _cloud(pkg, kind, B, N)
    q = O.gather_point(x, O.fps(x, M))
    xt, qt = torch.from_numpy(x).to(dev), torch.from_numpy(q).to(dev)
    ri = torch.zeros((B, M, ns), dtype=torch.int32, device=dev)
    rc = torch.zeros((B, M), dtype=torch.int32, device=dev)
    assert O.ref_gpu().pn2ref_query_ball_point(xt.data_ptr(), qt.data_ptr(), B, N, M, r, ns,
                                               ri.data_ptr(), rc.data_ptr()) == 0
    idx, cnt = pkg.tf_grouping.query_ball_point(r, ns, xt, qt)
    assert np.array_equal(cnt.cpu().numpy(), rc.cpu().numpy())
    assert np.array_equal(idx.cpu().numpy(), ri.cpu().numpy())


@pytest.mark.parametrize("C", [1, 3, 16, 64, 259])
def test_group_point(env, C):
    pkg, O, torch, dev = env
    rng = np.random.default_rng(C)
    pts = rng.standard_normal((2, 500, C)).astype(np.float32)
    idx = rng.integers(0, 500, (2, 70, 32)).astype(np.int32)
    got = pkg.tf_grouping.group_point(torch.from_numpy(pts).to(dev), torch.from_numpy(idx).to(dev))
    assert np.array_equal(_bits(got.cpu().numpy()), _bits(O.group_point(pts, idx)))


@pytest.mark.parametrize("C,use_xyz,xyz_last", [(0, True, False), (6, True, False),
                                                (64, True, False), (64, False, False),
                                                (320, True, True), (5, True, True)])
def test_group_concat(env, C, use_xyz, xyz_last):
    pkg, O, torch, dev = env
    x = _cloud(pkg, "scannet", 2, 2048)
    q = O.gather_point(x, O.fps(x, 128))
    idx, _ = O.ball_query(x, q, 0.2, 32)
    pts = pkg.synth.features_uniform(C + 1, (2, 2048, C)) if C else None
    t = lambda a: None if a is None else torch.from_numpy(a).to(dev)
    got, gx = pkg.pointnet_util.group_concat(t(x), t(pts), t(q), t(idx), use_xyz=use_xyz,
                                             xyz_last=xyz_last)
    ref, rgx = O.group_concat(x, pts, q, idx, use_xyz=use_xyz, xyz_last=xyz_last)
    assert np.array_equal(_bits(got.cpu().numpy()), _bits(ref))
    assert np.array_equal(_bits(gx.cpu().numpy()), _bits(rgx))


def test_sample_and_group_api(env):
    pkg, O, torch, dev = env
    x, f = pkg.synth.batch([3, 4], 4096, "scannet", with_features=True)
    new_xyz, new_points, idx, gxyz = pkg.pointnet_util.sample_and_group(
        512, 0.2, 32, torch.from_numpy(x).to(dev), torch.from_numpy(f).to(dev))
    nx = O.gather_point(x, O.fps(x, 512))
    bi, _ = O.ball_query(x, nx, 0.2, 32)
    npts, gx = O.group_concat(x, f, nx, bi)
    assert np.array_equal(_bits(new_xyz.cpu().numpy()), _bits(nx))
    assert np.array_equal(idx.cpu().numpy(), bi)
    assert np.array_equal(_bits(new_points.cpu().numpy()), _bits(npts))
    assert np.array_equal(_bits(gxyz.cpu().numpy()), _bits(gx))


NN_CASES = [(2, 512, 128), (2, 8192, 1024), (2, 64, 16), (1, 100, 3), (1, 100, 2), (1, 7, 1),
            (2, 1024, 4097)]


@pytest.mark.parametrize("B,n,m", NN_CASES)
def test_three_nn(env, B, n, m):
    pkg, O, torch, dev = env
    x1 = _cloud(pkg, "scannet", B, n, seed=5)
    x2 = _cloud(pkg, "scannet", B, m, seed=9)
    d, i = pkg.tf_interpolate.three_nn(torch.from_numpy(x1).to(dev), torch.from_numpy(x2).to(dev))
    rd, ri = O.three_nn(x1, x2)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(_bits(d.cpu().numpy()), _bits(rd))


def test_three_nn_ties(env):
    pkg, O, torch, dev = env
    x2 = _cloud(pkg, "grid", 2, 300)
    x1 = _cloud(pkg, "grid", 2, 500, seed=3) + np.float32(0.5)
    d, i = pkg.tf_interpolate.three_nn(torch.from_numpy(x1).to(dev), torch.from_numpy(x2).to(dev))
    rd, ri = O.three_nn(x1, x2)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(_bits(d.cpu().numpy()), _bits(rd))


NN_GRID_CASES = [
    ("fp4", 2, 8192, 1024),      # FP4 of the stack: unknowns = the cloud, knowns = its FPS
    ("scannet", 2, 3000, 700),
    ("grid", 2, 2000, 600),      # lattice: exact distance ties everywhere
    ("far", 1, 1000, 512),       # unknowns far outside the known cloud's bbox
    ("dup", 2, 700, 600),        # known cloud of one repeated point (one cell)
    ("scannet", 2, 500, 2),      # m < 3: unfilled slots stay (inf, 0)
    ("scannet", 1, 300, 1),
]


@pytest.mark.parametrize("kind,B,n,m", NN_GRID_CASES)
def test_three_nn_grid(env, kind, B, n, m):
    """three_nn over a grid of the known points (interp.hip three_nn_grid_kernel) gives the
    scan's (and the oracle's) idx and dist bit-exactly, with and without the unknown grid
    ordering the work; fp_interpolate over it equals the fused scan."""
    pkg, O, torch, dev = env
    if kind == "fp4":
        x1 = _cloud(pkg, "scannet", B, n, seed=4)
        x2 = O.gather_point(x1, O.fps(x1, m))
    elif kind == "far":
        x1 = _cloud(pkg, "uniform", B, n, seed=4) * np.float32(20.0) - np.float32(10.0)
        x2 = _cloud(pkg, "scannet", B, m, seed=6)
    else:
        x1 = _cloud(pkg, kind if kind != "dup" else "scannet", B, n, seed=4)
        x2 = _cloud(pkg, kind, B, m, seed=8)
        if kind == "grid":
            x1 = x1 + np.float32(0.5)
    t1, t2 = torch.from_numpy(x1).to(dev), torch.from_numpy(x2).to(dev)
    rd, ri = O.three_nn(x1, x2)
    ug = pkg.grid.PointGrid(t1, 0.1)
    # automatic cell edge (LDS-staged search) and a fine explicit edge (more cells than
    # points: the search reads the grid from global memory)
    for kg in (pkg.grid.PointGrid(t2), pkg.grid.PointGrid(t2, 0.02)):
        for u in (None, ug):
            d, i = pkg.tf_interpolate.three_nn(t1, t2, known_grid=kg, unknown_grid=u)
            assert np.array_equal(i.cpu().numpy(), ri)
            assert np.array_equal(_bits(d.cpu().numpy()), _bits(rd))
    if m >= 3:
        p1 = torch.from_numpy(pkg.synth.features_uniform(1, (B, n, 8))).to(dev)
        p2 = torch.from_numpy(pkg.synth.features_uniform(2, (B, m, 16))).to(dev)
        L = pkg.lib()
        fused = torch.empty((B, n, 24), device=dev)
        assert L.pn2_fp_fused(t1.data_ptr(), t2.data_ptr(), p1.data_ptr(), 8, p2.data_ptr(), 16,
                              B, n, m, fused.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        for u in (None, ug):
            a = pkg.pointnet_util.fp_interpolate(t1, t2, p1, p2, known_grid=kg, unknown_grid=u)
            assert torch.equal(a, fused)


FP_GRID_CASES = NN_GRID_CASES + [("scannet", 1, 8192, 4096)]  # m at the LDS bound


@pytest.mark.parametrize("kind,B,n,m", FP_GRID_CASES)
@pytest.mark.parametrize("C1,C2", [(0, 128), (9, 64), (8, 70), (6, 128)])
def test_fp_grid_fused(env, kind, B, n, m, C1, C2):
    """pn2_fp_grid_fused (each workgroup grids the known points in its own LDS, searches and
    writes its rows) = the oracle's three_nn (dist / idx bit-exact) and the fused scan's rows
    (pn2_fp_fused, bit for bit), with and without an unknown grid ordering the rows."""
    pkg, O, torch, dev = env
    if kind == "fp4":
        x1 = _cloud(pkg, "scannet", B, n, seed=4)
        x2 = O.gather_point(x1, O.fps(x1, m))
    elif kind == "far":
        x1 = _cloud(pkg, "uniform", B, n, seed=4) * np.float32(20.0) - np.float32(10.0)
        x2 = _cloud(pkg, "scannet", B, m, seed=6)
    else:
        x1 = _cloud(pkg, kind if kind != "dup" else "scannet", B, n, seed=4)
        x2 = _cloud(pkg, kind, B, m, seed=8)
        if kind == "grid":
            x1 = x1 + np.float32(0.5)
    t1, t2 = torch.from_numpy(x1).to(dev), torch.from_numpy(x2).to(dev)
    rd, ri = O.three_nn(x1, x2)
    L = pkg.lib()
    st = torch.cuda.current_stream().cuda_stream
    p1 = torch.from_numpy(pkg.synth.features_uniform(1, (B, n, max(C1, 1)))[..., :C1].copy()).to(dev)
    p2 = torch.from_numpy(pkg.synth.features_uniform(2, (B, m, C2))).to(dev)
    ref = torch.empty((B, n, C1 + C2), device=dev)
    if m >= 3:
        assert L.pn2_fp_fused(t1.data_ptr(), t2.data_ptr(), p1.data_ptr() if C1 else None, C1,
                              p2.data_ptr(), C2, B, n, m, ref.data_ptr(), st) == 0
    ug = pkg.grid.PointGrid(t1, 0.1)
    for u in (None, ug):
        out = torch.full((B, n, C1 + C2), float("nan"), device=dev)
        d = torch.empty((B, n, 3), device=dev)
        i = torch.empty((B, n, 3), dtype=torch.int32, device=dev)
        assert L.pn2_fp_grid_fused(t1.data_ptr() if u is None else None, t2.data_ptr(),
                                   None if u is None else u.buf.data_ptr(),
                                   p1.data_ptr() if C1 else None, C1, p2.data_ptr(), C2, B, n, m,
                                   out.data_ptr(), d.data_ptr(), i.data_ptr(), st) == 0
        assert np.array_equal(i.cpu().numpy(), ri)
        assert np.array_equal(_bits(d.cpu().numpy()), _bits(rd))
        if m >= 3:
            assert torch.equal(out, ref)
            # the interpolated columns against the oracle too (not only the other HIP kernel),
            # the concat columns as a copy
            oref = O.fp_fused(x1, x2, p1.cpu().numpy() if C1 else None, p2.cpu().numpy())
            np.testing.assert_allclose(out.cpu().numpy(), oref, **TOL)
            if C1:
                assert np.array_equal(_bits(out[..., C2:].cpu().numpy()), _bits(p1.cpu().numpy()))
        # without the neighbour outputs, through the op wrapper
        a = pkg.pointnet_util.fp_interpolate(t1, t2, p1 if C1 else None, p2, unknown_grid=u)
        if m >= 3 and pkg.tf_interpolate.use_grid(n, m):
            assert torch.equal(a, ref)
    # m beyond the LDS bound, and one neighbour output without the other
    assert L.pn2_fp_grid_fused(t1.data_ptr(), t2.data_ptr(), None, None, 0, p2.data_ptr(), C2, B,
                               n, 4097, out.data_ptr(), None, None, st) == -22
    assert L.pn2_fp_grid_fused(t1.data_ptr(), t2.data_ptr(), None, None, 0, p2.data_ptr(), C2, B,
                               n, m, out.data_ptr(), d.data_ptr(), None, st) == -22


@pytest.mark.parametrize("C", [1, 16, 128, 512])
def test_three_interpolate_and_idw(env, C):
    pkg, O, torch, dev = env
    x1 = _cloud(pkg, "scannet", 2, 1024, seed=2)
    x2 = _cloud(pkg, "scannet", 2, 256, seed=7)
    rd, ri = O.three_nn(x1, x2)
    w = pkg.tf_interpolate.idw_weights(torch.from_numpy(rd).to(dev)).cpu().numpy()
    rw = O.idw_weights(rd)
    np.testing.assert_allclose(w, rw, **TOL)
    pts = pkg.synth.features_uniform(C, (2, 256, C))
    got = pkg.tf_interpolate.three_interpolate(torch.from_numpy(pts).to(dev),
                                               torch.from_numpy(ri).to(dev),
                                               torch.from_numpy(rw).to(dev))
    assert np.array_equal(_bits(got.cpu().numpy()), _bits(O.three_interpolate(pts, ri, rw)))


@pytest.mark.parametrize("n,m,C1,C2", [(64, 16, 256, 512), (256, 64, 128, 256),
                                       (1024, 256, 64, 256), (8192, 1024, 0, 128),
                                       (8192, 1024, 6, 128), (300, 5, 3, 7),
                                       # channel counts whose vector columns do not split
                                       # evenly over the workgroups' channel slices
                                       # (__graft_entry__.smoke's FP layer: 2048 <- 256, 9 + 64)
                                       (2048, 256, 9, 64), (2048, 256, 9, 67), (1024, 128, 5, 60),
                                       (4096, 512, 9, 64), (8192, 1024, 9, 70), (512, 64, 12, 52),
                                       # even C1 not a multiple of 4: float2 concat columns
                                       (1024, 256, 6, 64), (512, 64, 2, 52), (256, 64, 10, 128)])
def test_fp_fused(env, n, m, C1, C2):
    pkg, O, torch, dev = env
    x1 = _cloud(pkg, "scannet", 2, n, seed=11)
    x2 = O.gather_point(x1, O.fps(x1, m))
    p1 = pkg.synth.features_uniform(1, (2, n, C1)) if C1 else None
    p2 = pkg.synth.features_uniform(2, (2, m, C2))
    t = lambda a: None if a is None else torch.from_numpy(a).to(dev)
    got = pkg.pointnet_util.fp_interpolate(t(x1), t(x2), t(p1), t(p2)).cpu().numpy()
    ref = O.fp_fused(x1, x2, p1, p2)
    np.testing.assert_allclose(got, ref, **TOL)
    if C1:
        assert np.array_equal(_bits(got[..., C2:]), _bits(p1))  # the concat is a copy


@pytest.mark.parametrize("ns,C", [(32, 64), (32, 128), (32, 512), (16, 64), (64, 256),
                                  (128, 128), (8, 32), (24, 64), (100, 8)])
def test_attention_reduce(env, ns, C):
    pkg, O, torch, dev = env
    rng = np.random.default_rng(ns * 1000 + C)
    B, M = 2, 37
    Q = rng.uniform(-1, 1, (B, M, C)).astype(np.float32)
    K = rng.uniform(-1, 1, (B, M, ns, C)).astype(np.float32)
    V = rng.uniform(-1, 1, (B, M, ns, C)).astype(np.float32)
    t = lambda a: torch.from_numpy(a).to(dev)
    got = pkg.attention_layer.attention_reduce(t(Q), t(K), t(V)).cpu().numpy()
    np.testing.assert_allclose(got, O.attn_reduce(Q, K, V), **TOL)


def _torch_attention(Q, K, V):
    """attention_layer.py:35-42 in plain torch (float64 on the CPU): the test's reference for
    the floating-point attention kernels, reshape quirk included."""
    import torch
    B, M, ns, C = K.shape
    H = C // 4
    q = Q.reshape(B, M, H, 1, 4)
    k = K.reshape(B, M, H, ns, 4)
    v = V.reshape(B, M, H, ns, 4)
    w = torch.softmax(q @ k.transpose(-1, -2) / 2.0, dim=-1)
    return (w @ v).reshape(B, M, C)


@pytest.mark.parametrize("ns,C", [(32, 64), (16, 128), (128, 256), (24, 12)])
def test_attention_reduce_grad(env, ns, C):
    """Backward of the attention reduction (pn2_attn_reduce_grad, through autograd) against
    torch autograd of the same math in float64; rtol = atol = 1e-5."""
    pkg, O, torch, dev = env
    rng = np.random.default_rng(ns + C)
    B, M = 2, 19
    Q = rng.uniform(-1, 1, (B, M, C)).astype(np.float32)
    K = rng.uniform(-1, 1, (B, M, ns, C)).astype(np.float32)
    V = rng.uniform(-1, 1, (B, M, ns, C)).astype(np.float32)
    G = rng.uniform(-1, 1, (B, M, C)).astype(np.float32)
    ts = [torch.from_numpy(a).to(dev).requires_grad_(True) for a in (Q, K, V)]
    out = pkg.attention_layer.attention_reduce(*ts)
    out.backward(torch.from_numpy(G).to(dev))
    rs = [torch.from_numpy(a).double().requires_grad_(True) for a in (Q, K, V)]
    ref = _torch_attention(*rs)
    ref.backward(torch.from_numpy(G).double())
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), **TOL)
    for t, r in zip(ts, rs):
        np.testing.assert_allclose(t.grad.cpu().numpy(), r.grad.numpy(), **TOL)


@pytest.mark.parametrize("mode", ["max", "avg", "weighted_avg", "max_and_avg"])
def test_group_pool(env, mode):
    pkg, O, torch, dev = env
    rng = np.random.default_rng(4)
    x = rng.uniform(-1, 1, (2, 50, 32, 64)).astype(np.float32)
    g = rng.uniform(-0.2, 0.2, (2, 50, 32, 3)).astype(np.float32)
    got = pkg.pointnet_util.group_pool(torch.from_numpy(x).to(dev), mode,
                                       torch.from_numpy(g).to(dev)).cpu().numpy()
    np.testing.assert_allclose(got, O.group_pool(x, g, mode), **TOL)


def test_gradients(env):
    pkg, O, torch, dev = env
    rng = np.random.default_rng(8)
    x = _cloud(pkg, "scannet", 2, 1024)
    idx = rng.integers(0, 1024, (2, 200)).astype(np.int32)
    og = rng.standard_normal((2, 200, 3)).astype(np.float32)
    g = pkg.tf_sampling.gather_point_grad(torch.from_numpy(x).to(dev),
                                          torch.from_numpy(idx).to(dev), torch.from_numpy(og).to(dev))
    np.testing.assert_allclose(g.cpu().numpy(), O.gather_point_grad(1024, idx, og), **TOL)
    pts = rng.standard_normal((2, 1024, 16)).astype(np.float32)
    gi = rng.integers(0, 1024, (2, 64, 32)).astype(np.int32)
    go = rng.standard_normal((2, 64, 32, 16)).astype(np.float32)
    g = pkg.tf_grouping.group_point_grad(torch.from_numpy(pts).to(dev),
                                         torch.from_numpy(gi).to(dev), torch.from_numpy(go).to(dev))
    np.testing.assert_allclose(g.cpu().numpy(), O.group_point_grad(1024, gi, go), **TOL)
    d, i = O.three_nn(_cloud(pkg, "scannet", 2, 512, 3), _cloud(pkg, "scannet", 2, 128, 4))
    w = O.idw_weights(d)
    go = rng.standard_normal((2, 512, 16)).astype(np.float32)
    g = pkg.tf_interpolate.three_interpolate_grad(torch.zeros((2, 128, 16), device=dev),
                                                  torch.from_numpy(i).to(dev),
                                                  torch.from_numpy(w).to(dev),
                                                  torch.from_numpy(go).to(dev))
    np.testing.assert_allclose(g.cpu().numpy(), O.three_interpolate_grad(128, i, w, go), **TOL)
    # autograd wiring: d/dpoints of sum(group_point(points, idx)) = occurrence counts
    p = torch.from_numpy(pts).to(dev).requires_grad_(True)
    pkg.tf_grouping.group_point(p, torch.from_numpy(gi).to(dev)).sum().backward()
    counts = np.zeros((2, 1024), np.float32)
    for b in range(2):
        np.add.at(counts[b], gi[b].ravel(), 1.0)
    np.testing.assert_allclose(p.grad.cpu().numpy(), np.repeat(counts[..., None], 16, -1), **TOL)


@pytest.mark.parametrize("config,B", [("cfg2", 4), ("cfg3", 2), ("cfg5", 2)])
def test_graph_replay_matches_eager(env, config, B):
    """The hipGraph-captured step (what bench.py times) reproduces the eager step exactly."""
    pkg, O, torch, dev = env
    inp = pkg.stack.make_inputs(config, list(range(10, 10 + B)), dev)
    eager = [o.clone() for o in pkg.stack.run(inp)]
    g = pkg.stack.GraphStep(inp)
    for _ in range(3):
        outs = g.replay()
    torch.cuda.synchronize()
    assert len(outs) == len(eager)
    for a, b in zip(outs, eager):
        assert torch.equal(a, b)


GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: p.rsplit("/", 1)[-1][:-4])
def test_hip_reproduces_golden(env, path):
    """Every golden vector the reference's own code produced (tests/golden/make_golden*.py),
    reproduced by the HIP path through the C ABI: indices bit-exact, floats bit-exact where
    the reference's expression order is kept, gradients (float atomics) within 1e-5."""
    pkg, O, torch, dev = env
    z = np.load(path, allow_pickle=False)
    d = {k: z[k] for k in z.files}
    meta = json.loads(str(d["meta"]))
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    op = meta["op"]
    if op in ("query_ball_point", "query_ball_point_gpu"):
        idx, cnt = pkg.tf_grouping.query_ball_point(meta["radius"], meta["nsample"],
                                                    T(d["xyz1"]), T(d["xyz2"]))
        idx, cnt = idx.cpu().numpy(), cnt.cpu().numpy()
        hit = d["idx"][..., 0] != -1
        assert np.array_equal(idx[hit], d["idx"][hit])
        if "pts_cnt" in d:
            assert np.array_equal(cnt, d["pts_cnt"])
    elif op == "group_point(+grad)":
        out = pkg.tf_grouping.group_point(T(d["points"]), T(d["idx"])).cpu().numpy()
        assert np.array_equal(_bits(out), _bits(d["out"]))
        g = pkg.tf_grouping.group_point_grad(T(d["points"]), T(d["idx"]), T(d["grad_out"]))
        np.testing.assert_allclose(g.cpu().numpy(), d["grad_points"], **TOL)
    elif op == "three_nn":
        dist, idx = pkg.tf_interpolate.three_nn(T(d["xyz1"]), T(d["xyz2"]))
        assert np.array_equal(idx.cpu().numpy(), d["idx"])
        assert np.array_equal(_bits(dist.cpu().numpy()), _bits(d["dist"]))
    elif op in ("three_interpolate", "three_interpolate(+grad)"):
        out = pkg.tf_interpolate.three_interpolate(T(d["points"]), T(d["idx"]), T(d["weight"]))
        assert np.array_equal(_bits(out.cpu().numpy()), _bits(d["out"]))
        if "grad_out" in d:
            g = pkg.tf_interpolate.three_interpolate_grad(T(d["points"]), T(d["idx"]),
                                                          T(d["weight"]), T(d["grad_out"]))
            np.testing.assert_allclose(g.cpu().numpy(), d["grad_points"], **TOL)
    elif op == "selection_sort":
        oi, oo = pkg.tf_grouping.select_top_k(int(meta["k"]), T(d["dist"]))
        assert np.array_equal(oi.cpu().numpy(), d["outi"])
        assert np.array_equal(_bits(oo.cpu().numpy()), _bits(d["out"]))
    elif op == "farthest_point_sample":
        idx, new_xyz = pkg.tf_sampling.farthest_point_sample_and_gather(int(meta["npoint"]),
                                                                        T(d["xyz"]))
        assert np.array_equal(idx.cpu().numpy(), d["idx"])
        assert np.array_equal(_bits(new_xyz.cpu().numpy()), _bits(d["new_xyz"]))
    elif op == "prob_sample":
        got = pkg.tf_sampling.prob_sample(T(d["inp"]), T(d["inpr"]))
        assert np.array_equal(got.cpu().numpy(), d["out"])
    else:
        pytest.fail(f"unknown golden op {op}")


@pytest.mark.parametrize("config,B", [("cfg2", 4), ("cfg3", 2), ("cfg5", 2)])
def test_side_stream_overlap_matches_single_stream(env, config, B):
    """The forked step (sampler chain on one stream, per-layer work on a side stream) gives
    exactly the single-stream outputs, eagerly and under hipGraph replay."""
    pkg, O, torch, dev = env
    inp = pkg.stack.make_inputs(config, list(range(20, 20 + B)), dev)
    single = [o.clone() for o in pkg.stack.Step(inp, overlap=False)()]
    forked = pkg.stack.Step(inp, overlap=True)()
    torch.cuda.synchronize()
    assert len(single) == len(forked)
    for a, b in zip(single, forked):
        assert torch.equal(a, b)
    g = pkg.stack.GraphStep(inp, overlap=True)
    for _ in range(3):
        outs = g.replay()
    torch.cuda.synchronize()
    for a, b in zip(single, outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("graphs", [True, False])
def test_pipelined_steps_match_single_stream(env, graphs):
    """Software-pipelined steps (two buffer sets, bench.py's default) produce, in both sets,
    exactly the single-stream step's outputs."""
    pkg, O, torch, dev = env
    inp = pkg.stack.make_inputs("cfg2", list(range(30, 34)), dev)
    single = [o.clone() for o in pkg.stack.Step(inp, overlap=False)()]
    pipe = pkg.stack.Pipeline(inp, graphs=graphs)
    for _ in range(5):
        pipe.run()
    last = pipe.join()
    torch.cuda.synchronize()
    for outs in [last] + [s.join() for s in pipe.sets]:
        assert len(outs) == len(single)
        for a, b in zip(single, outs):
            assert torch.equal(a, b)


def _ties(rng, shape, levels):
    return rng.integers(0, levels, shape).astype(np.float32)


@pytest.mark.parametrize("kind,B,m,n,k", [
    ("uniform", 2, 37, 300, 16), ("ties", 2, 40, 200, 32), ("ties", 1, 64, 64, 64),
    ("signed", 2, 17, 129, 1), ("ties", 2, 33, 1000, 100), ("dups", 1, 8, 40, 8)])
def test_select_top_k(env, kind, B, m, n, k):
    """select_top_k (knn.hip) against the oracle's literal selection sort and the reference's
    selection_sort_gpu on this GPU: both (b,m,n) outputs bit-exact, ties included (the swaps
    of the partial selection sort decide their order)."""
    pkg, O, torch, dev = env
    rng = np.random.default_rng(n + k)
    if kind == "uniform":
        d = rng.random((B, m, n)).astype(np.float32)
    elif kind == "signed":
        d = rng.standard_normal((B, m, n)).astype(np.float32)
    elif kind == "dups":
        d = np.zeros((B, m, n), np.float32)
    else:
        d = _ties(rng, (B, m, n), 5)
    outi, out = pkg.tf_grouping.select_top_k(k, torch.from_numpy(d).to(dev))
    ri, ro = O.selection_sort(d, k)
    assert np.array_equal(outi.cpu().numpy(), ri)
    assert np.array_equal(_bits(out.cpu().numpy()), _bits(ro))
    if O.have_ref_gpu():
        dt = torch.from_numpy(d).to(dev)
        gi = torch.zeros((B, m, n), dtype=torch.int32, device=dev)
        go = torch.zeros((B, m, n), dtype=torch.float32, device=dev)
        assert O.ref_gpu().pn2ref_selection_sort(dt.data_ptr(), B, m, n, k, gi.data_ptr(),
                                                 go.data_ptr()) == 0
        assert np.array_equal(gi.cpu().numpy(), ri), "oracle differs from selection_sort_gpu"


@pytest.mark.parametrize("kind,B,n,m,c,k", [
    ("scannet", 2, 2048, 256, 3, 32), ("grid", 2, 1000, 100, 3, 16), ("uniform", 1, 500, 64, 6, 8),
    ("dup", 1, 300, 10, 3, 20), ("scannet", 1, 8192, 128, 3, 64)])
def test_knn_point(env, kind, B, n, m, c, k):
    pkg, O, torch, dev = env
    if c == 3:
        x = _cloud(pkg, kind, B, n)
    else:
        x = np.random.default_rng(c).random((B, n, c)).astype(np.float32)
    q = x[:, ::max(1, n // m)][:, :m].copy()
    val, idx = pkg.tf_grouping.knn_point(k, torch.from_numpy(x).to(dev), torch.from_numpy(q).to(dev))
    rv, ri = O.knn_point(k, x, q)
    assert np.array_equal(idx.cpu().numpy(), ri)
    assert np.array_equal(_bits(val.cpu().numpy()), _bits(rv))


def test_sample_and_group_knn(env):
    pkg, O, torch, dev = env
    x = _cloud(pkg, "scannet", 2, 2048, seed=3)
    pts = pkg.synth.features_uniform(5, (2, 2048, 8))
    new_xyz, new_points, idx, grouped_xyz = pkg.pointnet_util.sample_and_group(
        128, 0.2, 16, torch.from_numpy(x).to(dev), torch.from_numpy(pts).to(dev), knn=True)
    rnx = O.gather_point(x, O.fps(x, 128))
    _, ridx = O.knn_point(16, x, rnx)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    rnp, rgx = O.group_concat(x, pts, rnx, ridx)
    assert np.array_equal(_bits(new_points.cpu().numpy()), _bits(rnp))


@pytest.mark.parametrize("kind,B,N,npoints", [
    ("scannet", 3, 8192, [1024, 256, 64, 16]), ("uniform", 2, 3000, [700, 128, 32]),
    ("grid", 2, 4096, [512, 100]), ("dup", 1, 700, [40, 20, 5, 3]), ("uniform", 2, 64, [16]),
    ("scannet", 1, 8192, [1024, 1000, 900, 50]), ("uniform", 2, 1024, [100, 300]),
    ("grid", 2, 1000, [1000, 700, 64]), ("dup", 3, 1024, [256, 64, 16]),
    ("fewuniq", 2, 1024, [512, 400])])
def test_fps_chain(env, kind, B, N, npoints):
    """pn2_fps_chain (every SSG sampler of a cloud in one workgroup) gives exactly the
    per-stage farthest_point_sample_and_gather results, and the oracle's indices."""
    pkg, O, torch, dev = env
    x = _cloud(pkg, kind, B, N)
    xt = torch.from_numpy(x).to(dev)
    outs = pkg.tf_sampling.farthest_point_sample_chain(npoints, xt)
    cur, cur_np = xt, x
    for (idx, nx), m in zip(outs, npoints):
        ridx, rnx = pkg.tf_sampling.farthest_point_sample_and_gather(m, cur)
        assert torch.equal(idx, ridx) and torch.equal(nx, rnx)
        assert np.array_equal(idx.cpu().numpy(), O.fps(cur_np, m))
        cur, cur_np = nx, nx.cpu().numpy()


def _grid_parts(buf, B, N):
    """(header words, offsets, per-cell sorted point rows) of every cloud of a grid buffer
    (csrc/grid.h layout): the order of the points inside a cell is not part of the contract."""
    import numpy as np_
    kcap = 32768
    off_bytes = ((32 + (kcap + 1) * 4) + 15) & ~15
    stride = off_bytes + N * 16
    raw = buf.cpu().numpy()
    out = []
    for b in range(B):
        g = raw[b * stride:(b + 1) * stride]
        hdr = g[:32].view(np_.uint32)
        ncell = int(g[28:32].view(np_.int32)[0])
        off = g[32:32 + (ncell + 1) * 4].view(np_.int32).copy()
        pts = g[off_bytes:off_bytes + N * 16].view(np_.uint32).reshape(N, 4)
        cells = [sorted(map(tuple, pts[off[c]:off[c + 1]])) for c in range(ncell)]
        out.append((hdr.copy(), off, cells))
    return out


@pytest.mark.parametrize("kind,B,N,npoints", [
    ("scannet", 3, 8192, [1024, 256, 64, 16]),  # culled sampler: grid built in its epilogue
    ("scannet", 1, 8192, [4096]),               # the epilogue's bound (M = 4096)
    ("dup", 1, 8192, [1024]),                    # one repeated point: a single cell
    ("uniform", 2, 3000, [700, 128, 32]),        # block-scan sampler + a grid build launch
    ("uniform", 2, 900, [300, 40]),              # stage 0 inside the chain kernel
    ("uniform", 2, 16384, [512])])               # MSG-size sampler + a grid build launch
def test_fps_chain_grid(env, kind, B, N, npoints):
    """pn2_fps_chain_grid: the chain's picks exactly as pn2_fps_chain, and grid0 = the
    automatic-edge pn2_grid_build over stage 0's new_xyz (same header and cell offsets, same
    points per cell); FP4 over it (pn2_fp_grid_fused_known, also through the native plan)
    equals the fused scan bit for bit, and an explicit-edge known grid falls back to the
    in-workgroup build with the same result."""
    pkg, O, torch, dev = env
    x = _cloud(pkg, kind, B, N)
    xt = torch.from_numpy(x).to(dev)
    ref = pkg.tf_sampling.farthest_point_sample_chain(npoints, xt)
    outs = [(torch.empty_like(i), torch.empty_like(n)) for i, n in ref]
    g0 = pkg.grid.PointGrid(outs[0][1], build=False)
    g0.buf.fill_(0xA5)
    pkg.tf_sampling.farthest_point_sample_chain(npoints, xt, out=outs, grid0=g0)
    for (i, n), (ri, rn) in zip(outs, ref):
        assert torch.equal(i, ri) and torch.equal(n, rn)
    built = pkg.grid.PointGrid(ref[0][1])
    for (h, o, c), (rh, ro, rc) in zip(_grid_parts(g0.buf, B, npoints[0]),
                                       _grid_parts(built.buf, B, npoints[0])):
        assert np.array_equal(h, rh) and np.array_equal(o, ro) and c == rc
    # the same launch recorded in a native plan
    outs2 = [(torch.empty_like(i), torch.empty_like(n)) for i, n in ref]
    g2 = pkg.grid.PointGrid(outs2[0][1], build=False)
    plan = pkg.plan.Plan()
    st = torch.cuda.current_stream()
    plan.fps_chain(npoints, xt, outs2, st, g2)
    plan.launch()
    torch.cuda.synchronize()
    assert torch.equal(g2.buf, g0.buf) or all(
        np.array_equal(a[1], b[1]) and a[2] == b[2]
        for a, b in zip(_grid_parts(g2.buf, B, npoints[0]), _grid_parts(g0.buf, B, npoints[0])))
    for (i, n), (ri, rn) in zip(outs2, ref):
        assert torch.equal(i, ri) and torch.equal(n, rn)
    # FP4 over the prebuilt grid
    m = npoints[0]
    if m < 3:
        return
    x2 = ref[0][1]
    C1, C2 = 9, 64
    p1 = torch.from_numpy(pkg.synth.features_uniform(1, (B, N, C1))).to(dev)
    p2 = torch.from_numpy(pkg.synth.features_uniform(2, (B, m, C2))).to(dev)
    L = pkg.lib()
    fused = torch.empty((B, N, C1 + C2), device=dev)
    assert L.pn2_fp_fused(xt.data_ptr(), x2.data_ptr(), p1.data_ptr(), C1, p2.data_ptr(), C2,
                          B, N, m, fused.data_ptr(), st.cuda_stream) == 0
    rd, ri = O.three_nn(x, x2.cpu().numpy())
    ug = pkg.grid.PointGrid(xt, 0.1)
    for kg in (g0, pkg.grid.PointGrid(x2, 0.02)):
        for u in (None, ug):
            out = torch.full((B, N, C1 + C2), float("nan"), device=dev)
            d = torch.empty((B, N, 3), device=dev)
            i = torch.empty((B, N, 3), dtype=torch.int32, device=dev)
            assert L.pn2_fp_grid_fused_known(
                kg.buf.data_ptr(), xt.data_ptr(), x2.data_ptr(),
                None if u is None else u.buf.data_ptr(), p1.data_ptr(), C1, p2.data_ptr(), C2,
                B, N, m, out.data_ptr(), d.data_ptr(), i.data_ptr(), st.cuda_stream) == 0
            assert torch.equal(out, fused)
            assert np.array_equal(i.cpu().numpy(), ri)
            assert np.array_equal(_bits(d.cpu().numpy()), _bits(rd))
    if pkg.tf_interpolate.use_grid(N, m):
        a = pkg.pointnet_util.fp_interpolate(xt, x2, p1, p2, known_grid=g0, unknown_grid=ug)
        assert torch.equal(a, fused)
