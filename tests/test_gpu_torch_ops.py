"""MI355X: the torch.ops.pn2 operators (csrc/torch_ops.cpp) against the oracle, their autograd
against the oracle's gradient restatements, torch.library.opcheck (schema, fake tensors,
autograd registration), and one SA layer under torch.compile(fullgraph=True) bit-exact against
eager and against the oracle. Tolerances: indices and copies bit-exact; IDW / attention /
gradient sums 1e-5 (north_star)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-5, atol=1e-5)


@pytest.fixture(scope="module")
def env():
    import torch

    import pn2hip
    from oracle import oracle as O
    O.set_threads(16)
    return pn2hip, pn2hip.ops, O, torch, torch.device("cuda:0")


def _crops(pn2hip, ids, N):
    return pn2hip.synth.batch(ids, N, "scannet")[0]


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


@pytest.mark.parametrize("N,M", [(1024, 256), (8192, 1024), (20000, 512)])
def test_fps_gather(env, N, M):
    pn2hip, ops, O, torch, dev = env
    x = _crops(pn2hip, [3, 4], N)
    xt = torch.from_numpy(x).to(dev)
    idx = ops.farthest_point_sample(M, xt)
    i2, nx = ops.farthest_point_sample_and_gather(M, xt)
    want = O.fps(x, M)
    assert np.array_equal(idx.cpu().numpy(), want)
    assert np.array_equal(i2.cpu().numpy(), want)
    assert np.array_equal(_bits(nx.cpu().numpy()), _bits(O.gather_point(x, want)))
    g = ops.gather_point(xt, idx)
    assert np.array_equal(_bits(g.cpu().numpy()), _bits(O.gather_point(x, want)))


@pytest.mark.parametrize("N,M,r,ns", [(8192, 1024, 0.1, 32), (1024, 256, 0.2, 32),
                                      (4096, 128, 0.4, 128)])
def test_ball_query_group(env, N, M, r, ns):
    pn2hip, ops, O, torch, dev = env
    x = _crops(pn2hip, [5, 6], N)
    q = O.gather_point(x, O.fps(x, M))
    xt, qt = torch.from_numpy(x).to(dev), torch.from_numpy(q).to(dev)
    idx, cnt = ops.query_ball_point(r, ns, xt, qt)
    widx, wcnt = O.ball_query(x, q, r, ns)
    assert np.array_equal(idx.cpu().numpy(), widx) and np.array_equal(cnt.cpu().numpy(), wcnt)
    pts = np.random.default_rng(0).standard_normal((2, N, 6)).astype(np.float32)
    pt = torch.from_numpy(pts).to(dev)
    assert np.array_equal(_bits(ops.group_point(pt, idx).cpu().numpy()),
                          _bits(O.group_point(pts, widx)))
    gx, np_ = ops.group_concat(xt, pt, qt, idx)
    wnp, wgx = O.group_concat(x, pts, q, widx)
    assert np.array_equal(_bits(np_.cpu().numpy()), _bits(wnp))
    assert np.array_equal(_bits(gx.cpu().numpy()), _bits(wgx))


@pytest.mark.parametrize("n,m,C", [(8192, 1024, 128), (256, 64, 256)])
def test_interp(env, n, m, C):
    pn2hip, ops, O, torch, dev = env
    x = _crops(pn2hip, [7, 8], n)
    k = O.gather_point(x, O.fps(x, m))
    xt, kt = torch.from_numpy(x).to(dev), torch.from_numpy(k).to(dev)
    d, i = ops.three_nn(xt, kt)
    wd, wi = O.three_nn(x, k)
    assert np.array_equal(i.cpu().numpy(), wi) and np.array_equal(_bits(d.cpu().numpy()), _bits(wd))
    w = ops.idw_weights(d)
    np.testing.assert_allclose(w.cpu().numpy(), O.idw_weights(wd), **TOL)
    p2 = np.random.default_rng(1).uniform(-1, 1, (2, m, C)).astype(np.float32)
    ww = O.idw_weights(wd)
    out = ops.three_interpolate(torch.from_numpy(p2).to(dev), i, torch.from_numpy(ww).to(dev))
    assert np.array_equal(_bits(out.cpu().numpy()), _bits(O.three_interpolate(p2, wi, ww)))
    p1 = np.random.default_rng(2).uniform(-1, 1, (2, n, 6)).astype(np.float32)
    fp = ops.fp_fused(xt, kt, torch.from_numpy(p1).to(dev), torch.from_numpy(p2).to(dev))
    np.testing.assert_allclose(fp.cpu().numpy(), O.fp_fused(x, k, p1, p2), **TOL)


def test_knn_select_attn_pool(env):
    pn2hip, ops, O, torch, dev = env
    rng = np.random.default_rng(3)
    x = _crops(pn2hip, [9], 2048)
    q = O.gather_point(x, O.fps(x, 128))
    v, i = ops.knn_point(16, torch.from_numpy(x).to(dev), torch.from_numpy(q).to(dev))
    wv, wi = O.knn_point(16, x, q)
    assert np.array_equal(i.cpu().numpy(), wi) and np.array_equal(_bits(v.cpu().numpy()), _bits(wv))
    dist = rng.integers(0, 50, (2, 64, 300)).astype(np.float32)  # many ties
    oi, oo = ops.select_top_k(10, torch.from_numpy(dist).to(dev))
    woi, woo = O.selection_sort(dist, 10)
    assert np.array_equal(oi.cpu().numpy(), woi) and np.array_equal(oo.cpu().numpy(), woo)
    Q = rng.standard_normal((2, 64, 64)).astype(np.float32)
    K = rng.standard_normal((2, 64, 32, 64)).astype(np.float32)
    V = rng.standard_normal((2, 64, 32, 64)).astype(np.float32)
    a = ops.attn_reduce(*(torch.from_numpy(t).to(dev) for t in (Q, K, V)))
    np.testing.assert_allclose(a.cpu().numpy(), O.attn_reduce(Q, K, V), **TOL)
    for mode, code in (("max", 0), ("avg", 1), ("max_and_avg", 3)):
        p = ops.group_pool(torch.from_numpy(K).to(dev), None, code)
        np.testing.assert_allclose(p.cpu().numpy(), O.group_pool(K, None, mode)[:, :, 0], **TOL)


def test_autograd_vs_oracle(env):
    """Gradients registered for the ops the reference registers them for (points only)."""
    pn2hip, ops, O, torch, dev = env
    rng = np.random.default_rng(4)
    x = _crops(pn2hip, [10, 11], 1024)
    q = O.gather_point(x, O.fps(x, 128))
    widx, _ = O.ball_query(x, q, 0.2, 16)
    pts = rng.standard_normal((2, 1024, 8)).astype(np.float32)
    go = rng.standard_normal((2, 128, 16, 8)).astype(np.float32)
    p = torch.from_numpy(pts).to(dev).requires_grad_(True)
    ops.group_point(p, torch.from_numpy(widx).to(dev)).backward(torch.from_numpy(go).to(dev))
    np.testing.assert_allclose(p.grad.cpu().numpy(), O.group_point_grad(1024, widx, go), **TOL)

    fidx = O.fps(x, 128)
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    og = rng.standard_normal((2, 128, 3)).astype(np.float32)
    ops.gather_point(xt, torch.from_numpy(fidx).to(dev)).backward(torch.from_numpy(og).to(dev))
    np.testing.assert_allclose(xt.grad.cpu().numpy(), O.gather_point_grad(1024, fidx, og), **TOL)

    wd, wi = O.three_nn(x, q)
    ww = O.idw_weights(wd)
    p2 = torch.from_numpy(rng.standard_normal((2, 128, 8)).astype(np.float32)).to(dev)
    p2.requires_grad_(True)
    gi = rng.standard_normal((2, 1024, 8)).astype(np.float32)
    ops.three_interpolate(p2, torch.from_numpy(wi).to(dev), torch.from_numpy(ww).to(dev)) \
        .backward(torch.from_numpy(gi).to(dev))
    np.testing.assert_allclose(p2.grad.cpu().numpy(), O.three_interpolate_grad(128, wi, ww, gi),
                               **TOL)

    # attention reduction: vs float64 torch autograd of the reference's reshape/softmax chain
    Q = torch.randn(2, 16, 32, device=dev, dtype=torch.float64)
    K = torch.randn(2, 16, 8, 32, device=dev, dtype=torch.float64)
    V = torch.randn(2, 16, 8, 32, device=dev, dtype=torch.float64)
    g = torch.randn(2, 16, 32, device=dev, dtype=torch.float64)

    def ref(Q, K, V):  # attention_layer.py:35-42
        B, M, ns, C = K.shape
        H = C // 4
        Kh = K.reshape(B, M, H, ns, 4)
        Vh = V.reshape(B, M, H, ns, 4)
        s = torch.einsum("bmhnd,bmhd->bmhn", Kh, Q.reshape(B, M, H, 4)) / 2.0
        a = torch.softmax(s, -1)
        return torch.einsum("bmhn,bmhnd->bmhd", a, Vh).reshape(B, M, C)

    t64 = [t.clone().requires_grad_(True) for t in (Q, K, V)]
    ref(*t64).backward(g)
    t32 = [t.float().clone().requires_grad_(True) for t in (Q, K, V)]
    ops.attn_reduce(*t32).backward(g.float())
    for a, b in zip(t32, t64):
        np.testing.assert_allclose(a.grad.cpu().numpy(), b.grad.cpu().numpy(), rtol=1e-4, atol=1e-5)


def test_opcheck(env):
    pn2hip, ops, O, torch, dev = env
    x = torch.from_numpy(_crops(pn2hip, [12], 1024)).to(dev)
    idx = ops.farthest_point_sample(64, x)
    q = ops.gather_point(x, idx)
    bidx, _ = ops.query_ball_point(0.2, 16, x, q)
    d, i = ops.three_nn(x, q)
    w = ops.idw_weights(d)
    pts = torch.randn(1, 1024, 8, device=dev)
    utils = ("test_schema", "test_autograd_registration", "test_faketensor")
    cases = [
        (torch.ops.pn2.farthest_point_sample, (64, x)),
        (torch.ops.pn2.gather_point, (x.clone().requires_grad_(True), idx)),
        (torch.ops.pn2.query_ball_point, (0.2, 16, x, q)),
        (torch.ops.pn2.group_point, (pts.clone().requires_grad_(True), bidx)),
        (torch.ops.pn2.three_nn, (x, q)),
        (torch.ops.pn2.three_interpolate, (torch.randn(1, 64, 8, device=dev).requires_grad_(True), i, w)),
        (torch.ops.pn2.attn_reduce, (torch.randn(1, 64, 16, device=dev).requires_grad_(True),
                                     torch.randn(1, 64, 16, 16, device=dev),
                                     torch.randn(1, 64, 16, 16, device=dev))),
    ]
    for op, args in cases:
        torch.library.opcheck(op, args, test_utils=utils)


def test_sa_layer_torch_compile(env):
    """One SSG SA layer (sample_and_group + max pool, pointnet_util.py:16-58,121-145) written
    against pn2hip.ops, compiled with fullgraph=True (no graph break: every op has a schema
    and a Meta kernel) on the aot_eager backend (AOT autograd over fake tensors, no generated
    kernels), equals eager bit-exactly, and its grouping equals the oracle."""
    pn2hip, ops, O, torch, dev = env

    def sa_layer(xyz, points):
        fidx, new_xyz = ops.farthest_point_sample_and_gather(256, xyz)
        idx, _ = ops.query_ball_point(0.2, 32, xyz, new_xyz)
        grouped_xyz = ops.group_point(xyz, idx) - new_xyz.unsqueeze(2)
        new_points = torch.cat([grouped_xyz, ops.group_point(points, idx)], dim=-1)
        return new_xyz, new_points, new_points.max(dim=2).values

    x = _crops(pn2hip, [13, 14], 2048)
    pts = np.random.default_rng(5).standard_normal((2, 2048, 6)).astype(np.float32)
    xt, pt = torch.from_numpy(x).to(dev), torch.from_numpy(pts).to(dev)
    compiled = torch.compile(sa_layer, fullgraph=True, backend="aot_eager")
    eager = sa_layer(xt, pt)
    got = compiled(xt, pt)
    for a, b in zip(got, eager):
        assert torch.equal(a, b)
    fidx = O.fps(x, 256)
    q = O.gather_point(x, fidx)
    widx, _ = O.ball_query(x, q, 0.2, 32)
    wnp, _ = O.group_concat(x, pts, q, widx)
    assert np.array_equal(_bits(got[1].cpu().numpy()), _bits(wnp))


def test_reference_names_drop_in(env):
    """`from tf_sampling import ...` (the reference models' import style) resolves to pn2hip."""
    pn2hip, ops, O, torch, dev = env
    pn2hip.install_reference_names()
    import sys
    from tf_grouping import query_ball_point  # noqa: F401
    from tf_sampling import farthest_point_sample
    assert sys.modules["tf_sampling"] is pn2hip.tf_sampling
    x = _crops(pn2hip, [15], 1024)
    got = farthest_point_sample(128, torch.from_numpy(x).to(dev))
    assert np.array_equal(got.cpu().numpy(), O.fps(x, 128))
