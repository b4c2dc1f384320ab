"""Seeded random-shape sweep of the geometric ops against the oracle (bit-exact), beyond the
hand-picked cases of test_gpu_parity.py: every case draws B, N, M, radius, nsample, C and the
cloud kind (uniform, ScanNet crop with duplicates, integer lattice with exact ties) from one
seed, then runs the mirror op chain of one SA layer (FPS + gather, ball query, group + centre
+ concat) and one FP layer (three_nn, IDW, interpolate + concat, both search paths) and
compares every index and float bit for bit. Sizes are bounded so the oracle finishes each case
in well under a second."""
import importlib

import numpy as np
import pytest

from conftest import PKG_NAME, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

CASES = 48


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


@pytest.fixture(scope="module")
def env():
    import torch

    from oracle import oracle as O
    O.set_threads(16)
    return importlib.import_module(PKG_NAME), O, torch, torch.device("cuda:0")


def _cloud(pkg, rng, kind, B, N):
    if kind == "lattice":
        g = np.stack(np.meshgrid(*[np.arange(12)] * 3, indexing="ij"), -1).reshape(-1, 3)
        return (g[rng.integers(0, len(g), (B, N))] * 0.05).astype(np.float32)
    seeds = [int(s) for s in rng.integers(0, 1 << 30, B)]
    return pkg.synth.batch(seeds, N, kind)[0]


@pytest.mark.parametrize("seed", range(CASES))
def test_random_sa_fp_layer_vs_oracle(env, seed):
    pkg, O, torch, dev = env
    rng = np.random.default_rng(1000 + seed)
    kind = ["uniform", "scannet", "lattice"][seed % 3]
    B = int(rng.integers(1, 5))
    N = int(rng.choice([37, 300, 513, 1024, 2047, 4096, 5000, 8192, 12000, 16384, 20000]))
    M = int(min(N, rng.choice([1, 16, 64, 100, 256, 512, 1024])))
    ns = int(rng.choice([1, 5, 8, 16, 24, 32, 64, 128]))
    radius = float(rng.choice([0.02, 0.05, 0.1, 0.2, 0.4, 0.8]))
    C = int(rng.choice([0, 3, 6, 16, 64]))
    xyz = _cloud(pkg, rng, kind, B, N)
    pts = rng.uniform(-1, 1, (B, N, C)).astype(np.float32) if C else None
    T = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    what = f"seed {seed}: {kind} B={B} N={N} M={M} ns={ns} r={radius} C={C}"

    # SA: FPS + gather (tf_sampling), ball query (tf_grouping), group + centre + concat
    fidx = O.fps(xyz, M)
    idx, new_xyz = pkg.tf_sampling.farthest_point_sample_and_gather(M, T(xyz))
    assert np.array_equal(idx.cpu().numpy(), fidx), what
    ref_new = O.gather_point(xyz, fidx)
    assert np.array_equal(_bits(new_xyz.cpu().numpy()), _bits(ref_new)), what
    bidx, cnt = pkg.tf_grouping.query_ball_point(radius, ns, T(xyz), new_xyz)
    ridx, rcnt = O.ball_query(xyz, ref_new, radius, ns)
    assert np.array_equal(cnt.cpu().numpy(), rcnt), what
    assert np.array_equal(bidx.cpu().numpy(), ridx), what
    got, gxyz = pkg.pointnet_util.group_concat(T(xyz), T(pts), new_xyz, bidx)
    rgot, rgxyz = O.group_concat(xyz, pts, ref_new, ridx)
    assert np.array_equal(_bits(got.cpu().numpy()), _bits(rgot)), what
    assert np.array_equal(_bits(gxyz.cpu().numpy()), _bits(rgxyz)), what

    # FP: the sampled level back onto the cloud (three_nn + IDW + interpolate + concat)
    C2 = int(rng.choice([3, 16, 64]))
    p2 = rng.uniform(-1, 1, (B, M, C2)).astype(np.float32)
    out = pkg.pointnet_util.fp_interpolate(T(xyz), new_xyz, T(pts), T(p2))
    assert np.array_equal(_bits(out.cpu().numpy()), _bits(O.fp_fused(xyz, ref_new, pts, p2))), what


@pytest.mark.parametrize("seed", range(16))
def test_random_knn_and_grads_vs_oracle(env, seed):
    """knn_point / select_top_k bit-exact; gather / group / interpolate gradients (float
    atomics: summation order not fixed) within 1e-5 of the oracle's sequential sums."""
    pkg, O, torch, dev = env
    rng = np.random.default_rng(5000 + seed)
    kind = ["uniform", "scannet", "lattice"][seed % 3]
    B = int(rng.integers(1, 4))
    n = int(rng.choice([16, 100, 513, 1024, 2048]))
    m = int(rng.choice([1, 7, 64, 256]))
    k = int(min(n, rng.choice([1, 3, 8, 16, 32])))
    xyz1 = _cloud(pkg, rng, kind, B, n)
    xyz2 = _cloud(pkg, rng, kind, B, m)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    what = f"seed {seed}: {kind} B={B} n={n} m={m} k={k}"
    val, idx = pkg.tf_grouping.knn_point(k, T(xyz1), T(xyz2))
    rval, ridx = O.knn_point(k, xyz1, xyz2)
    assert np.array_equal(idx.cpu().numpy(), ridx), what
    assert np.array_equal(_bits(val.cpu().numpy()), _bits(rval)), what

    C = int(rng.choice([3, 8, 64]))
    pts = T(rng.uniform(-1, 1, (B, n, C)).astype(np.float32))
    gidx = T(ridx.astype(np.int32))
    go = rng.uniform(-1, 1, (B, m, k, C)).astype(np.float32)
    g = pkg.tf_grouping.group_point_grad(pts, gidx, T(go)).cpu().numpy()
    np.testing.assert_allclose(g, O.group_point_grad(n, ridx, go), rtol=1e-5, atol=1e-5,
                               err_msg=what)
    fidx = O.fps(xyz1, min(n, m))
    gog = rng.uniform(-1, 1, (B, fidx.shape[1], 3)).astype(np.float32)
    g = pkg.tf_sampling.gather_point_grad(T(xyz1), T(fidx), T(gog)).cpu().numpy()
    np.testing.assert_allclose(g, O.gather_point_grad(n, fidx, gog), rtol=1e-5, atol=1e-5,
                               err_msg=what)
    if m >= 3:
        dist, nidx = O.three_nn(xyz1, xyz2)
        w = O.idw_weights(dist)
        p2 = T(rng.uniform(-1, 1, (B, m, C)).astype(np.float32))
        goi = rng.uniform(-1, 1, (B, n, C)).astype(np.float32)
        g = pkg.tf_interpolate.three_interpolate_grad(p2, T(nidx), T(w), T(goi)).cpu().numpy()
        np.testing.assert_allclose(g, O.three_interpolate_grad(m, nidx, w, goi), rtol=1e-5,
                                   atol=1e-5, err_msg=what)
