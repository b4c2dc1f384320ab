"""The host twins of the reference's CPU-only ops (ThreeNN, ThreeInterpolate(+Grad) are
registered for DEVICE_CPU only, tf_interpolate.cpp:187,222,262): pn2cpu_* (csrc/cpu_interp.cpp)
through the torch ops' CPU kernels and the tf_interpolate mirror, against the oracle and --
where oracle/_ref was built from /root/reference -- the reference's own threenn_cpu /
threeinterpolate_cpu / threeinterpolate_grad_cpu. Bit-exact: same fp32 expression order, and
the gradient's sums in the reference's order within a cloud. Runs without a GPU."""
import numpy as np
import pytest
import torch

from conftest import PKG_NAME

pytestmark = pytest.mark.filterwarnings("ignore::UserWarning")


@pytest.fixture(scope="module")
def env():
    import importlib

    from oracle import oracle as O
    pkg = importlib.import_module(PKG_NAME)
    try:
        pkg._torch_ops.ops()
    except RuntimeError as e:  # the torch-linked library is part of the build
        pytest.fail(str(e))
    return pkg, O


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def _clouds(kind, B, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "grid":  # exact distance ties everywhere
        return rng.integers(0, 6, (B, n, 3)).astype(np.float32)
    if kind == "dup":
        return np.tile(rng.random((1, 1, 3)).astype(np.float32), (B, n, 1))
    return rng.random((B, n, 3)).astype(np.float32)


NN = [("uniform", 2, 512, 128), ("grid", 2, 300, 200), ("dup", 1, 50, 40), ("uniform", 1, 7, 2),
      ("uniform", 1, 9, 1), ("uniform", 3, 2048, 600), ("uniform", 1, 0, 5), ("uniform", 0, 4, 4)]


@pytest.mark.parametrize("kind,B,n,m", NN)
def test_three_nn_host(env, kind, B, n, m):
    pkg, O = env
    x1, x2 = _clouds(kind, B, n, 1), _clouds(kind, B, m, 2)
    d, i = pkg.tf_interpolate.three_nn(torch.from_numpy(x1), torch.from_numpy(x2))
    assert d.device.type == "cpu" and d.shape == (B, n, 3) and i.dtype == torch.int32
    if B * n == 0:
        return
    rd, ri = O.three_nn(x1, x2)
    assert np.array_equal(i.numpy(), ri)
    assert np.array_equal(_bits(d.numpy()), _bits(rd))
    if O.have_ref_cpu():  # the reference's threenn_cpu itself
        fd, fi = O.ref_three_nn(x1, x2)
        assert np.array_equal(i.numpy(), fi) and np.array_equal(_bits(d.numpy()), _bits(fd))


@pytest.mark.parametrize("B,m,n,C", [(2, 64, 256, 16), (1, 3, 10, 1), (2, 128, 1024, 131),
                                     (1, 5, 0, 4)])
def test_three_interpolate_host_and_grad(env, B, m, n, C):
    pkg, O = env
    rng = np.random.default_rng(C)
    pts = rng.standard_normal((B, m, C)).astype(np.float32)
    idx = rng.integers(0, m, (B, n, 3)).astype(np.int32)
    idx[:, ::7, 1] = idx[:, ::7, 0]  # repeated neighbours: the grad's sums stack on one row
    w = rng.random((B, n, 3)).astype(np.float32)
    out = pkg.tf_interpolate.three_interpolate(torch.from_numpy(pts), torch.from_numpy(idx),
                                               torch.from_numpy(w))
    assert np.array_equal(_bits(out.numpy()), _bits(O.three_interpolate(pts, idx, w)))
    go = rng.standard_normal((B, n, C)).astype(np.float32)
    g = pkg.tf_interpolate.three_interpolate_grad(torch.from_numpy(pts), torch.from_numpy(idx),
                                                  torch.from_numpy(w), torch.from_numpy(go))
    if O.have_ref_cpu():  # the reference's own loops: same values and same summation order
        assert np.array_equal(_bits(out.numpy()), _bits(O.ref_three_interpolate(pts, idx, w)))
        assert np.array_equal(_bits(g.numpy()), _bits(O.ref_three_interpolate_grad(m, idx, w, go)))
    np.testing.assert_allclose(g.numpy(), O.three_interpolate_grad(m, idx, w, go),
                               rtol=1e-5, atol=1e-5)
    # autograd w.r.t. points (tf_interpolate.py:29-34) runs the CPU gradient kernel
    p = torch.from_numpy(pts).requires_grad_(True)
    pkg.tf_interpolate.three_interpolate(p, torch.from_numpy(idx), torch.from_numpy(w)).backward(
        torch.from_numpy(go))
    assert np.array_equal(_bits(p.grad.numpy()), _bits(g.numpy()))


def test_host_errors(env):
    pkg, O = env
    ti = pkg.tf_interpolate
    with pytest.raises(pkg._lib.InvalidArgumentError, match="ThreeNN expects"):
        ti.three_nn(torch.zeros(2, 5, 2), torch.zeros(2, 5, 3))
    with pytest.raises(pkg._lib.InvalidArgumentError, match=r"\(b,n,3\) weight"):
        ti.three_interpolate(torch.zeros(1, 4, 2), torch.zeros(1, 3, 3, dtype=torch.int32),
                             torch.zeros(1, 2, 3))
    with pytest.raises(TypeError):
        ti.three_nn(torch.zeros(1, 5, 3, dtype=torch.float64), torch.zeros(1, 5, 3))
    # the other ops keep no CPU path: a CPU tensor fails loudly
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pkg.tf_sampling.farthest_point_sample(4, torch.zeros(1, 16, 3))
