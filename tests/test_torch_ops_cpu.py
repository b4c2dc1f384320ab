"""CPU: the torch.ops.pn2 operator library (csrc/torch_ops.cpp -> libpn2torch.so) loads, every
schema is registered under the reference's names and argument order, the Meta kernels give the
reference output shapes (fake tensors / torch.compile), the shape checks raise ValueError with
the reference's OP_REQUIRES texts, and a CPU tensor is refused (no CPU fallback). No kernel
runs here; tests/test_gpu_torch_ops.py runs them on the MI355X."""
import pytest
import torch


@pytest.fixture(scope="module")
def ops():
    import pn2hip
    return pn2hip.ops


def test_schemas(ops):
    want = {
        "farthest_point_sample": "pn2::farthest_point_sample(int npoint, Tensor inp) -> Tensor",
        "gather_point": "pn2::gather_point(Tensor inp, Tensor idx) -> Tensor",
        "query_ball_point": "pn2::query_ball_point(float radius, int nsample, Tensor xyz1, "
                            "Tensor xyz2) -> (Tensor, Tensor)",
        "group_point": "pn2::group_point(Tensor points, Tensor idx) -> Tensor",
        "three_nn": "pn2::three_nn(Tensor xyz1, Tensor xyz2) -> (Tensor, Tensor)",
        "three_interpolate": "pn2::three_interpolate(Tensor points, Tensor idx, Tensor weight) "
                             "-> Tensor",
        "knn_point": "pn2::knn_point(int k, Tensor xyz1, Tensor xyz2) -> (Tensor, Tensor)",
        "select_top_k": "pn2::select_top_k(int k, Tensor dist) -> (Tensor, Tensor)",
        "attn_reduce": "pn2::attn_reduce(Tensor Q, Tensor K, Tensor V) -> Tensor",
    }
    for name, schema in want.items():
        assert str(getattr(ops, name)._schemas[""]) == schema
    for name in ops.NAMES:
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"pn2::{name}", "CUDA"), name
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"pn2::{name}", "Meta"), name
        # CPU kernels only for the reference's CPU-only ops (tf_interpolate.cpp:187,222,262)
        cpu = name in ("three_nn", "three_interpolate", "three_interpolate_grad")
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"pn2::{name}", "CPU") == cpu, name
    for name in ("gather_point", "group_point", "three_interpolate", "attn_reduce"):
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"pn2::{name}", "Autograd"), name


def test_meta_shapes(ops):
    m = lambda *s, dt=torch.float32: torch.empty(s, device="meta", dtype=dt)  # noqa: E731
    xyz, q = m(2, 1000, 3), m(2, 64, 3)
    assert ops.farthest_point_sample(64, xyz).shape == (2, 64)
    assert ops.farthest_point_sample(64, xyz).dtype == torch.int32
    i, nx = ops.farthest_point_sample_and_gather(64, xyz)
    assert i.shape == (2, 64) and nx.shape == (2, 64, 3)
    assert ops.gather_point(xyz, m(2, 64, dt=torch.int32)).shape == (2, 64, 3)
    idx, cnt = ops.query_ball_point(0.2, 32, xyz, q)
    assert idx.shape == (2, 64, 32) and cnt.shape == (2, 64) and idx.dtype == torch.int32
    assert ops.group_point(m(2, 1000, 7), idx).shape == (2, 64, 32, 7)
    gx, npts = ops.group_concat(xyz, m(2, 1000, 7), q, idx)
    assert gx.shape == (2, 64, 32, 3) and npts.shape == (2, 64, 32, 10)
    d, i3 = ops.three_nn(xyz, q)
    assert d.shape == (2, 1000, 3) and i3.dtype == torch.int32
    assert ops.three_interpolate(m(2, 64, 16), i3, d).shape == (2, 1000, 16)
    assert ops.fp_fused(xyz, q, m(2, 1000, 5), m(2, 64, 16)).shape == (2, 1000, 21)
    v, ik = ops.knn_point(8, xyz, q)
    assert v.shape == (2, 64, 8) and ik.shape == (2, 64, 8)
    assert ops.attn_reduce(m(2, 64, 16), m(2, 64, 32, 16), m(2, 64, 32, 16)).shape == (2, 64, 16)
    assert ops.group_pool(m(2, 64, 32, 16), None, 3).shape == (2, 64, 32)


@pytest.mark.parametrize("call,msg", [
    (lambda o, m: o.farthest_point_sample(0, m(1, 10, 3)), "FarthestPointSample expects positive npoint"),
    (lambda o, m: o.farthest_point_sample(4, m(1, 10, 2)),
     "FarthestPointSample expects (batch_size,num_points,3) inp shape"),
    (lambda o, m: o.query_ball_point(0.0, 8, m(1, 10, 3), m(1, 4, 3)), "QueryBallPoint expects positive radius"),
    (lambda o, m: o.query_ball_point(0.1, 0, m(1, 10, 3), m(1, 4, 3)), "QueryBallPoint expects positive nsample"),
    (lambda o, m: o.group_point(m(1, 10), m(1, 4, 8)),
     "GroupPoint expects (batch_size, num_points, channel) points shape"),
    (lambda o, m: o.three_nn(m(1, 10, 2), m(1, 4, 3)), "ThreeNN expects (b,n,3) xyz1 shape."),
    (lambda o, m: o.three_interpolate(m(1, 4, 5), m(1, 10, 2), m(1, 10, 3)),
     "ThreeInterpolate expects (b,n,3) idx shape"),
])
def test_reference_errors(ops, call, msg):
    m = lambda *s: torch.empty(s, device="meta")  # noqa: E731
    with pytest.raises(ValueError) as e:
        call(ops, m)
    assert msg in str(e.value)


def test_no_cpu_kernel(ops):
    with pytest.raises(NotImplementedError):
        ops.farthest_point_sample(4, torch.zeros(1, 10, 3))
