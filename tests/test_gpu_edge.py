"""Empty inputs through every op of the mirror: a zero-size batch, point set or query set gives
an empty output of the right shape (the reference's kernels loop zero times over such inputs),
without a launch and without an error."""
import importlib

import pytest

from conftest import PKG_NAME, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


@pytest.fixture(scope="module")
def env():
    import torch
    return importlib.import_module(PKG_NAME), torch, torch.device("cuda:0")


def test_empty_sampling(env):
    pkg, torch, dev = env
    ts = pkg.tf_sampling
    assert ts.farthest_point_sample(16, torch.zeros(0, 100, 3, device=dev)).shape == (0, 16)
    idx, nx = ts.farthest_point_sample_and_gather(4, torch.zeros(0, 50, 3, device=dev))
    assert idx.shape == (0, 4) and nx.shape == (0, 4, 3)
    g = ts.gather_point(torch.zeros(2, 10, 3, device=dev),
                        torch.zeros(2, 0, dtype=torch.int32, device=dev))
    assert g.shape == (2, 0, 3)
    assert ts.prob_sample(torch.ones(0, 5, device=dev), torch.zeros(0, 3, device=dev)).shape == (0, 3)


def test_empty_grouping(env):
    pkg, torch, dev = env
    tg = pkg.tf_grouping
    idx, cnt = tg.query_ball_point(0.1, 8, torch.rand(2, 100, 3, device=dev),
                                   torch.zeros(2, 0, 3, device=dev))
    assert idx.shape == (2, 0, 8) and cnt.shape == (2, 0)
    out = tg.group_point(torch.rand(2, 100, 5, device=dev),
                         torch.zeros(2, 0, 8, dtype=torch.int32, device=dev))
    assert out.shape == (2, 0, 8, 5)
    val, kidx = tg.knn_point(3, torch.rand(2, 10, 3, device=dev), torch.zeros(2, 0, 3, device=dev))
    assert val.shape == (2, 0, 3) and kidx.shape == (2, 0, 3)


def test_empty_interpolation(env):
    pkg, torch, dev = env
    ti = pkg.tf_interpolate
    dist, idx = ti.three_nn(torch.zeros(2, 0, 3, device=dev), torch.rand(2, 10, 3, device=dev))
    assert dist.shape == (2, 0, 3) and idx.shape == (2, 0, 3)
    out = ti.three_interpolate(torch.rand(2, 10, 4, device=dev),
                               torch.zeros(2, 0, 3, dtype=torch.int32, device=dev),
                               torch.zeros(2, 0, 3, device=dev))
    assert out.shape == (2, 0, 4)


def test_empty_gradients(env):
    """No index points at any input row, so every gradient is zero in the input's shape."""
    pkg, torch, dev = env
    pts = torch.rand(2, 10, 4, device=dev)
    g = pkg.tf_grouping.group_point_grad(pts, torch.zeros(2, 0, 8, dtype=torch.int32, device=dev),
                                         torch.zeros(2, 0, 8, 4, device=dev))
    assert g.shape == (2, 10, 4) and not g.any()
    xyz = torch.rand(2, 10, 3, device=dev)
    g = pkg.tf_sampling.gather_point_grad(xyz, torch.zeros(2, 0, dtype=torch.int32, device=dev),
                                          torch.zeros(2, 0, 3, device=dev))
    assert g.shape == (2, 10, 3) and not g.any()
    g = pkg.tf_interpolate.three_interpolate_grad(pts, torch.zeros(2, 0, 3, dtype=torch.int32, device=dev),
                                                  torch.zeros(2, 0, 3, device=dev),
                                                  torch.zeros(2, 0, 4, device=dev))
    assert g.shape == (2, 10, 4) and not g.any()


def test_empty_layers(env):
    pkg, torch, dev = env
    pu = pkg.pointnet_util
    xyz = torch.rand(2, 64, 3, device=dev)
    new_xyz = torch.zeros(2, 0, 3, device=dev)
    idx = torch.zeros(2, 0, 8, dtype=torch.int32, device=dev)
    g, gx = pu.group_concat(xyz, torch.rand(2, 64, 6, device=dev), new_xyz, idx)
    assert g.shape == (2, 0, 8, 9) and gx.shape == (2, 0, 8, 3)
    out = pu.fp_interpolate(torch.zeros(2, 0, 3, device=dev), xyz, None,
                            torch.rand(2, 64, 16, device=dev))
    assert out.shape == (2, 0, 16)
