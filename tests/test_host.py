"""CPU: host-side logic of the drop-in modules — argument checks with the reference's
InvalidArgumentError messages, the no-CPU-fallback rule, the synthetic generators, the
benchmark byte accounting, and the oracle's full step."""
import numpy as np
import pytest
import torch


def test_reference_error_messages(pn2):
    E = pn2.InvalidArgumentError
    x = torch.zeros(2, 10, 4)
    with pytest.raises(E, match="FarthestPointSample expects positive npoint"):
        pn2.tf_sampling.farthest_point_sample(0, torch.zeros(2, 10, 3))
    with pytest.raises(E, match=r"FarthestPointSample expects \(batch_size,num_points,3\) inp shape"):
        pn2.tf_sampling.farthest_point_sample(4, x)
    with pytest.raises(E, match=r"GatherPoint expects \(batch_size,num_result\) idx shape"):
        pn2.tf_sampling.gather_point(torch.zeros(2, 10, 3), torch.zeros(3, 4, dtype=torch.int32))
    with pytest.raises(E, match="QueryBallPoint expects positive radius"):
        pn2.tf_grouping.query_ball_point(0.0, 8, torch.zeros(1, 5, 3), torch.zeros(1, 2, 3))
    with pytest.raises(E, match="QueryBallPoint expects positive nsample"):
        pn2.tf_grouping.query_ball_point(0.1, 0, torch.zeros(1, 5, 3), torch.zeros(1, 2, 3))
    with pytest.raises(E, match=r"QueryBallPoint expects \(batch_size, npoint, 3\) xyz2 shape."):
        pn2.tf_grouping.query_ball_point(0.1, 4, torch.zeros(1, 5, 3), torch.zeros(1, 2, 2))
    with pytest.raises(E, match=r"GroupPoint expects \(batch_size, npoints, nsample\) idx shape"):
        pn2.tf_grouping.group_point(torch.zeros(1, 5, 3), torch.zeros(1, 2, dtype=torch.int32))
    with pytest.raises(E, match=r"ThreeNN expects \(b,n,3\) xyz1 shape."):
        pn2.tf_interpolate.three_nn(torch.zeros(1, 5), torch.zeros(1, 2, 3))
    with pytest.raises(E, match=r"ThreeInterpolate expects \(b,n,3\) weight shape"):
        pn2.tf_interpolate.three_interpolate(torch.zeros(1, 4, 8), torch.zeros(1, 6, 3, dtype=torch.int32),
                                             torch.zeros(1, 5, 3))


def test_no_cpu_fallback(pn2):
    """Well-formed CPU tensors are refused: the product path is the HIP library only (except
    ThreeNN / ThreeInterpolate(+Grad), the reference's own CPU-only ops, which run the host
    twins pn2cpu_*: tests/test_cpu_interp.py)."""
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pn2.tf_sampling.farthest_point_sample(4, torch.zeros(1, 10, 3))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pn2.tf_grouping.query_ball_point(0.2, 8, torch.zeros(1, 10, 3), torch.zeros(1, 4, 3))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pn2.attention_layer.attention_reduce(torch.zeros(1, 2, 8), torch.zeros(1, 2, 4, 8),
                                             torch.zeros(1, 2, 4, 8))


def test_synth_is_deterministic_and_tie_rich(pn2):
    a, fa = pn2.synth.scannet_crop(7)
    b, fb = pn2.synth.scannet_crop(7)
    c, _ = pn2.synth.scannet_crop(8)
    assert np.array_equal(a, b) and np.array_equal(fa, fb) and not np.array_equal(a, c)
    assert a.shape == (8192, 3) and fa.shape == (8192, 6) and a.dtype == np.float32
    assert len(np.unique(a, axis=0)) < 8192  # drawn with replacement: duplicates present
    assert a.min() > -0.01 and a[:, :2].max() < 1.91 and a[:, 2].max() < 3.01
    np.testing.assert_allclose(np.linalg.norm(fa[:, 3:], axis=1), 1.0, rtol=1e-6)
    assert (fa[:, :3] >= 0).all() and (fa[:, :3] <= 1).all()
    u = pn2.synth.uniform_cloud(3, 1024)
    assert u.shape == (1024, 3) and (u >= 0).all() and (u < 1).all()
    s = pn2.synth.splitmix64(0x5EED, 4)  # SplitMix64 reference values for seed 0x5EED
    assert s.dtype == np.uint64 and len(set(s.tolist())) == 4


def test_step_bytes_match_survey(pn2):
    """Algorithmic bytes per cloud: cfg2 12,631,488; cfg3 13,614,528
    geometric + 32,440,320 attention; cfg5 42,730,496. fp_concat is extra work this step does
    (the FP concat of points1) and is accounted separately."""
    by = pn2.stack.sa_fp_bytes("cfg2", 1)
    assert sum(v for k, v in by.items() if k != "fp_concat") == 12_631_488
    by = pn2.stack.sa_fp_bytes("cfg3", 1)
    assert sum(v for k, v in by.items() if k not in ("fp_concat", "attention")) == 13_614_528
    assert by["attention"] == 32_440_320
    by = pn2.stack.sa_fp_bytes("cfg5", 1)
    assert sum(by.values()) == 42_730_496
    assert pn2.stack.sa_fp_bytes("cfg2", 16)["fps"] == 16 * pn2.stack.sa_fp_bytes("cfg2", 1)["fps"]


def test_shard_ids_partition_the_batch(pn2):
    world, per = 8, 16
    ids = [i for r in range(world) for i in pn2.shard.shard_ids(r, world, per)]
    assert ids == list(range(world * per))
    with pytest.raises(ValueError):
        pn2.shard.shard_ids(8, 8, 16)


def test_oracle_step_shapes(pn2, orc):
    """The CPU restatement of one cfg2 step (the bench's cpu_baseline) on one cloud."""
    inp = pn2.stack.make_inputs("cfg2", [0], "cpu")
    np_inp = dict(inp)
    np_inp["xyz"] = inp["xyz"].numpy()
    np_inp["sa_out"] = [t.numpy() for t in inp["sa_out"]]
    np_inp["fp_out"] = [t.numpy() for t in inp["fp_out"]]
    outs = orc.run_stack_cpu(np_inp, "cfg2")
    shapes = [o.shape for o in outs]
    assert shapes == [(1, 1024, 32, 3), (1, 256, 32, 67), (1, 64, 32, 131), (1, 16, 32, 259),
                      (1, 64, 768), (1, 256, 384), (1, 1024, 320), (1, 8192, 128)]
    assert all(np.isfinite(o).all() for o in outs)


def test_param_store_names_and_initialisers(pn2):
    """tf_util.ParamStore: the reference's TF variable names, its initialisers for misses
    (xavier weights, zero biases, BN gamma 1 / beta 0 / mean 0 / variance 1), checkpoint
    arrays accepted as numpy and reshaped from the TF [1,1,cin,cout] kernel layout."""
    import numpy as np
    st = pn2.tf_util.ParamStore({"l/conv0/weights": np.ones((1, 1, 3, 8), np.float32)}, seed=1)
    p = st.conv("l/conv0", 3, 8)
    assert tuple(p["weights"].shape) == (3, 8) and float(p["weights"].sum()) == 24.0
    q = st.conv("l/conv1", 8, 16)
    assert set(st) >= {"l/conv1/weights", "l/conv1/biases", "l/conv1/bn/gamma",
                       "l/conv1/bn/beta", "l/conv1/bn/moving_mean", "l/conv1/bn/moving_variance"}
    lim = np.sqrt(6.0 / (8 + 16))
    w = q["weights"].numpy()
    assert np.abs(w).max() <= lim and w.std() > 0
    assert float(q["biases"].abs().sum()) == 0 and float(q["gamma"].sum()) == 16
    assert np.array_equal(st.conv("l/conv1", 8, 16)["weights"].numpy(), w)  # cached
    d = st.dense("s/ScannetAttentionLayer/dense", 4, 4)
    assert tuple(d["weights"].shape) == (4, 4)
