"""GPU parity of the scene-crop kernels (csrc/scene.hip), SURVEY.md §8(f)4.

- pn2_crop_sample (data_transformation.py:70-154, get_subset) against the numpy restatement
  oracle.crop_sample for the same random draws: every output BIT-EXACT (index work and copies;
  the sample weights are one fp32 product), and the per-try statistics (points in the area,
  labelled points, occupied voxel keys) equal.
- the whole-scene chunker (complete_scene_loader.py:4-131) against the reference function's
  own outputs (tests/golden/scene_chunks.json: SHA-256 per output, same np.random seed).
"""
import hashlib
import importlib
import json
import os

import numpy as np
import pytest

from conftest import PKG_NAME, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def env():
    import torch

    from oracle import oracle as O
    pkg = importlib.import_module(PKG_NAME)
    return pkg, O, torch, torch.device("cuda:0")


@pytest.mark.parametrize("scene_id,n", [(1, 20000), (4, 60000), (5, 3000)])
def test_scene_bbox(env, scene_id, n):
    pkg, O, torch, dev = env
    pts = pkg.synth.scannet_scene(scene_id, n)[0]
    got = pkg.data_transformation.scene_bbox(torch.from_numpy(pts).to(dev)).cpu().numpy()
    assert np.array_equal(got, np.concatenate([pts.min(0), pts.max(0)]))


@pytest.mark.parametrize("scene_id,n,B,K", [(1, 20000, 4, 8192), (4, 60000, 3, 8192),
                                            (5, 3000, 2, 1000), (6, 100000, 2, 4096)])
def test_crop_sample_vs_oracle(env, scene_id, n, B, K):
    pkg, O, torch, dev = env
    lib = pkg.lib()
    pts, lab, col, nrm = pkg.synth.scannet_scene(scene_id, n)
    g = np.random.default_rng(scene_id)
    T = 10
    centres = (g.uniform(0, 1, (B, T)).astype(np.float32) * np.float32(n)).astype(np.int32)
    u = g.uniform(0, 1, (B, K)).astype(np.float32)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    P, L, C, Nn = d(pts), d(lab), d(col), d(nrm)
    bbox = pkg.data_transformation.scene_bbox(P)
    ws = torch.zeros(int(lib.pn2_crop_workspace_size(B, n, T)) // 4 + 1, dtype=torch.int32,
                     device=dev)
    lw = d(np.asarray(O.GET_SUBSET_LABEL_WEIGHTS, np.float32))
    op = torch.empty((B, K, 3), dtype=torch.float32, device=dev)
    ol = torch.empty((B, K), dtype=torch.int32, device=dev)
    oc = torch.empty((B, K, 3), dtype=torch.int32, device=dev)
    on = torch.empty((B, K, 3), dtype=torch.float32, device=dev)
    ow = torch.empty((B, K), dtype=torch.float32, device=dev)
    dc, du = d(centres), d(u)
    rc = lib.pn2_crop_sample(P.data_ptr(), L.data_ptr(), C.data_ptr(), Nn.data_ptr(), n,
                             bbox.data_ptr(), dc.data_ptr(), B, T, du.data_ptr(), K,
                             lw.data_ptr(), lw.numel(), ws.data_ptr(), ws.numel() * 4,
                             op.data_ptr(), ol.data_ptr(), oc.data_ptr(), on.data_ptr(),
                             ow.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    for b in range(B):
        rp, rl, rcol, rn, rw, chosen, rstats = O.crop_sample(pts, lab, col, nrm, centres[b], u[b])
        assert chosen == T - 1  # the reference's 3n denominator: no try is ever valid
        assert np.array_equal(op[b].cpu().numpy(), rp)
        assert np.array_equal(ol[b].cpu().numpy(), rl)
        assert np.array_equal(oc[b].cpu().numpy(), rcol)
        assert np.array_equal(on[b].cpu().numpy(), rn)
        assert np.array_equal(ow[b].cpu().numpy(), rw)


def test_get_subset_mirror(env):
    """The Python mirror (reference signature) on top of the kernels."""
    pkg, O, torch, dev = env
    pts, lab, col, nrm = pkg.synth.scannet_scene(7, 25000)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    centres = np.arange(10, dtype=np.int32) * 997
    u = np.linspace(0, 0.999, 8192, dtype=np.float32)
    got = pkg.data_transformation.get_subset(d(pts), d(lab), d(col), d(nrm), 8192, centres, u)
    ref = O.crop_sample(pts, lab, col, nrm, centres, u)
    for a, b in zip(got, ref[:5]):
        assert np.array_equal(a.cpu().numpy(), b)
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    outs = pkg.data_transformation.get_subsets(d(pts), d(lab), None, None, 4, 2048, generator=gen)
    assert outs[0].shape == (4, 2048, 3) and outs[2] is None and outs[3] is None


def _digest(a):
    a = np.ascontiguousarray(a)
    return {"shape": list(a.shape), "dtype": str(a.dtype),
            "sha256": hashlib.sha256(a.tobytes()).hexdigest()}


def test_scene_chunker_vs_reference_golden(env):
    pkg, O, torch, dev = env
    csl = pkg.complete_scene_loader
    with open(os.path.join(HERE, "golden", "scene_chunks.json")) as f:
        cases = json.load(f)
    for case in cases:
        pts, lab, col, nrm = pkg.synth.scannet_scene(case["scene_id"], case["n_points"])
        np.random.seed(case["seed"])
        if case["variant"] == "test":
            res = csl.get_all_subsets_with_all_points_for_scene_numpy_test(pts, col, nrm)
            names = ["point_sets", "colors", "normals", "masks", "orig_idxs"]
        else:
            res = csl.get_all_subsets_with_all_points_for_scene_numpy(pts, lab, col, nrm)
            names = ["point_sets", "labels", "colors", "normals", "sample_weights", "masks",
                     "orig_idxs"]
        for name, arr in zip(names, res):
            assert _digest(arr) == case["outputs"][name], (case["scene_id"], name)
