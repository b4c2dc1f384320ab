#!/usr/bin/env python3
"""Generate the GPU golden vectors of tests/golden/ from the REFERENCE's own CUDA kernels.

The reference kernels (pointnet2_tensorflow/tf_ops/sampling/tf_sampling_g.cu:105-192 and
grouping/tf_grouping_g.cu:3-57) are compiled UNCHANGED for gfx950 into oracle/_ref/libref_gpu.so
(oracle/Makefile target `ref`, built in the container that has /root/reference; the .so then
travels to the GPU box with the repo snapshot). Run on the MI355X:
    python tests/golden/make_golden_gpu.py [out_dir] [--prob-only]   (default: tests/golden)
Nothing here reads /root/reference. Outputs:
    fps_*.npz   farthest_point_sample + gather_point of the reference kernels
    bqg_*.npz   query_ball_point of the reference kernel WITH its pts_cnt output
    prob_*.npz  prob_sample (cumsumKernel + binarysearchKernel, tf_sampling_g.cu:7-104)
Inputs are deterministic (synth.py SplitMix64 / fixed lattices). Cases follow SURVEY.md §8(c):
cfg1, one SA1 crop with duplicates, the N>3072 global-memory branch of the reference FPS
(tf_sampling_g.cu:133-141), N<512, N=1, npoint > #unique points, all-duplicate clouds and a
tie-heavy integer lattice.
"""
import importlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (before the HIP .so: one HIP runtime)

from oracle import oracle as O  # noqa: E402

pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
synth = pkg.synth
DEV = torch.device("cuda:0")
_ARGS = [a for a in sys.argv[1:] if not a.startswith("--")]
OUT = _ARGS[0] if _ARGS else HERE  # the GPU box merges back only gpurun_out/


def save(name, meta, **arrays):
    arrays["meta"] = np.array(json.dumps(meta))
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)
    print("wrote", name, {k: v.shape for k, v in arrays.items()}, flush=True)


def ref_fps(x, m):
    B, N = x.shape[:2]
    xt = torch.from_numpy(x).to(DEV)
    out = torch.zeros((B, m), dtype=torch.int32, device=DEV)
    assert O.ref_gpu().pn2ref_fps(xt.data_ptr(), B, N, m, out.data_ptr()) == 0
    new_xyz = torch.zeros((B, m, 3), dtype=torch.float32, device=DEV)
    assert O.ref_gpu().pn2ref_gather_point(xt.data_ptr(), out.data_ptr(), B, N, m,
                                           new_xyz.data_ptr()) == 0
    return out.cpu().numpy(), new_xyz.cpu().numpy()


def fps_case(name, x, m, src):
    x = np.ascontiguousarray(x, np.float32)
    idx, new_xyz = ref_fps(x, m)
    save(name, {"op": "farthest_point_sample", "npoint": m, "inputs": src,
                "ref": "tf_sampling_g.cu:105-181 (farthestpointsamplingKernel, gatherpointKernel) "
                       "compiled for gfx950, run on the MI355X"},
         xyz=x, idx=idx, new_xyz=new_xyz)


def bq_case(name, x, q, r, ns, src):
    B, N = x.shape[:2]
    M = q.shape[1]
    xt, qt = torch.from_numpy(x).to(DEV), torch.from_numpy(q).to(DEV)
    idx = torch.full((B, M, ns), -1, dtype=torch.int32, device=DEV)
    cnt = torch.full((B, M), -1, dtype=torch.int32, device=DEV)
    assert O.ref_gpu().pn2ref_query_ball_point(xt.data_ptr(), qt.data_ptr(), B, N, M, r, ns,
                                               idx.data_ptr(), cnt.data_ptr()) == 0
    save(name, {"op": "query_ball_point_gpu", "radius": r, "nsample": ns, "inputs": src,
                "ref": "tf_grouping_g.cu:3-36 (query_ball_point_gpu) compiled for gfx950",
                "note": "idx rows of queries with no hit stay -1 (the kernel leaves them "
                        "untouched); pts_cnt is written for every query"},
         xyz1=x, xyz2=q, idx=idx.cpu().numpy(), pts_cnt=cnt.cpu().numpy())


def sel_case(name, d, k, src):
    B, m, n = d.shape
    dt = torch.from_numpy(d).to(DEV)
    outi = torch.zeros((B, m, n), dtype=torch.int32, device=DEV)
    out = torch.zeros((B, m, n), dtype=torch.float32, device=DEV)
    assert O.ref_gpu().pn2ref_selection_sort(dt.data_ptr(), B, m, n, k, outi.data_ptr(),
                                             out.data_ptr()) == 0
    save(name, {"op": "selection_sort", "k": k, "inputs": src,
                "ref": "tf_grouping_g.cu:83-123 (selection_sort_gpu) compiled for gfx950"},
         dist=d, outi=outi.cpu().numpy(), out=out.cpu().numpy())


def prob_case(name, w, r, src):
    B, n = w.shape
    m = r.shape[1]
    wt, rt = torch.from_numpy(w).to(DEV), torch.from_numpy(r).to(DEV)
    out = torch.full((B, m), -1, dtype=torch.int32, device=DEV)
    assert O.ref_gpu().pn2ref_prob_sample(wt.data_ptr(), rt.data_ptr(), B, n, m,
                                          out.data_ptr()) == 0
    save(name, {"op": "prob_sample", "inputs": src,
                "ref": "tf_sampling_g.cu:7-104,197-201 (cumsumKernel, binarysearchKernel) "
                       "compiled for gfx950"},
         inp=w, inpr=r, out=out.cpu().numpy())


def prob_cases():
    rng = np.random.default_rng(13)
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    prob_case("prob_uniform", f32(rng.random((3, 1003))), f32(rng.random((3, 200))),
              "U[0,1) weights (3,1003): a partial last quad; 200 draws")
    prob_case("prob_chunks", f32(rng.random((2, 20001))), f32(rng.random((2, 300))),
              "U[0,1) weights (2,20001): 3 chunks of 8192, Kahan carry, partial quad")
    w = rng.exponential(1.0, (2, 8192)) ** 6  # wide dynamic range: rounding decides
    w[:, ::7] = 0.0
    r = rng.random((2, 256))
    r[:, :4] = [0.0, np.nextafter(np.float32(1), np.float32(0)), 0.5, 1e-7]
    prob_case("prob_skewed", f32(w), f32(r), "exp(1)^6 weights with zeros (2,8192); "
              "draws incl. 0, 1-ulp, 0.5, 1e-7")
    prob_case("prob_small", f32([[0.0, 0.0, 1.0, 0.0, 2.0], [1.0, 1.0, 1.0, 1.0, 1.0]]),
              f32(rng.random((2, 64))), "(2,5) with zero weights and ties")
    prob_case("prob_n1", f32([[3.0]]), f32([[0.0, 0.3, 0.99]]), "one category")


def main():
    if not O.have_ref_gpu():
        raise SystemExit("oracle/_ref/libref_gpu.so missing: build it with `make -C oracle ref`")
    prob_cases()
    if "--prob-only" in sys.argv:
        return
    fps_case("fps_uniform_cfg1", synth.batch([0], 1024, "uniform")[0], 256,
             "uniform U[0,1)^3 (1,1024) -> 256 (cfg1)")
    fps_case("fps_scannet_sa1", synth.batch([1], 8192, "scannet")[0], 1024,
             "ScanNet crop (1,8192) with duplicates -> 1024 (SSG SA1; global-memory branch)")
    fps_case("fps_scannet_msg", synth.batch([3], 16384, "scannet")[0], 512,
             "ScanNet crop (1,16384) -> 512 (MSG SA1)")
    fps_case("fps_scannet_sa2", synth.batch([4, 5], 1024, "scannet")[0], 256,
             "ScanNet crops (2,1024) -> 256 (SA2 sizes; LDS branch)")
    fps_case("fps_small_n", synth.batch([6], 300, "uniform")[0], 64, "uniform (1,300), N < 512")
    fps_case("fps_n1", np.array([[[0.3, 0.6, 0.9]]], np.float32), 4, "N = 1, npoint 4")
    rng = np.random.default_rng(7)
    uniq = rng.random((20, 3)).astype(np.float32)
    fps_case("fps_npoint_gt_unique", uniq[rng.integers(0, 20, 600)][None], 100,
             "600 draws of 20 unique points -> 100 (npoint > #unique)")
    fps_case("fps_all_dup", np.tile(np.float32([[0.25, 0.5, 0.75]]), (700, 1))[None], 40,
             "700 copies of one point -> 40")
    g = np.stack(np.meshgrid(*[np.arange(16)] * 3, indexing="ij"), -1).reshape(-1, 3)
    fps_case("fps_grid_ties", g[rng.integers(0, len(g), 4096)][None].astype(np.float32), 512,
             "16^3 integer lattice, 4096 draws -> 512 (massive exact ties)")
    x = synth.batch([8], 1024, "scannet")[0]
    bq_case("bqg_scannet_sa2", x, x[:, ::4].copy(), 0.2, 32, "ScanNet crop (1,1024), SA2 radius")
    x = synth.batch([9], 300, "uniform")[0]
    bq_case("bqg_uniform_sparse", x, x[:, ::6].copy(), 0.05, 8, "uniform (1,300), r=.05: cnt < ns")
    rng = np.random.default_rng(11)
    sel_case("sel_ties", rng.integers(0, 4, (2, 16, 96)).astype(np.float32), 24,
             "integer distances in [0,4): ties everywhere, k=24")
    x = synth.batch([10], 1024, "scannet")[0]
    q = x[:, ::32].copy()
    d = ((x[:, None, :, :] - q[:, :, None, :]) ** 2).sum(-1).astype(np.float32)
    sel_case("sel_scannet", d, 32, "squared distances of 32 queries to a (1,1024) ScanNet crop")


if __name__ == "__main__":
    main()
