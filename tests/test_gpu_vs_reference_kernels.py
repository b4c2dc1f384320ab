"""The reference's own CUDA kernels (tf_sampling_g.cu, tf_grouping_g.cu), compiled unchanged for
gfx950 into oracle/_ref/libref_gpu.so, against this library at the cfg2 step's shapes
(B = 16 ScanNet crops of 8,192 points, SSG SA1..SA4) on the same MI355X.

Every op's output must be identical (indices, gathered / grouped floats bit for bit), and every
op of this library must be faster than the reference kernel it replaces. The timings (GPU
events around each call, median of 5) are printed and written to
gpurun_out/ref_kernels_cfg2.json when that directory exists (profiles/r1/ keeps a copy).
The reference shim synchronises after every launch and allocates FPS's workspace per call
(tf_sampling.cpp:114-118 does the same through TF's allocator); the events bracket only the
GPU work, so that host cost is not counted against the reference.

three_nn / three_interpolate have no reference GPU kernel (tf_interpolate.cpp is CPU-only),
so the FP side is not part of this comparison.
"""
import importlib
import json
import os

import numpy as np
import pytest

from conftest import PKG_NAME, ROOT, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


def _time(torch, fn, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))  # us


def test_cfg2_ops_vs_reference_kernels():
    import torch

    from oracle import oracle as O
    if not O.have_ref_gpu():
        pytest.skip("oracle/_ref/libref_gpu.so not built")
    R = O.ref_gpu()
    pkg = importlib.import_module(PKG_NAME)
    S, ts, tg = pkg.stack, pkg.tf_sampling, pkg.tf_grouping
    dev = torch.device("cuda:0")
    inp = S.make_inputs("cfg2", list(range(16)), dev)
    xyz = inp["xyz"].contiguous()
    B = xyz.shape[0]
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    rows = []

    def row(op, shape, ref_us, ours_us):
        rows.append({"op": op, "shape": shape, "reference_us": round(ref_us, 1),
                     "ours_us": round(ours_us, 1), "speedup": round(ref_us / ours_us, 2)})

    level = xyz
    c_in = 0
    for i, (M, r, ns, c_out) in enumerate(S.SSG_SA):
        N = level.shape[1]
        # FPS (tf_sampling_g.cu:105-170 vs pn2_fps)
        ref_idx = torch.zeros((B, M), dtype=torch.int32, device=dev)
        t_ref = _time(torch, lambda: R.pn2ref_fps(level.data_ptr(), B, N, M, ref_idx.data_ptr()))
        ours = {}
        t_ours = _time(torch, lambda: ours.update(idx=ts.farthest_point_sample(M, level)))
        assert torch.equal(ours["idx"], ref_idx), f"SA{i + 1} FPS differs from the reference"
        row(f"SA{i + 1} farthest_point_sample", [B, N, M], t_ref, t_ours)
        # gather_point (tf_sampling_g.cu:172-181)
        ref_new = torch.zeros((B, M, 3), device=dev)
        t_ref = _time(torch, lambda: R.pn2ref_gather_point(level.data_ptr(), ref_idx.data_ptr(),
                                                           B, N, M, ref_new.data_ptr()))
        t_ours = _time(torch, lambda: ours.update(new=ts.gather_point(level, ours["idx"])))
        assert torch.equal(ours["new"], ref_new)
        row(f"SA{i + 1} gather_point", [B, N, M], t_ref, t_ours)
        new_xyz = ref_new
        # query_ball_point (tf_grouping_g.cu:3-36)
        ref_bi = torch.zeros((B, M, ns), dtype=torch.int32, device=dev)
        ref_cnt = torch.zeros((B, M), dtype=torch.int32, device=dev)
        t_ref = _time(torch, lambda: R.pn2ref_query_ball_point(
            level.data_ptr(), new_xyz.data_ptr(), B, N, M, r, ns, ref_bi.data_ptr(),
            ref_cnt.data_ptr()))
        t_ours = _time(torch, lambda: ours.update(bq=tg.query_ball_point(r, ns, level, new_xyz)))
        got_idx, got_cnt = ours["bq"]
        # rows without any hit are left uninitialised by the reference
        hit = ref_cnt > 0
        assert torch.equal(got_cnt, ref_cnt)
        assert torch.equal(got_idx[hit], ref_bi[hit]), f"SA{i + 1} ball query differs"
        row(f"SA{i + 1} query_ball_point", [B, N, M, ns], t_ref, t_ours)
        # group_point of the layer's input features (tf_grouping_g.cu:38-57)
        C = max(3, c_in)
        pts = torch.rand((B, N, C), generator=gen, device=dev)
        ref_g = torch.zeros((B, M, ns, C), device=dev)
        t_ref = _time(torch, lambda: R.pn2ref_group_point(pts.data_ptr(), got_idx.data_ptr(), B,
                                                          N, C, M, ns, ref_g.data_ptr()))
        t_ours = _time(torch, lambda: ours.update(g=tg.group_point(pts, got_idx)))
        assert torch.equal(ours["g"], ref_g)
        row(f"SA{i + 1} group_point", [B, N, C, M, ns], t_ref, t_ours)
        level, c_in = new_xyz.contiguous(), c_out

    tot_ref = sum(r["reference_us"] for r in rows)
    tot_ours = sum(r["ours_us"] for r in rows)
    out = {"workload": "cfg2 SA1..SA4 ops, B=16 ScanNet crops of 8192 points, one op at a time "
                       "on an idle MI355X (GPU events, median of 5)",
           "reference": "tf_sampling_g.cu + tf_grouping_g.cu compiled unchanged for gfx950 "
                        "(oracle/Makefile target ref)",
           "ops": rows, "sum_reference_us": round(tot_ref, 1), "sum_ours_us": round(tot_ours, 1),
           "sum_speedup": round(tot_ref / tot_ours, 2)}
    print(json.dumps(out, indent=1))
    gout = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(gout):
        with open(os.path.join(gout, "ref_kernels_cfg2.json"), "w") as f:
            json.dump(out, f, indent=1)
    slower = [r for r in rows if r["ours_us"] > r["reference_us"]]
    assert not slower, f"slower than the reference kernel: {slower}"
