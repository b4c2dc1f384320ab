"""bench.py's inputs that do not need a GPU: the committed PMC summary behind roofline.traffic,
the committed stamp summary behind roofline.latency, and the CPU baseline leg (a short
sample)."""
import importlib
import importlib.util
import os

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pmc_traffic_of_the_sa1_sampler(bench):
    traffic, src = bench.pmc_traffic("cfg2", 16)
    assert src and "pmc_traffic_cfg2_B16.json" in src
    # read the cloud once, write idx + new_xyz; the grid-building sampler (cfg2 since round 6)
    # also writes FP4's known grid
    grid = "fps_hotcull_grid_kernel" in src
    algorithmic = bench.sa1_algorithmic_bytes(16, 8192, 1024, grid)
    assert algorithmic == 16 * (8192 * 12 + 1024 * 16 + (32 + 1025 * 4 + 1024 * 16 if grid else 0))
    # WRITE_SIZE equals the outputs; FETCH_SIZE x2 (the gfx950 correction for 16 B per lane
    # reads) lands 26 % above the cloud bytes for the culled sampler (1.08x for v9), and the
    # grid build's read-back of the 12-byte picks counts double too
    assert 1.0 <= traffic / algorithmic <= 1.35, (traffic, algorithmic)


def test_latency_of_the_sa1_sampler(bench):
    v = bench.sa1_latency("cfg2", 0.47, 1024, 8192)
    assert abs(v["ns_per_pick"] - 0.47e6 / 1023) < 1e-6
    # the culled sampler's stamp summary: hot pick loop + per-round refreshes + setup
    assert v["rounds"] > 0 and v["hot_cycles_per_pick"] > 0 and v["source"].endswith(".json")
    # the latency floor (tools/ubench/pick_floor.hip): below the measured costs, and the
    # launch floor composes setup + (M - 1) picks + rounds
    assert 0 < v["floor_cycles_per_pick"] <= v["floor_pick_step_cycles"] <= v["hot_cycles_per_pick"]
    assert 0 < v["floor_round_cycles"] <= v["round_cycles"]
    want = v["floor_setup_cycles"] + 1023 * v["floor_cycles_per_pick"] + \
        v["rounds"] * v["floor_round_cycles"]
    assert abs(v["floor_launch_cycles"] - want) < 1e-6
    assert 0 < v["frac_pick"] <= 1 and 0 < v["frac_round"] <= 1
    m = bench.sa1_latency("cfg5", 0.36, 512, 16384)  # the MSG sampler: its own stamps
    assert m["source"].endswith("msg_cull_stamps.json") and m["rounds"] > 0
    assert 0 < m["frac_pick"] <= 1 and m["floor_launch_ms"] < 0.36


def test_cpu_baseline_leg(bench):
    r = bench.cpu_baseline("cfg2", 16, 0.2, 2)
    assert r["kind"] == "port" and r["cores"] == 2 and r["value"] > 0
    assert r["unit"] == "clouds/s"
    assert r["value_all_cores_at_measured_efficiency"] == pytest.approx(
        r["value_all_cores_extrapolated"] * r["scaling_efficiency_1_to_threads"])


@pytest.mark.parametrize("config", ["cfg2", "cfg3"])
def test_verify_checker_catches_a_wrong_step(bench, config):
    """bench.py's `verified` field: the checker passes the oracle's own outputs and fails a
    step whose one index, one copied float or one interpolated value is off."""
    import numpy as np
    import torch

    from oracle import oracle as O
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    inp = pkg.stack.make_inputs(config, [5], "cpu")
    np_inp = dict(inp, xyz=inp["xyz"].numpy(), feats=None if inp["feats"] is None else
                  inp["feats"].numpy(), sa_out=[t.numpy() for t in inp["sa_out"]],
                  fp_out=[t.numpy() for t in inp["fp_out"]])
    if "attn" in inp:
        np_inp["attn"] = [tuple(t.numpy() for t in q) for q in inp["attn"]]
    ref, _, inter = O.run_stack_cpu(np_inp, config, intermediates=True)
    T = lambda a: torch.tensor(a.numpy() if torch.is_tensor(a) else a)  # noqa: E731
    good = bench.verify_sets(config, [(inp, [T(r) for r in ref],
                                       {k: T(v) for k, v in inter.items()})], 2)
    assert good["failures"] == [] and good["clouds"] == 1
    bad_idx = {k: T(v) for k, v in inter.items()}
    bad_idx["bq2.idx"][0, 3, 5] += 1
    bad_copy = [T(r) for r in ref]
    bad_copy[0].view(-1)[17] = float(np.nextafter(np.float32(bad_copy[0].view(-1)[17]),
                                                   np.float32(9)))
    bad_fp = [T(r) for r in ref]
    bad_fp[-1][0, 0, 0] += 1e-3
    for outs, it, what in ((ref, bad_idx, "bq2.idx"), (bad_copy, inter, "sa1.new_points"),
                           (bad_fp, inter, "fp4.out")):
        r = bench.verify_sets(config, [(inp, [T(o) for o in outs],
                                        {k: T(v) for k, v in it.items()})], 2)
        assert r["failures"] and what in r["failures"][0], r["failures"]
