"""bench.py's inputs that do not need a GPU: the committed PMC summary behind roofline.traffic,
the static SA1 loop count behind roofline.valu, and the CPU baseline leg (a short sample)."""
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
    algorithmic = 16 * (8192 * 12 + 1024 * 16)  # read the cloud once, write idx + new_xyz
    assert 1.0 <= traffic / algorithmic <= 1.2, (traffic, algorithmic)


def test_valu_bound_of_the_sa1_sampler(bench):
    v = bench.sa1_valu_bound("cfg2", 702.0)
    assert v["floor_cycles_per_iteration"] == 4 * v["valu_instr_per_iteration"]
    assert 0.3 < v["frac"] < 1.0
    assert bench.sa1_valu_bound("cfg5", 1300.0) is None  # a different sampler instantiation


def test_cpu_baseline_leg(bench):
    r = bench.cpu_baseline("cfg2", 16, 0.2, 2)
    assert r["kind"] == "port" and r["cores"] == 2 and r["value"] > 0
    assert r["unit"] == "clouds/s"
