"""CPU: the C-ABI library builds, loads and exports every entry point include/*.h declares
(pn2hip.h: the reference ops; pn2plan.h: the native step executor).
No kernel is launched here (no GPU in the build container): only host functions and argument
checks that return before any HIP call."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("pn2hip.h", "pn2plan.h")]


def header_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(pn2(?:cpu)?_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_headers_are_all_listed():
    assert sorted(os.listdir(os.path.join(ROOT, "include"))) == sorted(os.path.basename(h) for h in HEADERS)


def test_header_declares_the_boundary():
    names = header_functions()
    for need in ("pn2_fps", "pn2_gather_point", "pn2_ball_query", "pn2_group_point",
                 "pn2_three_nn", "pn2_three_interpolate", "pn2_attn_reduce", "pn2_fp_fused",
                 "pn2_sample_and_group", "pn2_group_pool"):
        assert need in names


def test_library_exports_every_declared_symbol(pn2):
    lib = pn2.lib()
    so = pn2.LIB_PATH
    exported = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True,
                              check=True).stdout
    for name in header_functions():
        assert re.search(rf"\bT {name}$", exported, re.M), f"{name} not exported by {so}"
        assert getattr(lib, name) is not None


def test_ctypes_signatures_match_header(pn2):
    from importlib import import_module
    _lib = import_module("pointcloud-segmentation-attention_amd._lib")
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_library_is_gfx950_code_object(pn2):
    """The fat binary embedded in libpn2hip.so carries gfx950 code objects (and nothing else)."""
    data = open(pn2.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"amdgcn-amd-amdhsa--gfx942" not in data


def test_version_and_errors(pn2):
    lib = pn2.lib()
    assert b"gfx950" in lib.pn2_version()
    assert b"invalid" in lib.pn2_strerror(-22)
    assert lib.pn2_strerror(0) == b"ok"


def test_argument_checks_return_einval_without_launching(pn2):
    lib = pn2.lib()
    E = -22
    assert lib.pn2_fps(None, 1, 100, 0, None, None) == E          # npoint <= 0 (tf_sampling.cpp:99)
    assert lib.pn2_fps(None, -1, 100, 4, None, None) == E
    assert lib.pn2_fps(None, 2, 100, 4, None, None) == E          # null buffers
    assert lib.pn2_ball_query(None, None, 1, 10, 10, 0.0, 8, None, None, None) == E  # radius
    assert lib.pn2_ball_query(None, None, 1, 10, 10, 0.1, 0, None, None, None) == E  # nsample
    assert lib.pn2_attn_reduce(None, None, None, 1, 1, 32, 6, None, None) == E  # C % 4
    assert lib.pn2_attn_reduce_grad(None, None, None, None, 1, 1, 32, 8, None, None, None,
                                    None) == E  # null buffers
    assert lib.pn2_group_pool(None, None, 1, 1, 4, 8, 7, None, None) == E       # mode
    assert lib.pn2_fp_fused(None, None, None, 3, None, 4, 1, 4, 4, None, None) == E  # C1 w/o points1
    assert lib.pn2_prob_sample(None, None, 1, 0, 4, None, 0, None, None) == E  # n = 0
    assert lib.pn2_prob_sample(None, None, 2, 10, 4, None, 0, None, None) == E  # workspace
    assert lib.pn2_prob_sample_workspace_size(3, 100) == 1200
    # empty work is a no-op, not an error (nothing is launched)
    assert lib.pn2_prob_sample(None, None, 2, 10, 0, None, 0, None, None) == 0
    assert lib.pn2_gather_point(None, None, 0, 10, 10, None, None) == 0
    assert lib.pn2_three_nn(None, None, 0, 10, 10, None, None, None) == 0


def test_grid_contract(pn2):
    lib = pn2.lib()
    E = -22
    per = lib.pn2_grid_size(1, 0)
    assert per > 0 and per % 16 == 0
    assert lib.pn2_grid_size(3, 1000) == 3 * (per + 1000 * 16)
    assert lib.pn2_grid_build(None, 1, 100, 0.1, None, 0, None) == E           # no buffer
    assert lib.pn2_grid_build(None, 1, 100, float("nan"), None, 0, None) == E  # NaN edge
    assert lib.pn2_grid_build(None, 0, 100, 0.1, None, 0, None) == 0           # empty batch
    assert lib.pn2_ball_query_grid(None, None, 1, 10, 10, 0.1, 0, None, None, None) == E
    assert lib.pn2_ball_query_grid(None, None, 1, 200000, 10, 0.1, 8, None, None, None) == E
    assert lib.pn2_three_nn_grid(None, None, None, 1, 10, 10, None, None, None) == E
    # several radii in one launch: 1 <= nr <= 3, every array given
    import ctypes
    rad = (ctypes.c_float * 4)(0.1, 0.2, 0.4, 0.8)
    nsa = (ctypes.c_int * 4)(8, 8, 8, 8)
    ptrs = (ctypes.c_void_p * 4)()
    assert lib.pn2_ball_group_xyz_grid_radii(None, None, None, 1, 10, 10, 0, rad, nsa, ptrs, ptrs, ptrs, None) == E
    assert lib.pn2_ball_group_xyz_grid_radii(None, None, None, 1, 10, 10, 4, rad, nsa, ptrs, ptrs, ptrs, None) == E
    assert lib.pn2_ball_group_xyz_grid_radii(None, None, None, 1, 10, 10, 2, None, nsa, ptrs, ptrs, ptrs, None) == E
    assert lib.pn2_ball_group_xyz_grid_radii(None, None, None, 1, 10, 10, 2, rad, nsa, ptrs, ptrs, ptrs, None) == E
    assert lib.pn2_ball_group_xyz_grid_radii(None, None, None, 0, 10, 10, 2, rad, nsa, ptrs, ptrs, ptrs, None) == 0
    # the bitmasks' LDS bound (nr * ceil(N / 32) <= 4096) is checked before any launch
    fake = (ctypes.c_void_p * 4)(16, 16, 16, 16)
    assert lib.pn2_ball_group_xyz_grid_radii(16, 16, 16, 1, 50000, 10, 3, rad, nsa, fake, fake, fake, None) == E
    assert lib.pn2_three_nn_grid(None, None, None, 0, 10, 10, None, None, None) == 0
    assert lib.pn2_fp_apply(None, None, None, None, 3, None, 4, 1, 4, 4, None, None) == E
    # pn2_fp_grid_fused: m in [1, 4096], dist and idx together, points1 with C1 > 0
    assert lib.pn2_fp_grid_fused(None, None, None, None, 0, None, 4, 1, 10, 0, None, None, None, None) == E
    assert lib.pn2_fp_grid_fused(None, None, None, None, 0, None, 4, 1, 10, 4097, None, None, None, None) == E
    assert lib.pn2_fp_grid_fused(None, None, None, None, 3, None, 4, 1, 10, 10, None, None, None, None) == E
    assert lib.pn2_fp_grid_fused(None, None, None, None, 0, None, 4, 1, 10, 10, None, 1, None, None) == E
    assert lib.pn2_fp_grid_fused(None, None, None, None, 0, None, 4, 1, 10, 10, None, None, None, None) == E
    assert lib.pn2_fp_grid_fused(None, None, None, None, 0, None, 4, 0, 10, 10, None, None, None, None) == 0
    # pn2_fp_grid_fused_known: a known grid is required (16-byte aligned), then the same checks
    assert lib.pn2_fp_grid_fused_known(None, None, None, None, None, 0, None, 4, 0, 10, 10, None, None, None, None) == E
    assert lib.pn2_fp_grid_fused_known(8, None, None, None, None, 0, None, 4, 0, 10, 10, None, None, None, None) == E
    assert lib.pn2_fp_grid_fused_known(16, None, None, None, None, 0, None, 4, 1, 10, 4097, None, None, None, None) == E
    assert lib.pn2_fp_grid_fused_known(16, None, None, None, None, 0, None, 4, 1, 10, 10, None, None, None, None) == E
    assert lib.pn2_fp_grid_fused_known(16, None, None, None, None, 0, None, 4, 0, 10, 10, None, None, None, None) == 0
    # pn2_fps_chain_grid: grid0 required, sized for stage 0 and aligned (checked before any launch)
    npt = (ctypes.c_int * 1)(256)
    bufs1 = (ctypes.c_void_p * 1)(16)
    assert lib.pn2_fps_chain_grid(8, 2, 4096, 1, ctypes.addressof(npt), ctypes.addressof(bufs1),
                                  ctypes.addressof(bufs1), None, 0, None) == E
    assert lib.pn2_fps_chain_grid(8, 2, 4096, 1, ctypes.addressof(npt), ctypes.addressof(bufs1),
                                  ctypes.addressof(bufs1), 4096, lib.pn2_grid_size(2, 256) - 1,
                                  None) == E


def test_fps_workspace_contract(pn2):
    lib = pn2.lib()
    cap = lib.pn2_fps_max_points()
    assert cap >= 16384
    assert lib.pn2_fps_workspace_size(16, 8192) == 0
    assert lib.pn2_fps_workspace_size(2, cap + 1) == 2 * (cap + 1) * 4


@pytest.mark.parametrize("r", [0.1, 0.2, 0.4, 0.8, 0.3, 1.0, 1e-3, 7.5, 1e-19])
def test_ball_threshold_equals_sqrt_predicate(pn2, r):
    """d2 < T  <=>  max(sqrtf(d2), 1e-20f) < r  (tf_grouping_g.cu:24-25), checked on the fp32
    neighbourhood of T with numpy's correctly rounded float32 sqrt."""
    lib = pn2.lib()
    r32 = np.float32(r)
    T = np.float32(lib.pn2_ball_threshold(float(r32)))
    bits = T.view(np.int32)
    cand = np.arange(max(int(bits) - 64, 0), int(bits) + 64, dtype=np.int32).view(np.float32)
    s = np.maximum(np.sqrt(cand), np.float32(1e-20))
    assert np.array_equal(cand < T, s < r32)
    assert lib.pn2_ball_threshold(0.0) == 0.0


def test_sa1_loop_isa_matches_built_library():
    """profiles/r1/sa1_loop_isa.json (the VALU count behind bench.py's roofline.valu) describes
    the SA1 sampler loop of the library as built."""
    import json
    import sys
    import tempfile
    if not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("llvm-objdump not available")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import place_sa1_loop
    with tempfile.TemporaryDirectory() as t:
        _, body = place_sa1_loop.loop_body(
            os.path.join(ROOT, "pointcloud-segmentation-attention_amd", "libpn2hip.so"), t)
    valu = sum(1 for ln in body if ln.split()[0].startswith("v_"))
    with open(os.path.join(ROOT, "profiles", "r1", "sa1_loop_isa.json")) as f:
        assert json.load(f)["mix"]["valu"] == valu


def test_sa1_sampler_loop_placement():
    """The SA1 sampler's iteration loop sits at a code offset = 4 mod 8 in the built library
    (the placement measured ~6 % faster than 0 mod 8; tools/place_sa1_loop.py chooses it)."""
    import sys
    import tempfile
    if not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("llvm-objdump not available")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import place_sa1_loop
    with tempfile.TemporaryDirectory() as t:
        off = place_sa1_loop.loop_offset(
            os.path.join(ROOT, "pointcloud-segmentation-attention_amd", "libpn2hip.so"), t)
    assert off % 8 == 4, off


def test_mlp_contract(pn2):
    """Shared-MLP entry points: packed size, and shape / chain checks that return EINVAL
    before any launch (no GPU needed)."""
    from importlib import import_module
    _lib = import_module(pn2.__name__ + "._lib")
    lib, E = pn2.lib(), -22
    # [cout32][cin8][64] float4 + scale + shift
    assert lib.pn2_mlp_packed_size(3, 32) == (1 * 1 * 256 + 2 * 32) * 4
    assert lib.pn2_mlp_packed_size(259, 512) == (16 * 33 * 256 + 2 * 512) * 4
    assert lib.pn2_mlp_packed_size(0, 32) == 0
    assert lib.pn2_mlp_pack(None, None, None, None, 3, 32, None, 0, None) == E
    L = _lib.MlpLayer
    fake = 1 << 20  # 16-byte aligned, never dereferenced by the checks
    good = (L * 2)(L(fake, 9, 32, 1), L(fake, 32, 64, 1))
    bad_chain = (L * 2)(L(fake, 9, 32, 1), L(fake, 16, 64, 1))
    misaligned = (L * 1)(L(fake + 4, 9, 32, 1))
    assert lib.pn2_shared_mlp(fake, 10, 9, 0, good, fake, None) == E        # no layers
    assert lib.pn2_shared_mlp(fake, 10, 9, 7, good, fake, None) == E        # > max layers
    assert lib.pn2_shared_mlp(fake, 10, 9, 2, bad_chain, fake, None) == E   # cin != prev cout
    assert lib.pn2_shared_mlp(fake, 10, 8, 2, good, fake, None) == E        # cin != input width
    assert lib.pn2_shared_mlp(fake, 10, 9, 1, misaligned, fake, None) == E
    assert lib.pn2_shared_mlp(None, 0, 9, 2, good, None, None) == 0         # no rows
    # group source: width = C + 3 with use_xyz; pool mode range
    assert lib.pn2_group_mlp(fake, fake, fake, fake, 1, 10, 6, 4, 8, 1, 2, good, 4, fake,
                             None) == E
    assert lib.pn2_group_mlp(fake, fake, fake, fake, 1, 10, 7, 4, 8, 1, 2, good, 0, fake,
                             None) == E
    assert lib.pn2_group_mlp(fake, fake, fake, fake, 1, 10, 6, 4, 0, 1, 2, good, 0, fake,
                             None) == E                                       # nsample 0
    assert lib.pn2_group_mlp(None, fake, None, None, 0, 10, 6, 4, 8, 1, 2, good, 0, None,
                             None) == 0                                       # empty batch
    assert lib.pn2_group_mlp(None, None, None, None, 0, 10, 6, 4, 8, 1, 2, good, 0, None,
                             None) == E                     # points NULL: the width is 3
    assert lib.pn2_fp_mlp(fake, fake, None, 3, fake, 6, 1, 4, 4, 2, good, fake, None) == E


def test_scene_contract(pn2):
    lib, E = pn2.lib(), -22
    fake = 1 << 20
    assert lib.pn2_scene_bbox(None, 0, None, None, 0, None) == E
    assert lib.pn2_scene_bbox(fake, 10, fake, fake, 0, None) == E           # workspace too small
    assert lib.pn2_crop_sample(fake, fake, None, None, 100, fake, fake, 2, 0, fake, 16, None, 0,
                               fake, 1 << 30, fake, fake, None, None, fake, None) == E  # T = 0
    assert lib.pn2_crop_sample(None, None, None, None, 100, None, None, 0, 10, None, 16, None, 0,
                               None, 0, None, None, None, None, None, None) == 0     # no crops
    assert lib.pn2_crop_sample(fake, fake, fake, None, 100, fake, fake, 2, 10, fake, 16, None, 0,
                               fake, 1 << 30, fake, fake, None, None, fake, None) == E  # colors w/o out
    assert lib.pn2_subvolume_select(None, 0, None, 4, 0.2, None, None, None, None) == 0
    assert lib.pn2_subvolume_select(None, 10, None, 4, 0.2, None, None, None, None) == E
    assert lib.pn2_subvolume_slices(4096) == 1 and lib.pn2_subvolume_slices(4097) == 2
    assert lib.pn2_gather_rows(fake, 10, 6, fake, 4, fake, None) == E        # row bytes % 4
    assert lib.pn2_gather_rows(None, 10, 8, None, 0, None, None) == 0


def test_plan_records_and_checks_without_launching(pn2):
    """include/pn2plan.h: operations are validated when recorded; an empty plan launches as a
    no-op (no HIP call)."""
    lib = pn2.lib()
    E = -22
    p = lib.pn2_plan_create()
    assert p
    try:
        assert lib.pn2_plan_size(p) == 0
        assert lib.pn2_plan_mark_timed(p) == E            # nothing to mark
        assert lib.pn2_plan_launch(p) == 0                 # empty: nothing enqueued
        assert lib.pn2_plan_launch_timed(p, None, None) == 0
        assert lib.pn2_plan_graph(p, None, None) == E      # null graph exec
        assert lib.pn2_plan_record(p, None, None) == E     # null event
        assert lib.pn2_plan_wait(p, None, None) == E
        npoint = (ctypes.c_int * 2)(256, 64)
        bufs = (ctypes.c_void_p * 2)(16, 32)
        # the pn2_fps_chain checks: a fed stage above 1024 points, too many stages, null xyz
        big = (ctypes.c_int * 2)(2048, 64)
        assert lib.pn2_plan_fps_chain(p, 8, 2, 4096, 2, ctypes.addressof(big), ctypes.addressof(bufs),
                                      ctypes.addressof(bufs), None) == E
        assert lib.pn2_plan_fps_chain(p, 8, 2, 4096, 5, ctypes.addressof(npoint), ctypes.addressof(bufs),
                                      ctypes.addressof(bufs), None) == E
        assert lib.pn2_plan_fps_chain(p, None, 2, 4096, 2, ctypes.addressof(npoint),
                                      ctypes.addressof(bufs), ctypes.addressof(bufs), None) == E
        # pn2_plan_fps_chain_grid: grid0 smaller than pn2_grid_size(B, npoint[0]) or not
        # 16-byte aligned
        need = lib.pn2_grid_size(2, 256)
        for g, nb in ((4096, need - 1), (4104, need)):
            assert lib.pn2_plan_fps_chain_grid(p, 8, 2, 4096, 2, ctypes.addressof(npoint),
                                               ctypes.addressof(bufs), ctypes.addressof(bufs),
                                               g, nb, None) == E
        assert lib.pn2_plan_size(p) == 0                   # nothing appended on error
        assert lib.pn2_plan_fps_chain(p, 8, 2, 4096, 2, ctypes.addressof(npoint),
                                      ctypes.addressof(bufs), ctypes.addressof(bufs), None) == 0
        assert lib.pn2_plan_size(p) == 1
        assert lib.pn2_plan_fps_chain_grid(p, 8, 2, 4096, 2, ctypes.addressof(npoint),
                                           ctypes.addressof(bufs), ctypes.addressof(bufs),
                                           4096, need, None) == 0
        assert lib.pn2_plan_size(p) == 2
        assert lib.pn2_plan_mark_timed(p) == 0
    finally:
        lib.pn2_plan_destroy(p)
    assert lib.pn2_plan_size(None) == E
    assert lib.pn2_plan_launch(None) == E
