"""GPU parity at the BASELINE.json batch sizes, collected FIRST among the GPU tests (the file
name sorts before every other test_gpu_*), so that a `-x` stop elsewhere cannot hide them.

What bench.py times -- the cfg2 / cfg3 / cfg5 steps at B = 16 / 16 / 8, eagerly and as the
software-pipelined hipGraph replay, and cfg4's per-rank shards -- checked output by output
against the CPU oracle with the bar north_star sets, per output:
  * bit-exact (np.array_equal on the bit patterns): every index and every copy -- the samplers'
    idx and new_xyz (tf_sampling_g.cu:105-181), the ball-query idx (tf_grouping_g.cu:3-36),
    the grouped [xyz - new_xyz, points] / MSG [points, xyz] (tf_grouping_g.cu:40-57,
    pointnet_util.py:40,52,191), the three_nn idx and dist (tf_interpolate.cpp:60-103), and
    the copied points1 columns of each FP output (pointnet_util.py:226);
  * rtol = atol = 1e-5: the interpolated FP columns (IDW weights + three_interpolate,
    pointnet_util.py:218-223, tf_interpolate.cpp:107-127) and the attention reduction
    (attention_layer.py:29-45).
Then every SA1-size sampler schedule on tie-heavy clouds, and the golden vectors the
reference's own FPS kernel produced (fps_*.npz by the kernel on the GPU, fpsemul_*.npz by the
kernel text on 512 CPU threads).
"""
import glob
import importlib
import json
import os

import numpy as np
import pytest

from conftest import PKG_NAME, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

TOL = dict(rtol=1e-5, atol=1e-5)
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def env():
    import torch

    from oracle import oracle as O
    O.set_threads(16)
    pkg = importlib.import_module(PKG_NAME)
    return pkg, O, torch, torch.device("cuda:0")


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def _exact(name, got, want):
    assert got.shape == want.shape, (name, got.shape, want.shape)
    if got.dtype == np.int32 or want.dtype == np.int32:
        bad = got != want
    else:
        bad = _bits(got) != _bits(want)
    assert not bad.any(), f"{name}: {int(bad.sum())} of {bad.size} values differ (bit-exact bar)"


def _close(name, got, want):
    assert got.shape == want.shape, (name, got.shape, want.shape)
    np.testing.assert_allclose(got, want, err_msg=f"{name} (1e-5 bar)", **TOL)


def _np_inputs(inp):
    np_inp = {k: v for k, v in inp.items()}
    for k in ("xyz", "feats"):
        np_inp[k] = None if inp[k] is None else inp[k].cpu().numpy()
    for k in ("sa_out", "fp_out"):
        if k in inp:
            np_inp[k] = [t.cpu().numpy() for t in inp[k]]
    if "attn" in inp:
        np_inp["attn"] = [tuple(t.cpu().numpy() for t in qkv) for qkv in inp["attn"]]
    return np_inp


def check_step(O, config, inp, outs, inter):
    """Every output and intermediate of one step against the oracle, each with its own bar.
    Returns the oracle's outputs."""
    ref, labels, rinter = O.run_stack_cpu(_np_inputs(inp), config, intermediates=True)
    assert len(outs) == len(ref) == len(labels)
    for g, r, (name, how) in zip(outs, ref, labels):
        g = g.cpu().numpy()
        if how is None:
            _exact(name, g, r)
        elif how == "tol":
            _close(name, g, r)
        else:  # FP output: [interpolated (C2 columns), points1 copy]
            _close(name + "[:C2] interpolated", g[..., :how], r[..., :how])
            _exact(name + "[C2:] points1 copy", g[..., how:], r[..., how:])
    # the step's index results: samplers, ball queries, and the FP searches that ran as their
    # own kernel (the others are checked through their FP outputs and test_step_three_nn)
    assert inter, "the step recorded no intermediates"
    for name, t in inter.items():
        _exact(name, t.cpu().numpy(), rinter[name])
    for name in rinter:
        if name.startswith(("fps", "bq")):
            assert name in inter, f"{name} missing from the step's intermediates"
    return ref


CONFIGS = [("cfg2", 16), ("cfg3", 16), ("cfg5", 8)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("config,B", CONFIGS)
def test_stack_full_size(env, config, B):
    """The benchmark step at its BASELINE.json batch (cfg2/cfg3 B = 16, cfg5 B = 8: the launch
    geometry of ball query and grouping depends on it), eagerly on the overlapped streams."""
    pkg, O, torch, dev = env
    inp = pkg.stack.make_inputs(config, list(range(B)), dev)
    step = pkg.stack.Step(inp)
    outs = step()
    torch.cuda.synchronize()
    check_step(O, config, inp, outs, step.intermediates())


def _poison_sampled(pipe, torch):
    """Overwrite every set's sampled coordinates (the buffers the side lanes read) with 1e6:
    a consumer that does not wait for its sampler then groups / interpolates against these
    (in bounds: no neighbour within any radius, huge but finite distances) and the step's
    outputs differ from the oracle's."""
    for s in pipe.sets:
        v = s.step.v
        for _, nx in (v.get("chain") or v.get("fps_out")):
            nx.fill_(1e6)
    torch.cuda.synchronize()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("lanes,native,layout,own,direct", [
    (1, False, "a", False, True), (1, True, "a", False, True),
    (2, True, "a", False, True), (3, True, "b", False, True),
    (3, True, "b", True, True), (3, True, "b", True, False)])
@pytest.mark.parametrize("config,B", CONFIGS)
def test_pipeline_full_size(env, config, B, lanes, native, layout, own, direct):
    """What bench.py times: the software-pipelined hipGraph steps over 3 buffer sets, at the
    BASELINE batch, after several rotations, with one, two or three sampler streams
    (consecutive steps' samplers concurrent), enqueued by the Python task loop or by the native
    plan (include/pn2plan.h) -- its side segments' kernels launched directly
    (pn2_plan_graph_direct) or as graph launches (direct=False) -- side layouts a and b
    (stack.side_layout), the later samplers behind SA1 or on a stream of their own (chain_own).
    The sampled coordinates of every set are poisoned before the last three steps (a missing
    wait then shows), and the last two steps' outputs (one per sampler stream) are compared
    with the oracle."""
    pkg, O, torch, dev = env
    # every set its own clouds (as bench.py runs it): a set that read another set's buffers
    # would give outputs that match no oracle run
    sets = [pkg.stack.make_inputs(config, list(range(100 + i * B, 100 + (i + 1) * B)), dev)
            for i in range(3)]
    inp = sets[0]
    pipe = pkg.stack.Pipeline(inp, graphs=True, nsets=3, sampler_lanes=lanes,
                              native_plan=native, layout=layout, chain_own=own,
                              set_inputs=sets, direct=direct)
    assert len(pipe.lane0) == lanes
    assert pipe.native_plan == native
    if native:  # every (set, sampler stream) plan exists before the first step
        assert all(getattr(s, "plans", None) for s in pipe.sets), "plans not built up front"
        for s in pipe.sets:  # every side segment is a plain kernel chain: all go in directly
            for p in s.plans.values():
                want = "direct" if direct else "graph"
                assert p.launches[want] > 0 and sum(p.launches.values()) == p.launches[want], \
                    p.launches
    for _ in range(7):
        pipe.run()
    pipe.join()
    _poison_sampled(pipe, torch)
    for _ in range(3):
        pipe.run()
    outs = pipe.join()
    assert pipe.check_faults() == 0
    for back in (1, 2):
        s = pipe.sets[(pipe.k - back) % len(pipe.sets)]
        check_step(O, config, sets[(pipe.k - back) % 3], s.outs if back > 1 else outs,
                   s.intermediates())
    # the checker bench.py's `verified` field runs, over every set
    runs = pipe.outputs_by_set()
    assert len(runs) == 3
    for sinp, souts, sinter in runs:
        bad = O.compare_stack(_np_inputs(sinp), config, [o.cpu().numpy() for o in souts],
                              {k: v.cpu().numpy() for k, v in sinter.items()})
        assert not bad, bad


@pytest.mark.timeout(300)
def test_pipeline_rotations_equal_eager(env):
    """Concurrency: the cfg2 pipeline (3 sampler streams, layout b, native plan, direct
    launches) for 12 rotations over 3 sets of distinct clouds, the sampled coordinates poisoned
    before every other rotation; every set's outputs and index intermediates after every
    rotation equal the same clouds' eager step bit for bit. (A race inside the sampler chain's
    publishing -- a 16-byte centre write -- showed here once in ~40 rotations:
    profiles/r5/chain_hot/tools.jsonl, pipe_stress_b128_publish.json; tools/pipe_stress.py
    runs longer.)"""
    pkg, O, torch, dev = env
    S = pkg.stack
    B = 16
    sets = [S.make_inputs("cfg2", list(range(100 + i * B, 100 + (i + 1) * B)), dev)
            for i in range(3)]
    refs = []
    for inp in sets:
        st = S.Step(inp)
        outs = st()
        torch.cuda.synchronize()
        refs.append(([o.clone() for o in outs], {k: v.clone() for k, v in st.intermediates().items()}))
    pipe = S.Pipeline(sets[0], graphs=True, nsets=3, sampler_lanes=3, native_plan=True,
                      layout="b", chain_own=False, set_inputs=sets, direct=True)
    for rot in range(12):
        if rot % 2 == 1:
            _poison_sampled(pipe, torch)
        for _ in range(3):
            pipe.run()
        pipe.join()
        for si, (_, souts, sinter) in enumerate(pipe.outputs_by_set()):
            ro, ri = refs[si]
            for i, (g, r) in enumerate(zip(souts, ro)):
                assert torch.equal(g, r) or torch.equal(g.view(torch.int32), r.view(torch.int32)), \
                    (rot, si, i)
            for name, t in sinter.items():
                assert torch.equal(t, ri[name]), (rot, si, name)
    assert pipe.check_faults() == 0


@pytest.mark.timeout(300)
@pytest.mark.parametrize("rank", [1, 7])
def test_cfg4_rank_shard(env, rank):
    """cfg4 (B = 128 over 8 GPUs, 16 per rank): the shard a rank owns (global cloud ids from
    shard.shard_ids, 16-31 for rank 1, 112-127 for rank 7) run on this GPU; outputs and the
    per-cloud checksums that bench.py gathers equal the oracle's for the same global clouds."""
    pkg, O, torch, dev = env
    ids = pkg.shard.shard_ids(rank, 8, 16)
    assert ids == list(range(16 * rank, 16 * rank + 16))
    inp = pkg.stack.make_inputs("cfg2", ids, dev)
    step = pkg.stack.Step(inp)
    outs = step()
    torch.cuda.synchronize()
    ref = check_step(O, "cfg2", inp, outs, step.intermediates())
    got = pkg.shard.cloud_checksums([o.cpu() for o in outs], 16)
    want = pkg.shard.cloud_checksums([torch.from_numpy(r) for r in ref], 16)
    np.testing.assert_allclose(got.numpy(), want.numpy(), rtol=1e-6, atol=1e-3)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("config", ["cfg2", "cfg3"])
def test_step_three_nn(env, config):
    """three_nn of every FP level of the step, at the full batch, through the same search the
    step uses (the grid search over the known points, ordered by the SA1 ball-query grid for
    FP4): idx and dist bit-exact (tf_interpolate.cpp:60-103)."""
    pkg, O, torch, dev = env
    inp = pkg.stack.make_inputs(config, list(range(16)), dev)
    step = pkg.stack.Step(inp)
    step()
    torch.cuda.synchronize()
    levels = step.v["xyz"]
    grid1 = step.v.get("grid1")
    for k in range(4):
        lvl = 3 - k
        x1, x2 = levels[lvl], levels[lvl + 1]
        d, i = pkg.tf_interpolate.three_nn(x1, x2, unknown_grid=grid1 if lvl == 0 else None)
        rd, ri = O.three_nn(x1.cpu().numpy(), x2.cpu().numpy())
        _exact(f"nn{k + 1}.idx", i.cpu().numpy(), ri)
        _exact(f"nn{k + 1}.dist", d.cpu().numpy(), rd)


def _cloud(pkg, kind, B, N, seed=0):
    if kind in ("scannet", "uniform"):
        return pkg.synth.batch(range(seed, seed + B), N, kind)[0]
    if kind == "dup":  # every point the same: all distances tie
        return np.tile(np.array([[0.25, 0.5, 0.75]], np.float32), (B, N, 1)).reshape(B, N, 3)
    if kind == "grid":  # integer lattice: massive exact ties
        g = np.stack(np.meshgrid(*[np.arange(16)] * 3, indexing="ij"), -1).reshape(-1, 3)
        rng = np.random.default_rng(seed)
        return np.stack([g[rng.integers(0, len(g), N)] for _ in range(B)]).astype(np.float32)
    if kind == "fewuniq":  # 300 distinct points drawn with replacement: npoint > #unique
        rng = np.random.default_rng(seed)
        u = rng.random((300, 3)).astype(np.float32)
        return np.stack([u[rng.integers(0, 300, N)] for _ in range(B)])
    raise ValueError(kind)


# SA1-size clouds (4096 < N <= 8192) run the culled hot-set sampler by default; every schedule
# pn2_fps_gather_sched offers there (PN2_FPS_AUTO, PN2_FPS_BLOCKSCAN = the v9 block scan)
# must give the oracle's
# indices: ScanNet crops with duplicates, uniform, the integer lattice (exact ties everywhere),
# npoint beyond the distinct points, npoint > N, tiny npoint, odd N.
SAMPLER_CASES = [
    ("scannet", 16, 8192, 1024), ("uniform", 4, 8192, 1024), ("grid", 4, 8192, 1024),
    ("grid", 2, 8192, 4000), ("dup", 2, 5000, 40), ("fewuniq", 2, 8192, 600),
    ("scannet", 2, 4097, 4097), ("uniform", 2, 6000, 7000), ("scannet", 3, 8192, 2),
    ("scannet", 3, 8192, 1), ("scannet", 2, 7777, 1500),
]
# MSG SA1-size clouds (8192 < N <= 16384, cfg5): the culled sampler with its coordinates in L2
# (AUTO) or the v9 512 x 32 block scan
MSG_SAMPLER_CASES = [
    ("scannet", 8, 16384, 512), ("uniform", 2, 16384, 512), ("grid", 2, 16384, 1024),
    ("grid", 1, 16384, 4000), ("dup", 1, 12000, 40), ("fewuniq", 2, 16384, 600),
    ("scannet", 1, 8193, 8193), ("uniform", 1, 12000, 13000), ("scannet", 2, 16384, 1),
    ("scannet", 2, 11111, 2000),
]


def _sched(pkg, torch, x, M, sched):
    B, N = x.shape[0], x.shape[1]
    idx = torch.empty((B, M), dtype=torch.int32, device=x.device)
    nx = torch.empty((B, M, 3), dtype=torch.float32, device=x.device)
    rc = pkg._lib.lib().pn2_fps_gather_sched(x.data_ptr(), B, N, M, idx.data_ptr(),
                                             nx.data_ptr(), sched,
                                             torch.cuda.current_stream().cuda_stream)
    return rc, idx, nx


@pytest.mark.parametrize("sched,kind,B,N,M",
                         [(s,) + c for s in (0, 1) for c in SAMPLER_CASES]
                         + [(s,) + c for s in (0, 1) for c in MSG_SAMPLER_CASES])
def test_fps_sampler_schedules(env, sched, kind, B, N, M):
    pkg, O, torch, dev = env
    x = _cloud(pkg, kind, B, N, seed=3)
    rc, idx, new_xyz = _sched(pkg, torch, torch.from_numpy(x).to(dev), M, sched)
    assert rc == 0, rc
    torch.cuda.synchronize()
    assert pkg._lib.lib().pn2_fault_status(1) == 0, "the sampler stored a device fault"
    ref = O.fps(x, M)
    _exact(f"schedule {sched} idx", idx.cpu().numpy(), ref)
    _exact(f"schedule {sched} new_xyz", new_xyz.cpu().numpy(), O.gather_point(x, ref))


def test_fps_schedule_rejections(env):
    """Schedules exist only where the culled sampler is the default: PN2_EINVAL elsewhere
    (any non-AUTO schedule at small N, unknown ids -- among them the removed 128-entry and
    lean schedules, 6-8), never a silent fallback."""
    pkg, O, torch, dev = env
    L = pkg._lib
    x = torch.from_numpy(_cloud(pkg, "scannet", 1, 16384)).to(dev)
    for gone in (6, 7, 8):
        assert _sched(pkg, torch, x[:, :8192].contiguous(), 64, gone)[0] == L.PN2_EINVAL
    assert _sched(pkg, torch, x[:, :4096].contiguous(), 64, L.PN2_FPS_BLOCKSCAN)[0] == L.PN2_EINVAL
    assert _sched(pkg, torch, x, 64, 5)[0] == L.PN2_EINVAL
    assert _sched(pkg, torch, x, 64, L.PN2_FPS_AUTO)[0] == 0


POLLTEST_LIB = os.path.join(os.path.dirname(HERE), PKG_NAME, "csrc", "build",
                            "libpn2hip_polltest.so")


def test_fps_poll_bound_reports_fault(env):
    """The culled sampler fails loudly: a build whose cold-wave poll bound is tiny
    (-DPN2_FPS_POLL_LIMIT=4, csrc/Makefile target polltest) must store PN2_FAULT_FPS_POLL,
    which pn2_fault_status reads and the next sampler call returns as PN2_EFAULT."""
    import ctypes
    pkg, O, torch, dev = env
    assert os.path.exists(POLLTEST_LIB), "build it: make -C <pkg>/csrc polltest"
    h = ctypes.CDLL(POLLTEST_LIB)
    for name in ("pn2_fps_gather", "pn2_fault_status"):
        fn = getattr(h, name)
        fn.restype, fn.argtypes = pkg._lib.SIGNATURES[name]
    x = torch.from_numpy(_cloud(pkg, "scannet", 4, 8192)).to(dev)
    idx = torch.empty((4, 1024), dtype=torch.int32, device=dev)
    nx = torch.empty((4, 1024, 3), dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    assert h.pn2_fps_gather(x.data_ptr(), 4, 8192, 1024, idx.data_ptr(), nx.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert h.pn2_fault_status(0) == pkg._lib.PN2_FAULT_FPS_POLL
    assert h.pn2_fps_gather(x.data_ptr(), 4, 8192, 1024, idx.data_ptr(), nx.data_ptr(),
                            st) == pkg._lib.PN2_EFAULT
    torch.cuda.synchronize()
    h.pn2_fault_status(1)  # this call's own (equally broken) launch did not run: clear
    # the product library is unaffected
    assert pkg._lib.lib().pn2_fault_status(0) == 0


def _chain_call(h, x, npoints, dev, torch):
    """pn2_fps_chain through library handle h: [(idx, new_xyz)] per stage, and the return code."""
    import ctypes
    B, N = x.shape[0], x.shape[1]
    outs = [(torch.empty((B, m), dtype=torch.int32, device=dev),
             torch.empty((B, m, 3), dtype=torch.float32, device=dev)) for m in npoints]
    npt = (ctypes.c_int * len(npoints))(*npoints)
    ib = (ctypes.c_void_p * len(npoints))(*[o[0].data_ptr() for o in outs])
    nb = (ctypes.c_void_p * len(npoints))(*[o[1].data_ptr() for o in outs])
    rc = h.pn2_fps_chain(x.data_ptr(), B, N, len(npoints), ctypes.addressof(npt),
                         ctypes.addressof(ib), ctypes.addressof(nb),
                         torch.cuda.current_stream().cuda_stream)
    return rc, outs


def test_fps_chain_poll_bound_reports_fault(env):
    """The sampler chain's hot-set stages report a cold wave's wait past its poll bound too
    (PN2_FAULT_FPS_POLL; the polltest build's bound is 4 polls). The cold waves go on waiting
    after reporting, so the stage's picks stay exact (they give up only at a hard bound that
    only a hung hot wave reaches)."""
    import ctypes
    pkg, O, torch, dev = env
    h = ctypes.CDLL(POLLTEST_LIB)
    for name in ("pn2_fps_chain", "pn2_fault_status"):
        fn = getattr(h, name)
        fn.restype, fn.argtypes = pkg._lib.SIGNATURES[name]
    x = _cloud(pkg, "scannet", 2, 1024)
    rc, outs = _chain_call(h, torch.from_numpy(x).to(dev), [256, 64], dev, torch)
    assert rc == 0
    torch.cuda.synchronize()
    assert h.pn2_fault_status(1) == pkg._lib.PN2_FAULT_FPS_POLL
    ref = O.fps(x, 256)
    _exact("chain stage 0 idx", outs[0][0].cpu().numpy(), ref)
    _exact("chain stage 1 idx", outs[1][0].cpu().numpy(), O.fps(O.gather_point(x, ref), 64))
    assert pkg._lib.lib().pn2_fault_status(0) == 0


TORNTEST_LIB = os.path.join(os.path.dirname(HERE), PKG_NAME, "csrc", "build",
                            "libpn2hip_torntest.so")


def test_publish_tag_check_catches_torn_reads(env):
    """The samplers' pick publishing (fps_cull.h hot_publish): a build that writes the count
    BEFORE the centre, ~800 cycles ahead of it (-DPN2_PUBLISH_BROKEN=1, csrc/Makefile target
    torntest), lets the cold waves read slots that are not yet written. Their tag check must
    catch every such read (pn2_torn_reads counts them: > 0 here) and wait, so both users of the
    publish -- the SA1 culled sampler and the SA2-4 chain -- stay index-exact."""
    import ctypes
    pkg, O, torch, dev = env
    assert os.path.exists(TORNTEST_LIB), "build it: make -C <pkg>/csrc torntest"
    h = ctypes.CDLL(TORNTEST_LIB)
    for name in ("pn2_fps_gather", "pn2_fps_chain", "pn2_fault_status"):
        fn = getattr(h, name)
        fn.restype, fn.argtypes = pkg._lib.SIGNATURES[name]
    h.pn2_torn_reads.restype, h.pn2_torn_reads.argtypes = ctypes.c_uint, []
    st = torch.cuda.current_stream().cuda_stream
    h.pn2_torn_reads()  # (clear)
    # the SA1 sampler
    x = _cloud(pkg, "scannet", 8, 8192, seed=5)
    xt = torch.from_numpy(x).to(dev)
    idx = torch.empty((8, 1024), dtype=torch.int32, device=dev)
    nx = torch.empty((8, 1024, 3), dtype=torch.float32, device=dev)
    assert h.pn2_fps_gather(xt.data_ptr(), 8, 8192, 1024, idx.data_ptr(), nx.data_ptr(), st) == 0
    torch.cuda.synchronize()
    torn_sa1 = h.pn2_torn_reads()
    ref = O.fps(x, 1024)
    _exact("torn-build SA1 idx", idx.cpu().numpy(), ref)
    _exact("torn-build SA1 new_xyz", nx.cpu().numpy(), O.gather_point(x, ref))
    # the chain (1,024 -> 256 -> 64 -> 16) over a raw cloud: over the SA1 picks its stages
    # would be prefixes (fps_prefix_holds) and no stage would sample
    nx1 = _cloud(pkg, "scannet", 8, 1024, seed=6)
    rc, outs = _chain_call(h, torch.from_numpy(nx1).to(dev), [256, 64, 16], dev, torch)
    assert rc == 0
    torch.cuda.synchronize()
    torn_chain = h.pn2_torn_reads()
    cur = nx1
    for k, ((i, n), m) in enumerate(zip(outs, [256, 64, 16])):
        r = O.fps(cur, m)
        _exact(f"torn-build chain stage {k} idx", i.cpu().numpy(), r)
        cur = O.gather_point(cur, r)
        _exact(f"torn-build chain stage {k} new_xyz", n.cpu().numpy(), cur)
    assert h.pn2_fault_status(1) == 0
    print(f"torn reads caught: SA1 {torn_sa1}, chain {torn_chain}")
    assert torn_sa1 > 0 and torn_chain > 0, (torn_sa1, torn_chain)


def _chain_vs_oracle(pkg, O, torch, dev, p, npoints, what):
    """pn2_fps_chain over p (B, n, 3) against the oracle's samplers stage by stage."""
    rc, outs = _chain_call(pkg._lib.lib(), torch.from_numpy(np.ascontiguousarray(p)).to(dev),
                           npoints, dev, torch)
    assert rc == 0
    torch.cuda.synchronize()
    cur, refs = p, []
    for k, ((i, n), m) in enumerate(zip(outs, npoints)):
        r = O.fps(cur, m)
        _exact(f"{what} stage {k} idx", i.cpu().numpy(), r)
        cur = O.gather_point(cur, r)
        _exact(f"{what} stage {k} new_xyz", n.cpu().numpy(), cur)
        refs.append(r)
    return refs


def test_chain_over_sampler_output_is_prefix(env):
    """A chain over an earlier sampler's picks (SA2-4 over the SA1 sampler's new_xyz): every
    stage is the prefix of its input (pick j of the SA1 sampling was the farthest point of the
    whole cloud, hence of its picks), which fps_prefix_holds verifies -- unique maxima at every
    step -- before the chain kernel writes the outputs as copies. Exact against the oracle's
    samplers stage by stage, on ScanNet and uniform clouds (and the property itself holds)."""
    pkg, O, torch, dev = env
    for kind in ("scannet", "uniform"):
        x = _cloud(pkg, kind, 4, 8192, seed=11)
        nx1 = O.gather_point(x, O.fps(x, 1024))
        refs = _chain_vs_oracle(pkg, O, torch, dev, nx1, [256, 64, 16], f"{kind} prefix chain")
        for r, m in zip(refs, [256, 64, 16]):
            assert (r == np.arange(m)[None]).all(), kind
        # MSG (cfg5): 512 picks -> 128
        nx1 = O.gather_point(x, O.fps(x, 512))
        _chain_vs_oracle(pkg, O, torch, dev, nx1, [128], f"{kind} msg prefix chain")


def test_chain_prefix_check_rejects(env):
    """Inputs that look like sampler output but are not prefixes -- two picks swapped; a later
    point on an early pick (a tie at that pick's maximum, which the reference's tie order gives
    to the other point); a tie in the stage's last step; duplicates of pick 0 -- must fail the
    check and run the stages as samplers: exact against the oracle."""
    pkg, O, torch, dev = env
    x = _cloud(pkg, "scannet", 4, 8192, seed=12)
    nx1 = O.gather_point(x, O.fps(x, 1024))
    cases = {}
    p = nx1.copy(); p[:, [100, 101]] = p[:, [101, 100]]; cases["swap 100/101"] = p
    p = nx1.copy(); p[:, 700] = p[:, 200]; cases["tie at pick 200"] = p
    p = nx1.copy(); p[:, 900] = p[:, 255]; cases["tie at pick 255"] = p
    p = nx1.copy(); p[:, 513] = p[:, 1]; cases["tie at pick 1"] = p
    p = nx1.copy(); p[:, 1:] = p[:, :1]; cases["all equal"] = p
    for what, p in cases.items():
        refs = _chain_vs_oracle(pkg, O, torch, dev, p, [256, 64, 16], what)
        if what.startswith("swap") or what == "tie at pick 200":
            assert not (refs[0] == np.arange(256)[None]).all(), what  # really not a prefix


FPS_GOLDEN = sorted(glob.glob(os.path.join(HERE, "golden", "fps*.npz")))


@pytest.mark.parametrize("path", FPS_GOLDEN, ids=lambda p: p.rsplit("/", 1)[-1][:-4])
def test_fps_golden_first(env, path):
    """The reference FPS kernel's own outputs (fps_*: tf_sampling_g.cu run on this GPU model;
    fpsemul_*: the kernel text on 512 CPU threads), reproduced index for index."""
    pkg, O, torch, dev = env
    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    idx, new_xyz = pkg.tf_sampling.farthest_point_sample_and_gather(
        int(meta["npoint"]), torch.from_numpy(np.ascontiguousarray(z["xyz"])).to(dev))
    _exact("idx", idx.cpu().numpy(), z["idx"])
    if "new_xyz" in z.files:
        _exact("new_xyz", new_xyz.cpu().numpy(), z["new_xyz"])
