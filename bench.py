#!/usr/bin/env python3
"""Benchmark: 8192-point clouds per second through the PointNet++ SA + FP geometric path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg5] [--batch B]

One step = every geometric op of the SSG SA x4 + FP x4 stack (stack.py) over one batch of
B clouds per GPU (cfg2: B = 16 ScanNet-crop clouds of 8192 points, BASELINE.json configs[1]).
Inputs are generated and made resident in HBM before the timed region. For N > 1 the driver
launches one process per GPU (torch.distributed.run); every rank owns B clouds (batch split,
weak scaling, no collective in the data path); the timed region is bracketed by a barrier and
torch.cuda.synchronize() and the max over ranks is reported. Rank 0 prints ONE JSON line.
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# HIP hardware queues per process (GPU_MAX_HW_QUEUES, set from --hw-queues before HIP starts;
# the GPU box exports 4). Streams map onto them round-robin. Measured on one box
# (scripts/archive/r5/ab_queues.sh): with 4 queues the geometric step runs 21.7k
# clouds/s, with 8 or 16 the side lanes run fully beside the SA1 sampler and slow it from
# 0.72 to 0.81 ms (18.7k clouds/s) -- while the whole-model step gains (11.2k -> 14.5k).
DEFAULT_HW_QUEUES = 4
# The geometric step's pipeline layout per config, measured on MI355X (DESIGN.md §3.6,
# profiles/r3/plan/): sampler streams (consecutive steps' samplers run concurrently, one
# workgroup per cloud each), side-lane layout (stack.side_layout), hardware queues (one per
# stream: samplers + side lanes) and buffer sets (how far the host may run ahead).
# chain: the later samplers (SA2.. chain) behind SA1 on its sampler stream, or on a stream of
# their own (profiles/r3/chainown: cfg2 65.6k -> 69.8k, cfg3 50.7k -> 54.3k clouds/s; cfg5 no
# gain). cfg2's sets: 5 (round 6, the driver's command, ten interleaved runs each, profiles/r6/
# sets20, sets20b: median 78.4k, min 76.8k against 75.0k / 70.1k with 9; 4 / 6 / 7 sets 75.6 /
# 75.3 / 76.5k; 500 steps 92.1 / 90.9k against 90.5 / 90.4k): the side lanes bound the step, and
# fewer sets hold the samplers' run-ahead -- and the CUs it takes from the side work -- shorter.
LAYOUTS = {"cfg2": {"lanes": 3, "side": "b", "queues": 7, "sets": 5, "chain": "own"},
           "cfg3": {"lanes": 2, "side": "a", "queues": 6, "sets": 6, "chain": "own"},
           "cfg5": {"lanes": 5, "side": "a", "queues": 8, "sets": 10, "chain": "behind"}}

PKG = "pointcloud-segmentation-attention_amd"
METRIC = "8192-pt clouds/sec through SA+FP layers, 1/2/4/8 MI355X; HBM GB/s vs peak"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
WORKLOADS = {
    "cfg2": "cfg2: B=16 8192-pt ScanNet crops per GPU, SSG SA x4 + FP x4 geometry "
            "(FPS+gather, ball query, group/centre/concat, three_nn+IDW+interpolate+concat)",
    "cfg3": "cfg3: cfg2 with rgb+normal features (C=9 grouped at SA1) + attention reduction "
            "in every SA",
    "cfg5": "cfg5: MSG SA1+SA2 grouping, B=8 16384-pt ScanNet crops per GPU",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cpu_share():
    """Host threads this process may use: the box's CPU share (OMP_NUM_THREADS, 16 on the
    GPU box), bounded by the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(env))) if env and env.isdigit() else aff


def cpu_baseline(config, B_per_step, seconds, threads):
    """The oracle (C restatement of the reference's CPU loops, oracle/pn2_oracle.c) timed on
    this host over a bounded sample of the same workload, twice: single-threaded (the
    reference's loops are serial) and on `threads` threads (OpenMP over clouds; default: the
    box's CPU share). The machine's full core count and CPU model are stated, and the
    all-cores rate is extrapolated linearly from the measured per-thread rate (an upper
    bound for the CPU, so the GPU ratio against it is the conservative one)."""
    from oracle import oracle as O
    pkg = importlib.import_module(PKG)

    def timed(nthreads, budget):
        O.set_threads(nthreads)
        B = max(nthreads, 1)
        inp = pkg.stack.make_inputs(config, list(range(B)), "cpu")
        np_inp = dict(inp)
        np_inp["xyz"] = inp["xyz"].numpy()
        np_inp["feats"] = None if inp["feats"] is None else inp["feats"].numpy()
        for k in ("sa_out", "fp_out"):
            if k in inp:
                np_inp[k] = [t.numpy() for t in inp[k]]
        if "attn" in inp:
            np_inp["attn"] = [tuple(t.numpy() for t in qkv) for qkv in inp["attn"]]
        O.run_stack_cpu(np_inp, config)  # warm-up (page-in, OpenMP pool)
        clouds, t0 = 0, time.perf_counter()
        while True:
            O.run_stack_cpu(np_inp, config)
            clouds += B
            el = time.perf_counter() - t0
            if el >= budget:
                return clouds / el, clouds, el

    nproc = os.cpu_count() or 1
    v1, c1, e1 = timed(1, seconds / 2)
    vt, ct, et = timed(threads, seconds / 2)
    est_all = v1 * nproc
    eff = vt / (v1 * threads)  # measured 1 -> `threads` scaling efficiency
    return {"value": vt, "unit": "clouds/s", "cores": threads, "kind": "port",
            "value_1core": v1, "value_threads": vt, "threads": threads,
            "scaling_efficiency_1_to_threads": eff,
            "cores_all": nproc, "value_all_cores_extrapolated": est_all,
            "value_all_cores_at_measured_efficiency": est_all * eff,
            "cpu_model": _cpu_model(),
            "sample": f"{config} steps of the C restatement oracle/pn2_oracle.c: {c1} clouds "
                      f"(1 per call) in {e1:.1f} s on 1 thread; {ct} clouds ({threads} per call, "
                      f"OpenMP over clouds) in {et:.1f} s on {threads} threads (the box's CPU "
                      f"share); all-cores figures = 1-core rate x {nproc} (nproc), linear (an upper "
                      "bound) and at the measured 1->threads efficiency, extrapolated, not run "
                      "(the box allows its CPU share only)"}


def cfg1_leg(dev, seconds=2.0):
    """BASELINE.json configs[0] (BASELINE.md:61): B = 1, N = 1024 uniform points, ONE SA layer
    (npoint 256, r 0.2, nsample 32, xyz only): farthest-point sampling + gather + ball query +
    grouping. CPU: the C restatement (oracle/pn2_oracle.c, the reference's loops) on 1 thread,
    repeated for ~`seconds`; GPU: pointnet_util.sample_and_group on this device (the same four
    ops; HIP events, median of 50), both per layer call, and the outputs compared."""
    import numpy as np
    import torch
    from oracle import oracle as O
    pkg = importlib.import_module(PKG)
    x = pkg.synth.batch([0], 1024, "uniform")[0]
    O.set_threads(1)

    def cpu_sa():
        idx = O.fps(x, 256)
        nx = O.gather_point(x, idx)
        bidx, _ = O.ball_query(x, nx, 0.2, 32)
        return nx, bidx, O.group_concat(x, None, nx, bidx)[0]
    ref = cpu_sa()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        cpu_sa()
        n += 1
    cpu_ms = (time.perf_counter() - t0) / n * 1e3
    xt = torch.from_numpy(x).to(dev)
    sg = pkg.pointnet_util.sample_and_group
    for _ in range(5):
        out = sg(256, 0.2, 32, xt, None)
    ts = []
    for _ in range(50):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = sg(256, 0.2, 32, xt, None)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    same = (np.array_equal(out[0].cpu().numpy(), ref[0]) and np.array_equal(out[2].cpu().numpy(), ref[1])
            and np.array_equal(out[1].cpu().numpy().view(np.int32), ref[2].view(np.int32)))
    return {"workload": "cfg1: B=1, N=1024 uniform, one SA layer (FPS 256 + gather + ball query "
                        "r=0.2 ns=32 + grouping), BASELINE.json configs[0]",
            "cpu_ms_per_call_1core": cpu_ms, "cpu_calls": n, "cpu_kind": "port",
            "gpu_ms_per_call": ts[len(ts) // 2], "gpu_over_cpu": cpu_ms / ts[len(ts) // 2],
            "gpu_note": "pointnet_util.sample_and_group on the MI355X, HIP events around one call "
                        "(four launches), median of 50",
            "outputs_equal": bool(same)}


def copy_peak(dev, mib=1024, reps=5):
    """A measured HBM figure beside the 8 TB/s nominal (BASELINE.md:75): a float4 copy kernel
    (pn2_copy_f4: four 16-byte loads in flight per thread, 16 workgroups per CU, the form
    MI355X_MICROARCH.md measures 6.29 TB/s with) of `mib` MiB, read + write bytes per second,
    best of `reps`; torch's copy_ (hipMemcpyAsync) beside it for reference."""
    import torch
    L = importlib.import_module(PKG).lib()
    n = mib * 1024 * 1024 // 4
    a = torch.empty(n, dtype=torch.float32, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    st = torch.cuda.current_stream(dev).cuda_stream

    def best_ms(fn):
        fn()
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best

    def kernel():
        rc = L.pn2_copy_f4(a.data_ptr(), b.data_ptr(), n * 4, cus, st)
        if rc:
            raise RuntimeError(f"pn2_copy_f4: {rc}")

    ms = best_ms(kernel)
    assert torch.equal(a, b)
    ms_torch = best_ms(lambda: b.copy_(a))
    del a, b
    return {"GBps": 2 * n * 4 / (ms * 1e-3) / 1e9, "bytes": 2 * n * 4,
            "torch_copy_GBps": round(2 * n * 4 / (ms_torch * 1e-3) / 1e9, 1),
            "method": f"float4 copy kernel (pn2_copy_f4, {cus} CUs x 16 workgroups) of {mib} "
                      f"MiB, read + write bytes, best of {reps}"}


def pmc_traffic(config, B):
    """HBM bytes per launch of the SA1 sampler from the committed rocprofv3 --pmc summary
    (profiles/<round>/pmc_traffic_<config>_B<B>.json, written by tools/pmc_summary.py from
    separate FETCH_SIZE and WRITE_SIZE passes of this bench). Counters cannot be read inside
    this (unprofiled) process, so the figure is the profiled run's, for the same workload."""
    files = _profile_files(f"pmc_traffic_{config}_B{B}.json")
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    ks = [k for k in d["kernels"] if k.startswith(("fps_hotcull", "fps_v"))]
    if not ks:
        return None, None
    k = max(ks, key=lambda k: d["kernels"][k]["fetch_bytes"] or 0)  # SA1 = largest sampler
    e = d["kernels"][k]
    # FETCH_SIZE x2: the gfx950 correction of MI355X_MICROARCH.md (HBM section); for this
    # kernel it lands within 6 % of the algorithmic read bytes, and WRITE_SIZE equals the
    # idx + new_xyz bytes exactly.
    return e["fetch_bytes_x2"] + e["write_bytes"], os.path.relpath(files[-1], ROOT) + f" [{k}]"


def sa1_algorithmic_bytes(B, N, M1, known_grid):
    """Algorithmic bytes of one SA1 sampler launch: the cloud read once (N x 12), idx + new_xyz
    written (M1 x 16), per cloud; with known_grid (the sampler's workgroups grid their picks for
    FP4, pn2_fps_chain_grid) also that grid: header, max(M1, 64) + 1 offsets, M1 sorted points
    (csrc/grid.h)."""
    grid = 32 + (max(M1, 64) + 1) * 4 + M1 * 16 if known_grid else 0
    return B * (N * 12 + M1 * 16 + grid)


MAX_CLOCK_GHZ = 2.4  # MI355X_MICROARCH.md, chip-level parameters


def _profile_files(name):
    """Committed profile files of this name, oldest first: profiles/r<N>/ and profiles/r<N>/*/,
    by round, a round's end-of-round evidence (final/) last."""
    import glob
    import re
    files = (glob.glob(os.path.join(ROOT, "profiles", "*", name)) +
             glob.glob(os.path.join(ROOT, "profiles", "*", "*", name)))

    def key(p):
        rel = os.path.relpath(p, os.path.join(ROOT, "profiles"))
        m = re.match(r"r(\d+)", rel)
        return (int(m.group(1)) if m else -1, "/final/" in "/" + rel, rel)
    return sorted(files, key=key)


def _latest_profile(name):
    files = _profile_files(name)
    if not files:
        return None, None
    with open(files[-1]) as f:
        return json.load(f), os.path.relpath(files[-1], ROOT)


def sa1_latency(config, fps_ms, M1, N):
    """The SA1 sampler's own bound: its picks are a serial chain (tf_sampling_g.cu:124-168), one
    CU per cloud. Measured: the committed stamp summary of the culled sampler
    (profiles/<round>/sa1_cull_stamps.json, tools/stamp_fps_cull.py: cycles per pick of the hot
    wave, rounds, cycles per round, setup). Floor: the same pieces run ALONE on one CU
    (profiles/<round>/sampler_floor.json, tools/ubench/pick_floor.hip): the dependent chain of
    one pick (lane best of 4, 64-lane DPP max, winner, coordinates, distance update) and the
    synchronisation skeleton of a round end (3 barriers + 2 cross-wave reductions, 16 waves),
    plus the cloud read at one CU's share of HBM. floor = setup + (M - 1) x pick + rounds x
    round; frac = floor / measured launch (1 = the launch runs at the floor)."""
    out = {"ns_per_pick": fps_ms * 1e6 / max(1, M1 - 1)}
    # cfg2/cfg3 SA1 (8192 -> 1024) and cfg5's MSG SA1 (16384 -> 512) are stamped separately
    st, st_src = _latest_profile("msg_cull_stamps.json" if config == "cfg5" else
                                 "sa1_cull_stamps.json")
    fl, fl_src = _latest_profile("sampler_floor.json")
    if config in ("cfg2", "cfg3", "cfg5") and st:
        out.update({k: st[k] for k in ("hot_cycles_per_pick", "rounds", "round_cycles",
                                      "setup_cycles", "kernel_cycles") if k in st})
        out["source"] = st_src
    if fl:
        out.update({"floor_cycles_per_pick": fl["pick_chain_cycles"],
                    "floor_pick_step_cycles": fl["pick_step_cycles"],
                    "floor_round_cycles": fl["round_sync_cycles"], "floor_source": fl_src})
        # the cloud read once at one CU's share of the HBM peak (8 TB/s over 256 CUs)
        out["floor_setup_cycles"] = N * 12 / (HBM_PEAK_GBPS / 256 / MAX_CLOCK_GHZ)
        if "rounds" in out:
            floor = (out["floor_setup_cycles"] + (M1 - 1) * out["floor_cycles_per_pick"]
                     + out["rounds"] * out["floor_round_cycles"])
            out["floor_launch_cycles"] = floor
            out["floor_launch_ms"] = floor / (MAX_CLOCK_GHZ * 1e6)
            if "hot_cycles_per_pick" in out:
                out["frac_pick"] = out["floor_cycles_per_pick"] / out["hot_cycles_per_pick"]
                out["frac_round"] = out["floor_round_cycles"] / out["round_cycles"]
    return out


def verify_sets(config, runs, threads):
    """The CHECKER (outside every timed region): each buffer set's last step -- its inputs,
    outputs and index intermediates -- against the oracle (oracle/pn2_oracle.c, the C
    restatement pinned to the reference's own code) with north_star's bars: bit-exact indices
    and copies, 1e-5 for interpolated features and the attention reduction."""
    from oracle import oracle as O
    O.set_threads(threads)
    fails, clouds, t0 = [], 0, time.perf_counter()
    for inp, outs, inter in runs:
        np_inp = dict(inp)
        np_inp["xyz"] = inp["xyz"].cpu().numpy()
        np_inp["feats"] = None if inp["feats"] is None else inp["feats"].cpu().numpy()
        for k in ("sa_out", "fp_out"):
            if k in inp:
                np_inp[k] = [t.cpu().numpy() for t in inp[k]]
        if "attn" in inp:
            np_inp["attn"] = [tuple(t.cpu().numpy() for t in qkv) for qkv in inp["attn"]]
        fails += O.compare_stack(np_inp, config, [o.cpu().numpy() for o in outs],
                                 {k: v.cpu().numpy() for k, v in inter.items()})
        clouds += int(inp["B"])
    return {"sets": len(runs), "clouds": clouds, "failures": fails[:8],
            "seconds": time.perf_counter() - t0, "threads": threads,
            "checker": "oracle.compare_stack: every output and index intermediate of each "
                       "buffer set's last step vs oracle/pn2_oracle.c (bit-exact indices and "
                       "copies; rtol=atol=1e-5 interpolated features / attention)"}


def _e2e_child(args, e2e):
    """The whole-model measurement in a child process (`bench.py --model`, same config, queues
    and steps). HIP maps streams to hardware queues round-robin in creation order, so in the
    geometric step's process the model's streams land on other queues than in a standalone
    run (12.7-13.1k vs 16.2-16.4k clouds/s). Fills e2e and returns True, or
    returns False (the caller then measures in process)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--model", "--config", args.config,
           "--steps", str(args.e2e_steps), "--warmup", str(min(args.warmup, 5)),
           "--no-cpu-baseline", "--time-every", str(args.time_every), "--sets", "3",
           "--lane0-priority", args.lane0_priority, "--hw-queues", str(DEFAULT_HW_QUEUES)]
    if args.batch:
        cmd += ["--batch", str(args.batch)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=dict(os.environ))
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1] \
            if r.returncode == 0 else None
    except (subprocess.TimeoutExpired, IndexError):
        line = None
    if not line:
        log("e2e child failed; measuring in process")
        return False
    d = json.loads(line)
    e2e.update({"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"],
                "steps": d["steps"], "sa1_sampler_ms": d["roofline"]["avg_launch_ms"],
                "checksum": d["checksum"], "lane0_priority": d["config"]["lane0_priority"],
                "process": "child (bench.py --model)"})
    return True


def launch_ranks(ngpus, argv):
    """`bench.py --gpus N` outside torch.distributed.run: launch N ranks of this script on one
    node (torch.distributed.run, rendezvous on 127.0.0.1) as a child process and return its
    exit status. Rank 0 prints the JSON line. The reference's only parallelism is this batch
    split (pointnet2_tensorflow/train_multi_gpu.py:181-190)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ngpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between ranks)
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"launching {ngpus} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def dry_run(args):
    """The multi-rank plumbing without kernels (CPU, gloo): shard ids, per-rank synthetic
    inputs, barrier-bracketed timing with the max over ranks, per-cloud checksum gather."""
    import torch.distributed as dist
    pkg = importlib.import_module(PKG)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    B = args.batch or (8 if args.config == "cfg5" else 16)
    ids = pkg.shard.shard_ids(rank, world, B)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    inp = pkg.stack.make_inputs(args.config, ids, "cpu")
    outs = [inp["xyz"]] + ([inp["feats"]] if inp["feats"] is not None else []) \
        + list(inp["sa_out"]) + list(inp.get("fp_out", []))
    if world > 1:
        dist.barrier()
    elapsed = pkg.shard.max_over_ranks(time.perf_counter() - t0)
    sums = pkg.shard.gather_checksums(pkg.shard.cloud_checksums(outs, B))
    # what each rank would run: its shard of every buffer set, and the hardware-queue setting
    # its HIP runtime would start with (bench.py sets it before anything touches the GPU)
    mine = {"rank": rank, "ids": ids, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            "set_ids": [pkg.shard.set_ids(rank, world, B, i) for i in range(args.sets)]}
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "clouds/s", "n_gpus": world,
                          "dry_run": True, "clouds": world * B, "clouds_per_rank": B,
                          "elapsed_max_over_ranks": elapsed,
                          "checksum": float(sums.sum().item()),
                          "per_cloud_checksums": [float(x) for x in sums.tolist()],
                          "ranks": ranks, "sets": args.sets,
                          "config": {"config": args.config, "clouds_per_gpu": B,
                                     "global_batch": world * B,
                                     "parallelism": f"dp{world} (batch split)"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500,
                    help="timed steps (the pipelined steps' fill and drain are amortised over "
                         "them: cfg2 63-64k clouds/s at 50 steps, 68-71k at 400, 72k at 1000, "
                         "profiles/r3/steps)")
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="clouds per GPU (default: config's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the multi-threaded CPU baseline leg (default: the box's "
                         "CPU share, OMP_NUM_THREADS / affinity)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="launch every op from Python instead of replaying the captured hipGraphs")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run the whole step on one stream (no side stream beside the sampler chain)")
    ap.add_argument("--time-every", type=int, default=10,
                    help="bracket every Nth timed step's SA1 sampler with HIP events (the "
                         "roofline's launch time is their mean; two event packets on lane 0 "
                         "per bracketed step cost ~10 us of step time, DESIGN.md §5)")
    ap.add_argument("--sets", type=int, default=None,
                    help="buffer sets the pipelined steps rotate over (>= 2; default: the "
                         "config's LAYOUTS entry, 3 for --model)")
    ap.add_argument("--sampler-lanes", type=int, default=None,
                    help="streams the pipelined steps' samplers alternate over (consecutive "
                         "steps' samplers run at the same time on different CUs; default: the "
                         "config's LAYOUTS entry, 1 for --model)")
    ap.add_argument("--side-layout", choices=["a", "b", "c", "d"], default=None,
                    help="side-lane layout with several sampler streams (stack.side_layout; "
                         "default: the config's LAYOUTS entry)")
    ap.add_argument("--chain", choices=["own", "own2", "own3", "behind"], default=None,
                    help="with several sampler streams: the later samplers (SA2.. chain) on a "
                         "stream of their own or behind SA1 on its sampler stream (default: the "
                         "config's LAYOUTS entry)")
    ap.add_argument("--private-side", action="store_true",
                    help="every buffer set gets its own side streams (side work of consecutive "
                         "steps runs concurrently; needs 1 + 2 x sets + sampler lanes - 1 "
                         "hardware queues)")
    ap.add_argument("--diag-only", choices=["samplers", "side"], default=None,
                    help="DIAGNOSTIC: time only the samplers or only the side-lane work of each "
                         "step (the line is marked diagnostic; never a benchmark result)")
    ap.add_argument("--no-native-plan", action="store_true",
                    help="enqueue each step with the Python task loop instead of one call into "
                         "the native plan executor (include/pn2plan.h)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="join every step before the next (no overlap of step k's side work "
                         "with step k+1's samplers)")
    ap.add_argument("--model", action="store_true",
                    help="the step is the whole segmentation model's inference forward "
                         "(SA/FP geometry + fused MLPs + head) instead of the geometry alone")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (default: the environment's, else "
                         f"{DEFAULT_HW_QUEUES}; <= 32)")
    ap.add_argument("--graph-launch", action="store_true",
                    help="A/B: launch each side segment as its captured hipGraph instead of its "
                         "kernels directly (pn2_plan_graph_direct; DESIGN.md §3.6d)")
    ap.add_argument("--fp4-known-grid", choices=["lane", "sampler", "off"], default=None,
                    help="A/B: FP4's known-point grid built by a launch on FP4's lane, "
                         "by the SA1 sampler after its last pick (pn2_fps_chain_grid), or by "
                         "each FP4 workgroup in LDS (off); default: per config "
                         "(stack.FP4_KNOWN_GRID_BY_CONFIG)")
    ap.add_argument("--lane0-priority", choices=["auto", "default", "high"], default="auto",
                    help="stream priority of lane 0 (the SA1 sampler chain); auto = default "
                         "for the geometric step, high for the whole model")
    ap.add_argument("--e2e-in-process", action="store_true",
                    help="measure the e2e field in this process after the geometric step "
                         "(default at N = 1: a fresh child process, `bench.py --model`, whose "
                         "streams get the hardware-queue mapping of a standalone run)")
    ap.add_argument("--e2e-steps", type=int, default=20,
                    help="after the geometric measurement, time this many whole-model steps "
                         "(reported as 'e2e'; 0 = skip)")
    ap.add_argument("--timeline", default=None, metavar="PATH",
                    help="DIAGNOSTIC: bracket every timed sampler with events and write, per "
                         "step, the host's wait / enqueue times and the GPU times of the sampler "
                         "and of each side lane's end (relative to one base event) to PATH (JSON)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the post-run oracle check of every buffer set's last step (the "
                         "line's `verified` is then null)")
    ap.add_argument("--latency-reps", type=int, default=10,
                    help="un-pipelined single steps timed after the run (latency_ms_per_batch)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rank plumbing only, on the CPU over gloo: every rank builds "
                         "its shard's synthetic inputs and checksums them per cloud; max-over-"
                         "ranks timing and the checksum gather run as in the real bench; no "
                         "kernels, value = null (tests/test_bench_launcher.py)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the ranks as children BEFORE anything touches the GPU
        # (this process never initialises HIP), and exit with the launcher's status
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    lay = LAYOUTS[args.config]
    if args.sampler_lanes is None:
        args.sampler_lanes = 1 if args.model else lay["lanes"]
    if args.sets is None:
        args.sets = 3 if args.model else lay["sets"]
    if args.sets < 2:
        ap.error("--sets: a pipelined run needs at least 2 buffer sets")
    if args.side_layout is None:
        args.side_layout = lay["side"]
    if args.chain is None:
        args.chain = lay["chain"]
    if args.hw_queues is None and not args.model and args.sampler_lanes == lay["lanes"]:
        args.hw_queues = lay["queues"]  # one queue per stream (the box's default is 4)
    if args.hw_queues is not None:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(1, args.hw_queues)))
    else:
        os.environ.setdefault("GPU_MAX_HW_QUEUES", str(DEFAULT_HW_QUEUES))
    if args.dry_run:  # (after the queue setting: every rank reports what HIP would see)
        return dry_run(args)

    import torch
    import torch.distributed as dist

    pkg = importlib.import_module(PKG)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI

    B = args.batch or (8 if args.config == "cfg5" else 16)
    ids = pkg.shard.shard_ids(rank, world, B)  # contiguous batch split

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # Lane 0 (the SA1 sampler chain) runs on the current stream. "high" makes it a
    # high-priority stream (HIP keeps a separate queue pool per priority, so the sampler never
    # waits behind side-lane work in a shared queue). Measured (scripts/archive/r5/ab_prio.sh,
    # DESIGN.md §3.6): the geometric step is faster with the default priority (21.8k vs 18.9k
    # clouds/s: with its side lanes fully concurrent the latency-bound sampler slows 0.715 ->
    # 0.80 ms), the whole model with high (its side lanes carry most of the work). "auto" =
    # default for the geometric step, high for the whole model.
    # Created only when used: a stream made before the step's side lanes takes a hardware
    # queue, and one of the side lanes then shares one (stack.side_stream).
    def measure(model, steps, warmup):
        prio = args.lane0_priority
        if prio == "auto":
            prio = "high" if model else "default"
        lane0 = (torch.cuda.Stream(device=dev, priority=-1) if prio == "high"
                 else torch.cuda.current_stream(dev))
        with torch.cuda.stream(lane0):
            return _measure(model, steps, warmup) + (prio,)

    def _measure(model, steps, warmup):
        """W warm-up steps, then K timed steps between barrier + synchronize; then, outside the
        timed region, the sampler fault word, the oracle check of every buffer set's last step
        and the latency of one un-pipelined step. Returns (max-over-ranks elapsed seconds, mean
        SA1-sampler ms, last outputs, post-run checks)."""
        overlap = not args.no_overlap
        pipelined = overlap and not args.no_pipeline
        # every buffer set holds its own clouds (shard.set_ids): consecutive pipelined steps
        # sample different clouds, never one input replayed
        set_inputs = ([pkg.stack.make_inputs(args.config, pkg.shard.set_ids(rank, world, B, i),
                                             dev, model=model) for i in range(args.sets)]
                      if pipelined else None)
        inp = set_inputs[0] if pipelined else pkg.stack.make_inputs(args.config, ids, dev,
                                                                     model=model)
        torch.cuda.synchronize()
        if pipelined:
            pkg.stack.TIMING_EVENTS = bool(args.timeline) and not model
            pkg.stack.FP4_KNOWN_GRID = args.fp4_known_grid
            pipe = pkg.stack.Pipeline(inp, graphs=not args.eager, nsets=args.sets,
                                      sampler_lanes=1 if model else args.sampler_lanes,
                                      private_streams=model or args.private_side,
                                      native_plan=not args.no_native_plan,
                                      only=args.diag_only, layout=args.side_layout,
                                      chain_own=args.chain.startswith("own"),
                                      chain_streams=int(args.chain[3:] or 1)
                                      if args.chain.startswith("own") else 1,
                                      set_inputs=set_inputs,
                                      direct=not args.graph_launch)
            # every buffer set's step once, before the warm-up (Pipeline.prime)
            primed = pipe.prime()
        else:
            step = pkg.stack.Step(inp, overlap=overlap)
            graph = None if args.eager else pkg.stack.GraphStep(inp, overlap=overlap)
            primed = 0

        def run_step(events=None):
            if pipelined:
                return pipe.run(events)
            if graph is not None:
                return graph.replay(events)
            return step.run(events)

        def finish():
            return pipe.join() if pipelined else None

        for _ in range(warmup):
            run_step()
        finish()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        barrier()
        if pipelined:
            pipe.host_wait_s = pipe.host_launch_s = 0.0
            if args.timeline and not model:
                pipe.start_trace()
        t0 = time.perf_counter()
        outs = None
        every = 1 if (args.timeline and pipelined and not model) else args.time_every
        timed_k = [] if args.diag_only == "side" else \
            [k for k in range(steps) if k % every == 0]
        for k in range(steps):
            outs = run_step(ev[k] if k in timed_k else None)
        outs = finish() or outs
        torch.cuda.synchronize()
        barrier()
        elapsed = pkg.shard.max_over_ranks(time.perf_counter() - t0, dev)
        timed = [ev[k] for k in timed_k]
        fps_ms = (sum(a.elapsed_time(b) for a, b in timed) / len(timed)  # SA1 sampler, per launch
                  if timed else float("nan"))
        if pipelined:  # host time per step: waiting for a free buffer set / enqueueing a step
            host["wait_ms_per_step"] = pipe.host_wait_s / steps * 1e3
            host["enqueue_ms_per_step"] = pipe.host_launch_s / steps * 1e3
            if getattr(pipe, "trace", None) is not None:
                with open(args.timeline, "w") as fh:
                    json.dump({"elapsed_ms": elapsed * 1e3, "steps": pipe.finish_trace()}, fh)
        post = {"primed_steps": primed}
        # the sampler fault word (include/pn2hip.h pn2_fault_status) after the timed steps:
        # a fault raises here, so a fast but wrong line is never printed
        post["fault_status"] = pipe.check_faults() if pipelined else \
            pkg._lib.check_device_faults(dev) or 0
        if not model and args.diag_only is None and not args.no_verify:
            runs = (pipe.outputs_by_set() if pipelined else
                    [(inp, (graph.step if graph is not None else step).outputs(),
                      (graph.step if graph is not None else step).intermediates())])
            threads = max(1, (args.cpu_threads or _cpu_share()) // world)
            post["verify"] = verify_sets(args.config, runs, threads)
            ok = pkg.shard.min_over_ranks(0.0 if post["verify"]["failures"] else 1.0, dev)
            post["verified"] = ok == 1.0
        # one step alone, enqueued and joined (no pipelining): the latency of one batch
        lat = []
        for _ in range(args.latency_reps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            run_step()
            finish()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t1)
        if lat:
            lat.sort()
            post["latency_ms_per_batch"] = pkg.shard.max_over_ranks(lat[len(lat) // 2], dev) * 1e3
            post["latency_ms_per_batch_min"] = lat[0] * 1e3
        return elapsed, fps_ms, outs, post

    overlap = not args.no_overlap
    pipelined = overlap and not args.no_pipeline
    host = {}
    elapsed, fps_ms, outs, post, prio0 = measure(args.model, args.steps, args.warmup)
    host_geom = dict(host)
    # per-cloud output checksums, gathered (outside the timed region) so ranks can be compared
    sums = pkg.shard.gather_checksums(pkg.shard.cloud_checksums(outs, B))
    e2e = None
    if not args.model and args.e2e_steps > 0 and pkg.stack.CONFIGS[args.config][1] == "ssg":
        e2e = {}
        child = world == 1 and not args.e2e_in_process and _e2e_child(args, e2e)
        if not child:
            # after the geometric step: the stream-to-queue mapping is round-robin in creation
            # order, and creating the model's streams first cost the geometric step 29 %
            e_el, e_fps, e_outs, _, e_prio = measure(True, args.e2e_steps, min(args.warmup, 5))
            e_sums = pkg.shard.gather_checksums(pkg.shard.cloud_checksums(e_outs, B))
            e2e.update({"value": world * B * args.e2e_steps / e_el, "unit": "clouds/s",
                        "ms_per_step": e_el / args.e2e_steps * 1e3, "steps": args.e2e_steps,
                        "sa1_sampler_ms": e_fps, "checksum": float(e_sums.sum().item()),
                        "lane0_priority": e_prio, "process": "same as the geometric step"})
        e2e.update({
               "model": ("pointnet2_sem_seg_attention with rgb+normal inputs, inference "
                         "forward: SA x4 (fused group + MLP, Dense q/k/v on the matrix cores, "
                         "attention reduction + batch norm)" if args.config == "cfg3" else
                         "pointnet2_sem_seg inference forward: SA x4 (fused group + MLP + max "
                         "pool)") + ", FP x4 (fused interpolation + MLP), fc1+fc2 head fused "
                        "into FP4; fp32 matrix cores; reference initialisers, fixed seed"})

    if rank == 0:
        clouds = world * B * args.steps
        value = clouds / elapsed
        by = pkg.stack.sa_fp_bytes(args.config, B)
        step_bytes = sum(by.values())
        N, _, _, _ = pkg.stack.CONFIGS[args.config]
        M1 = (pkg.stack.MSG_SA if args.config == "cfg5" else pkg.stack.SSG_SA)[0][0]
        # algorithmic bytes of the timed SA1 sampler launch (FPS + fused gather): read the
        # cloud once (N x 12), write idx + new_xyz (M1 x (4 + 12)), per cloud; plus FP4's known
        # grid when the sampler's workgroups build it (cfg2)
        kg_mode = (None if args.model or args.config == "cfg5" else
                   pkg.stack.FP4_KNOWN_GRID or pkg.stack.FP4_KNOWN_GRID_BY_CONFIG.get(args.config))
        fps_bytes = sa1_algorithmic_bytes(B, N, M1, kg_mode == "sampler")
        achieved = fps_bytes / (fps_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(args.config, B)
        lat = sa1_latency(args.config, fps_ms, M1, N)
        hbm = {"achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
               "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
               "traffic_source": traffic_src, "algorithmic_bytes_per_launch": fps_bytes}
        if "floor_launch_ms" in lat:
            # the bound that applies: the serial pick chain (HBM is 1.8 MB per launch); time-
            # like, so achieved = the measured launch, peak = its floor, frac = peak / achieved
            roof = {"bound": "latency", "achieved": fps_ms * 1e6, "peak": lat["floor_launch_ms"] * 1e6,
                    "unit": "ns per launch", "frac": lat["floor_launch_ms"] / fps_ms}
        else:
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBPS}
        result = {
            "metric": METRIC, "value": value, "unit": "clouds/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: SplitMix64 ScanNet-crop clouds (8192 drawn with replacement from "
                    "12k surface points); " + ("random-init model weights (reference "
                    "initialisers)" if args.model else "U[-1,1) stand-ins for the MLP outputs"),
            "config": {"workload": ("whole-model inference forward, " if args.model else "")
                       + WORKLOADS[args.config], "config": args.config,
                       "clouds_per_gpu": B, "global_batch": world * B, "points": N,
                       "parallelism": f"dp{world} (batch split)",
                       "launch": "eager" if args.eager else
                       ("samplers: direct launches; side lanes: hipGraph replay"
                        + ("; one native plan call per step (include/pn2plan.h), side "
                           + ("segments as graph launches" if args.graph_launch else
                              "kernels launched directly")
                           if pipelined and not args.no_native_plan else "")),
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0")),
                       "fp4_known_grid": None if args.model or args.config == "cfg5"
                       else (pkg.stack.FP4_KNOWN_GRID
                             or pkg.stack.FP4_KNOWN_GRID_BY_CONFIG.get(args.config, "off")),
                       "lane0_priority": prio0,
                       "streams": (("SA1 sampler + 3 side streams" if args.sampler_lanes <= 1 or args.model
                                    else f"{args.sampler_lanes} sampler streams (consecutive steps' "
                                    f"samplers concurrent; SA2.. samplers "
                                    + ("behind SA1" if args.chain == "behind" else
                                       "on their own stream" if args.chain == "own" else
                                       f"on {args.chain[3:]} streams of their own, by buffer set")
                                    + ") + side streams "
                                    f"(layout {args.side_layout})"
                                    + (" per buffer set" if args.private_side else ""))
                                   if overlap else "one stream")
                       + (f", steps software-pipelined over {args.sets} buffer sets, each set "
                          "its own clouds" if pipelined else "")},
            "roofline": dict(
                {"kernel": f"SA1 sampler (FPS + gather fused): {B} clouds x {N} pts -> {M1}, "
                           "one workgroup per cloud"},
                **roof, traffic=traffic, traffic_source=traffic_src, avg_launch_ms=fps_ms,
                algorithmic_bytes_per_launch=fps_bytes, latency=lat, hbm=hbm,
                note="the SA1 sampler is a chain of M-1 dependent picks on one CU per cloud: "
                     "its bound is latency (floor from tools/ubench/pick_floor.hip, "
                     "roofline.latency); the HBM figures (roofline.hbm) are structurally low"),
            "host": host_geom or None,
            "step_hbm": {"algorithmic_bytes": step_bytes,
                         "achieved_GBps": step_bytes * world / (elapsed / args.steps) / 1e9,
                         "frac": step_bytes * world / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBPS},
            "checksum": float(sums.sum().item()),
            "primed_steps": post.get("primed_steps"),
            "primed_note": "before the warm-up steps, every buffer set's step ran once and was "
                           "waited for (stack.Pipeline.prime): each set's first plan launch is "
                           "then outside the timed region",
            "verified": post.get("verified"),
            "verify": post.get("verify"),
            "fault_status": post.get("fault_status"),
            "latency_ms_per_batch": post.get("latency_ms_per_batch"),
            "latency_ms_per_batch_min": post.get("latency_ms_per_batch_min"),
            "latency_note": "one B-cloud step enqueued and joined alone (no pipelining), host "
                            f"clock, median of {args.latency_reps}, max over ranks",
        }
        if e2e is not None:
            result["e2e"] = e2e
        if args.diag_only:
            result["diagnostic"] = f"only the {args.diag_only} of each step ran: not a benchmark result"
        if world == 1 and not args.model:
            try:  # (outside the timed region, after it)
                result["roofline"]["hbm"]["copy_peak_measured"] = copy_peak(dev)
            except Exception as e:  # a reported figure, never the product
                log(f"copy peak failed: {e!r}")
        if world == 1 and not args.no_cpu_baseline and not args.model:
            try:
                result["cpu_baseline"] = cpu_baseline(args.config, B, args.cpu_seconds,
                                                      args.cpu_threads or _cpu_share())
                cb = result["cpu_baseline"]
                cb["cfg1"] = cfg1_leg(dev)
                # vs_baseline stays null (BASELINE.md publishes no number for this metric);
                # the GPU/CPU ratios against the measured and extrapolated CPU rates:
                cb["gpu_over_cpu"] = {"1core": value / cb["value_1core"],
                                      f"{cb['threads']}threads": value / cb["value_threads"],
                                      "all_cores_extrapolated":
                                          value / cb["value_all_cores_extrapolated"],
                                      "all_cores_at_measured_efficiency":
                                          value / cb["value_all_cores_at_measured_efficiency"]}
            except Exception as e:  # the baseline is reported, never the product
                log(f"cpu baseline failed: {e!r}")
                result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
