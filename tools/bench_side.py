#!/usr/bin/env python3
"""Standalone cost of every task of one pipelined step (stack.Step / GraphStep segments) at a
BASELINE batch: each launch segment's tasks (stack.Step.segments(): the side segments and the
direct sampler launches) called `inner` times inside one captured hipGraph, replayed alone on
one stream (nothing else on the GPU), HIP events around it, median of `reps`. Per task: us per launch,
its algorithmic bytes (each input read once, each output written once) and
the rate over them. The sum over the side tasks is the side work's full-chip time per step.

    python tools/bench_side.py [--config cfg2|cfg3|cfg5] [--json out.json]
"""
import argparse
import importlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def task_bytes(S, config, B):
    """Algorithmic bytes per task name of the SSG / MSG step (B clouds)."""
    N, kind, with_feat, attn = S.CONFIGS[config]
    out = {}
    if kind == "ssg":
        n_in, c_in = N, (6 if with_feat else 0)
        levels, chans = [N], [c_in]
        for i, (M, _, ns, c_out) in enumerate(S.SSG_SA):
            grp = n_in * (3 + c_in) * 4 + M * 12 + M * ns * 4 + M * 4 + M * ns * (3 + c_in) * 4
            out[f"sa{i + 1}"] = grp
            if attn:
                out["att"] = out.get("att", 0) + M * c_out * 4 + 2 * M * ns * c_out * 4 \
                    + M * c_out * 4
            levels.append(M)
            chans.append(c_out)
            n_in, c_in = M, c_out
        out["sa234"] = out.pop("sa2") + out.pop("sa3") + out.pop("sa4")
        out["grid1"] = N * 12 + N * 16
        c2 = S.SSG_SA[3][3]
        fp = {}
        for k in range(4):
            lvl = 3 - k
            n, m, c1 = levels[lvl], levels[lvl + 1], chans[lvl]
            fp[k] = n * 12 + m * 12 + m * c2 * 4 + n * c1 * 4 + n * (c1 + c2) * 4
            c2 = S.SSG_FP_OUT[k]
        out["fp4"] = fp[3]
        out["fp123"] = fp[0] + fp[1] + fp[2]
        out["fps1"] = N * 12 + S.SSG_SA[0][0] * 16
        out["fps234"] = sum(a * 12 + b[0] * 16 for a, b in
                            zip([s[0] for s in S.SSG_SA[:3]], S.SSG_SA[1:]))
    else:
        n_in, c_in = N, 0
        for i, (M, radii, nss, couts) in enumerate(S.MSG_SA):
            tot = sum(n_in * (3 + c_in) * 4 + M * 12 + M * ns * 4 + M * 4 + M * ns * (3 + c_in) * 4
                      for ns in nss)
            out[f"sa{i + 1}"] = tot
            out[f"fps{i + 1}"] = n_in * 12 + M * 16
            n_in, c_in = M, sum(couts)
        out["grid1"] = N * 12 + N * 16
    return {k: v * B for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--inner", type=int, default=10)
    ap.add_argument("--json", default=None)
    ap.add_argument("--fp4-known-grid", choices=["lane", "sampler", "off"], default=None,
                    help="stack.FP4_KNOWN_GRID (A/B)")
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    S = pkg.stack
    S.FP4_KNOWN_GRID = args.fp4_known_grid
    dev = torch.device("cuda:0")
    B = 8 if args.config == "cfg5" else 16
    inp = S.make_inputs(args.config, list(range(B)), dev)
    gs = S.GraphStep(inp, segments=True, chain_lane=-1 if args.config != "cfg5" else 0,
                     layout="b" if args.config == "cfg2" else "a")
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()

    def timeit(fn):
        # `inner` calls captured into one hipGraph and replayed: GPU time only (a launch's host
        # cost is more than some of these kernels take)
        with torch.cuda.stream(st):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for _ in range(args.inner):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                g.replay()
                b.record(st)
                b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3 / args.inner)
        return statistics.median(ts)

    by = task_bytes(S, args.config, B)
    res = {}
    for seg in gs.step.segments():
        key = S.Step.segment_key(seg)
        us = timeit(lambda seg=seg: [t.fn() for t in seg])
        b = sum(by.get(t.name, 0) for t in seg)
        res[key] = {"us": round(us, 2), "bytes": b,
                    "TBps": round(b / us / 1e6, 3) if b else None}
    side = [k for k, v in res.items() if not k.startswith("fps")]
    res["side_sum_us"] = round(sum(res[k]["us"] for k in side), 2)
    res["config"] = args.config
    print(json.dumps(res))
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
