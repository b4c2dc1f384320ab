#!/usr/bin/env python3
"""Host-side cost of enqueueing one pipelined step (stack.Pipeline.run): for the geometric
step and the whole model, the mean wall time of run() itself, split into the wait for the
buffer set's previous side work and the launches. If the launches alone approach the GPU's
step time, the host, not the GPU, sets the pace.

    python tools/host_overhead.py [--config cfg2] [--steps 40]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--sampler-lanes", type=int, default=1)
    ap.add_argument("--geometry-only", action="store_true")
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    hi = torch.cuda.Stream(device=dev, priority=-1)
    for model in ((False,) if args.geometry_only else (False, True)):
        with torch.cuda.stream(hi if model else torch.cuda.current_stream(dev)):
            inp = pkg.stack.make_inputs(args.config, list(range(16)), dev, model=model)
            pipe = pkg.stack.Pipeline(inp, nsets=3, private_streams=model,
                                      sampler_lanes=1 if model else args.sampler_lanes)
            for _ in range(5):
                pipe.run()
            pipe.join()
            torch.cuda.synchronize()
            wait_s = launch_s = 0.0
            t0 = time.perf_counter()
            for _ in range(args.steps):
                s = pipe.sets[pipe.k % len(pipe.sets)]
                a = time.perf_counter()
                if s.step.ran:
                    s.step.lane_done[1].synchronize()
                b = time.perf_counter()
                pipe.run()
                c = time.perf_counter()
                wait_s += b - a
                launch_s += c - b
            pipe.join()
            torch.cuda.synchronize()
            total = time.perf_counter() - t0
            ntasks = len(pipe.sets[0].step.tasks)
            print(json.dumps({"model": model, "sampler_lanes": 1 if model else args.sampler_lanes,
                              "tasks_per_step": ntasks,
                              "ms_per_step": round(total / args.steps * 1e3, 3),
                              "host_wait_ms": round(wait_s / args.steps * 1e3, 3),
                              "host_launch_ms": round(launch_s / args.steps * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
