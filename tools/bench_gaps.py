#!/usr/bin/env python3
"""Dependency-latency probe (run under rocprofv3 --kernel-trace): kernel A (an FPS launch,
~60 us) followed by kernel B (a tiny gather) under different orderings; the trace's
timestamps give the GPU-side gap from A's end to B's start for each case.
Cases (each repeated 5x, separated by a sync):
  same      A; B on one stream
  event     A; timing-event record; B on one stream
  waitidle  A; wait on an idle other stream; B
  cross     A on s1; B on s2 after s2.wait_event(A's event)
  graph     graph(A) replay; graph(B) replay on one stream
Labelled by B's grid size (case index + 1 blocks)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    L = pkg.lib()
    dev = torch.device("cuda:0")
    x = torch.from_numpy(pkg.synth.batch(range(16), 8192, "scannet")[0]).to(dev)
    idx = torch.empty((16, 64), dtype=torch.int32, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def A():
        L.pn2_fps(x.data_ptr(), 16, 8192, 64, idx.data_ptr(), torch.cuda.current_stream().cuda_stream)

    def B(case):  # gather of (case+1) x 256 points: the grid size labels the case in the trace
        m = 256 * (case + 1)
        gi = torch.zeros((1, m), dtype=torch.int32, device=dev)
        out = torch.empty((1, m, 3), device=dev)
        L.pn2_gather_point(x.data_ptr(), gi.data_ptr(), 1, 8192, m, out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)

    gA, gB = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    gi5 = torch.zeros((1, 256 * 5), dtype=torch.int32, device=dev)
    out5 = torch.empty((1, 256 * 5, 3), device=dev)
    A(); torch.cuda.synchronize()
    with torch.cuda.graph(gA):
        A()
    with torch.cuda.graph(gB):
        L.pn2_gather_point(x.data_ptr(), gi5.data_ptr(), 1, 8192, 256 * 5, out5.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    for rep in range(5):
        A(); B(0); torch.cuda.synchronize()
        A(); e = torch.cuda.Event(enable_timing=True); e.record(); B(1); torch.cuda.synchronize()
        A(); torch.cuda.current_stream().wait_stream(s2); B(2); torch.cuda.synchronize()
        with torch.cuda.stream(s1):
            A(); ev = torch.cuda.Event(); ev.record(s1)
        s2.wait_event(ev)
        with torch.cuda.stream(s2):
            B(3)
        torch.cuda.synchronize()
        gA.replay(); gB.replay(); torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
