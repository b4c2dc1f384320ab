#!/usr/bin/env python3
"""Micro-benchmark of the attention reduction (pn2_attn_reduce, attn_reduce_kernel<32>) at the
cfg3 SA shapes (B = 16, ns = 32; M x C = 1024 x 64, 256 x 128, 64 x 256, 16 x 512).
Back-to-back launches between HIP events, median of 20; GB/s over Q + K + V + out."""
import importlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    dev = torch.device("cuda:0")
    L = pkg.lib()
    st = torch.cuda.current_stream().cuda_stream

    def timeit(fn, reps=20, inner=20):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(inner):
                fn()
            b.record(); b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / inner)
        return statistics.median(ts)

    B, ns = 16, 32
    res = {}
    for name, M, C in (("sa1", 1024, 64), ("sa2", 256, 128), ("sa3", 64, 256), ("sa4", 16, 512)):
        Q = torch.rand((B, M, C), device=dev) - 0.5
        K = torch.rand((B, M, ns, C), device=dev) - 0.5
        V = torch.rand((B, M, ns, C), device=dev) - 0.5
        out = torch.empty((B, M, C), device=dev)

        def run():
            assert L.pn2_attn_reduce(Q.data_ptr(), K.data_ptr(), V.data_ptr(), B, M, ns, C,
                                     out.data_ptr(), st) == 0
        us = timeit(run)
        nbytes = (Q.numel() + K.numel() + V.numel() + out.numel()) * 4
        res[name] = {"us": round(us, 1), "GBps": round(nbytes / us / 1e3, 0)}
    # the four layers in one launch (pn2_attn_reduce_layers, what the cfg3 step runs)
    import ctypes
    bufs, tot = [], 0
    arr = (pkg._lib.AttnLayer * 4)()
    for i, (M, C) in enumerate(((1024, 64), (256, 128), (64, 256), (16, 512))):
        Q = torch.rand((B, M, C), device=dev) - 0.5
        K = torch.rand((B, M, ns, C), device=dev) - 0.5
        V = torch.rand((B, M, ns, C), device=dev) - 0.5
        out = torch.empty((B, M, C), device=dev)
        bufs += [Q, K, V, out]
        arr[i] = pkg._lib.AttnLayer(Q.data_ptr(), K.data_ptr(), V.data_ptr(), M, ns, C,
                                    out.data_ptr())
        tot += (Q.numel() + K.numel() + V.numel() + out.numel()) * 4
    us = timeit(lambda: L.pn2_attn_reduce_layers(ctypes.addressof(arr), 4, B, st))
    res["layers4"] = {"us": round(us, 1), "GBps": round(tot / us / 1e3, 0)}
    res["lib"] = os.path.basename(os.environ.get("PN2HIP_LIB") or "libpn2hip.so")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
