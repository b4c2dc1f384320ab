#!/usr/bin/env python3
"""CPU model of the grid three_nn's wave box (interp.hip grid_nn3_wave) at FP4: per chunk of
consecutive unknowns (the SA1 grid's order; 16 = a wave of quads), the known points of the
cell box around the chunk's bounding box grown by a margin (in cell edges of the automatic
grid), and the share of unknowns whose third-nearest distance that box does not certify (they
fall back to the shell walk). numpy only (its own FPS), ScanNet-like synthetic clouds.

    python tools/sim_nn_box.py [--clouds 2] [--chunk 16] [--margins 0.45,0.6,0.8]"""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fps(x, m):
    idx = np.zeros(m, np.int64)
    d = np.full(len(x), np.inf)
    for i in range(1, m):
        d = np.minimum(d, ((x - x[idx[i - 1]]) ** 2).sum(1))
        idx[i] = int(np.argmax(d))
    return idx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clouds", type=int, default=2)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--m", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=16)
    ap.add_argument("--margins", default="0.45,0.6,0.8")
    a = ap.parse_args()
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    x = pkg.synth.batch(range(a.clouds), a.n, "scannet")[0]
    for b in range(a.clouds):
        X = x[b].astype(np.float64)
        K = X[fps(X, a.m)]
        lo, hi = K.min(0), K.max(0)
        e = (np.prod(hi - lo) / (a.m / 2)) ** (1 / 3)  # grid.h's automatic edge (~2 per cell)
        dims = (np.floor((hi - lo) / e) + 1).astype(int)
        while dims.prod() > max(a.m, 64):
            e *= 1.25
            dims = (np.floor((hi - lo) / e) + 1).astype(int)
        kc = np.clip(np.floor((K - lo) / e), 0, dims - 1).astype(int)
        ulo = X.min(0)
        ud = (np.floor((X.max(0) - ulo) / 0.1) + 1).astype(int)
        uc = np.clip(np.floor((X - ulo) / 0.1), 0, ud - 1).astype(int)
        order = np.argsort((uc[:, 2] * ud[1] + uc[:, 1]) * ud[0] + uc[:, 0], kind="stable")
        for mf in (float(v) for v in a.margins.split(",")):
            mg = mf * e
            cands, fails = [], 0
            for c0 in range(0, a.n, a.chunk):
                U = X[order[c0:c0 + a.chunk]]
                c_lo = np.clip(np.floor((U.min(0) - mg - lo) / e), 0, dims - 1).astype(int)
                c_hi = np.clip(np.floor((U.max(0) + mg - lo) / e), 0, dims - 1).astype(int)
                inbox = np.all((kc >= c_lo) & (kc <= c_hi), 1)
                cands.append(int(inbox.sum()))
                blo, bhi = lo + c_lo * e, lo + (c_hi + 1) * e
                gap = np.full(len(U), np.inf)
                for ax in range(3):
                    if c_lo[ax] > 0:
                        gap = np.minimum(gap, U[:, ax] - blo[ax])
                    if c_hi[ax] < dims[ax] - 1:
                        gap = np.minimum(gap, bhi[ax] - U[:, ax])
                Kc = K[inbox]
                d3 = (np.sort(((U[:, None, :] - Kc[None]) ** 2).sum(-1), 1)[:, 2] if len(Kc) >= 3
                      else np.full(len(U), np.inf))
                fails += int(np.sum(~(d3 < gap ** 2)))
            c = np.array(cands)
            print(f"cloud {b}: edge {e:.3f}, {dims.prod()} cells, chunk {a.chunk}, margin "
                  f"{mf} edges: candidates per unknown mean {c.mean():.0f} median "
                  f"{np.median(c):.0f} p90 {np.percentile(c, 90):.0f} max {c.max()}; "
                  f"fall back {fails / a.n:.5f}")


if __name__ == "__main__":
    main()
