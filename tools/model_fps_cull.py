#!/usr/bin/env python3
"""numpy model of the culled hot-set sampler schedule (fps_cull): how many
refreshes a threshold-selected hot set of K points needs for the SA1 crops, and what fraction
of the (cell, centre) distance updates a box test skips when the cold points are Morton-sorted
into cells of C points. The picks are checked against a brute-force exact FPS (same fp32
arithmetic and tie order as tf_sampling_g.cu:105-170).

    python tools/model_fps_cull.py [--clouds 2] [--K 128] [--cells 64,256,512]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
INIT = np.float32(1e38)


def d2(p, c):
    d = (p - c).astype(np.float32)
    return ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)


def key(k):
    return (k % 512) * 65536 + k // 512


def fps_exact(x, M):
    n = len(x)
    t = np.full(n, INIT, np.float32)
    keys = key(np.arange(n))
    out = [0]
    for _ in range(M - 1):
        t = np.minimum(t, d2(x, x[out[-1]]))
        m = t.max()
        cand = np.flatnonzero(t == m)
        out.append(int(cand[np.argmin(keys[cand])]))
    return np.array(out)


def morton(x, bits=10):
    lo, hi = x.min(0), x.max(0)
    q = np.clip(((x - lo) / np.maximum(hi - lo, 1e-12) * (2 ** bits - 1)).astype(np.int64), 0,
                2 ** bits - 1)
    code = np.zeros(len(x), np.int64)
    for b in range(bits):
        for a in range(3):
            code |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return code


def box_lb(lo, hi, c):
    g = np.maximum(np.maximum((lo - c).astype(np.float32), (c - hi).astype(np.float32)),
                   np.float32(0))
    return ((g[..., 0] * g[..., 0] + g[..., 1] * g[..., 1]) + g[..., 2] * g[..., 2]).astype(
        np.float32)


def simulate(x, M, K, C, fracs, ref_prev=False):
    """ref_prev: thresholds are fractions of the previous round's threshold (or of the stall's
    value) instead of the exact maximum, so each cold wave can count before the round's barrier"""
    n = len(x)
    order = np.argsort(morton(x), kind="stable")
    ncell = (n + C - 1) // C
    cell_of = np.empty(n, np.int64)
    cell_of[order] = np.arange(n) // C
    lo = np.stack([x[cell_of == c].min(0) for c in range(ncell)])
    hi = np.stack([x[cell_of == c].max(0) for c in range(ncell)])
    members = [np.flatnonzero(cell_of == c) for c in range(ncell)]
    keys = key(np.arange(n))
    t = np.full(n, INIT, np.float32)
    tmax = np.full(ncell, INIT, np.float32)
    picks, pending = [0], [0]
    st = dict(refresh=0, stall=0, pairs=0, pairs_full=0, hot_picks=0)
    ref = np.float32(3e38)
    while len(picks) < M:
        st["refresh"] += 1
        for c in pending:  # cold pass with the box test against the stale cell maxima
            lb = box_lb(lo, hi, x[c])
            st["pairs_full"] += ncell
            for ci in np.flatnonzero(lb < tmax):
                st["pairs"] += 1
                m = members[ci]
                t[m] = np.minimum(t[m], d2(x[m], x[c]))
        pending = []
        tmax = np.array([t[m].max() for m in members], np.float32)
        top = t.max()
        base = ref if ref_prev else top
        tau = None
        for f in fracs:  # smallest threshold whose hot set fits
            cand = np.float32(base * np.float32(f))
            if cand < top and np.count_nonzero(t > cand) <= K:
                tau = cand
                break
        if tau is None:  # stalled: one exact block argmax
            st["stall"] += 1
            cand = np.flatnonzero(t == top)
            p = int(cand[np.argmin(keys[cand])])
            picks.append(p)
            pending.append(p)
            ref = top
            continue
        ref = tau
        H = np.flatnonzero(t > tau)
        hv = t[H].copy()
        while len(picks) < M:
            m = hv.max()
            if not m > tau:
                break
            cand = np.flatnonzero(hv == m)
            p = int(H[cand[np.argmin(keys[H[cand]])]])
            picks.append(p)
            pending.append(p)
            st["hot_picks"] += 1
            hv = np.minimum(hv, d2(x[H], x[p]))
    st["culled_frac"] = 1 - st["pairs"] / max(st["pairs_full"], 1)
    return np.array(picks), st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clouds", type=int, default=2)
    ap.add_argument("--N", type=int, default=8192)
    ap.add_argument("--M", type=int, default=1024)
    ap.add_argument("--K", default="128")
    ap.add_argument("--cells", default="64,256,512")
    ap.add_argument("--kind", default="scannet")
    ap.add_argument("--ref-prev", action="store_true")
    ap.add_argument("--fracs", default="0.5,0.7,0.8,0.85,0.9,0.93,0.95,0.97,0.98,0.99,0.995")
    a = ap.parse_args()
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    fr = [float(v) for v in a.fracs.split(",")]
    for cid in range(a.clouds):
        x = pkg.synth.batch([cid], a.N, a.kind)[0][0]
        ref = fps_exact(x, a.M)
        for K in [int(v) for v in a.K.split(",")]:
            for C in [int(v) for v in a.cells.split(",")]:
                p, st = simulate(x, a.M, K, C, fr, a.ref_prev)
                st.update(cloud=cid, K=K, C=C, exact=bool(np.array_equal(p, ref)))
                print(json.dumps(st), flush=True)


if __name__ == "__main__":
    main()
