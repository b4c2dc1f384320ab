#!/usr/bin/env python3
"""FPS golden vectors from the reference kernel TEXT run on CPU threads (no GPU compiler).

oracle/_ref/libref_fps_emul.so is tf_sampling_g.cu:105-170 (farthestpointsamplingKernel)
compiled by g++ under a one-block CUDA emulation: 512 std::threads, `__syncthreads()` =
std::barrier, `__shared__` = function statics, one barrier added after :165 to close the
write-after-read race on dists_i (oracle/fps_emul_head.h, oracle/Makefile target `ref`,
SURVEY.md §0.4 and §8(c)). Built only in the container that has /root/reference.

    python tests/golden/make_golden_fps_emul.py

1. Writes fpsemul_*.npz (op farthest_point_sample: xyz, idx, new_xyz = xyz[idx]) for the
   tie-heavy integer lattice, an all-duplicate cloud and one SA1 ScanNet crop (8192 -> 1024).
   tests/test_oracle_golden.py checks the oracle against them, tests/test_gpu_parity.py the
   HIP sampler.
2. Runs the emulation on the input of every fps_*.npz (those came from the reference CUDA
   compiled by hipcc and run on gfx950, make_golden_gpu.py) and asserts the same indices;
   the comparison is recorded in fps_emul_check.json (sha256 of each idx array).
"""
import ctypes
import glob
import hashlib
import importlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "oracle", "_ref", "libref_fps_emul.so")
REF = "tf_sampling_g.cu:105-170 (farthestpointsamplingKernel) on 512 CPU threads, std::barrier " \
      "for __syncthreads, one barrier added after :165 (oracle/fps_emul_head.h)"


def emul_fps(x, m, threads=512):
    lib = ctypes.CDLL(LIB)
    x = np.ascontiguousarray(x, np.float32)
    B, N, _ = x.shape
    idx = np.zeros((B, m), np.int32)
    rc = lib.pn2emul_fps(B, N, m, threads, x.ctypes.data_as(ctypes.c_void_p),
                         idx.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
    return idx


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def save(name, x, m, inputs):
    t = time.time()
    idx = emul_fps(x, m)
    new_xyz = np.take_along_axis(x, idx[..., None].astype(np.int64), axis=1)
    meta = {"op": "farthest_point_sample", "npoint": m, "inputs": inputs, "ref": REF}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), xyz=x, idx=idx, new_xyz=new_xyz,
                        meta=np.array(json.dumps(meta)))
    print(f"wrote {name} {x.shape} -> {m} in {time.time() - t:.1f} s", flush=True)


def main():
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    rng = np.random.default_rng(2024)
    g = np.stack(np.meshgrid(*[np.arange(12)] * 3, indexing="ij"), -1).reshape(-1, 3)
    save("fpsemul_lattice_ties", g[rng.integers(0, len(g), 2048)][None].astype(np.float32), 384,
         "12^3 integer lattice, 2048 draws -> 384 (massive exact ties)")
    save("fpsemul_all_dup", np.tile(np.float32([[0.5, 0.25, 0.125]]), (1200, 1))[None], 24,
         "one point repeated 1200 times -> 24 (every distance ties at 0)")
    save("fpsemul_scannet_sa1", pkg.synth.batch([11], 8192, "scannet")[0], 1024,
         "SA1 ScanNet crop (synth cloud id 11, 8192 drawn with replacement) -> 1024")
    check = {}
    for path in sorted(glob.glob(os.path.join(HERE, "fps_*.npz"))):
        z = np.load(path, allow_pickle=False)
        x, want = z["xyz"], z["idx"]
        got = emul_fps(x, want.shape[1])
        name = os.path.basename(path)[:-4]
        check[name] = {"shape": list(x.shape), "npoint": int(want.shape[1]),
                       "equal": bool(np.array_equal(got, want)), "idx_sha256": sha(got)}
        print(name, check[name], flush=True)
        assert check[name]["equal"], f"{name}: emulation differs from the gfx950 reference run"
    with open(os.path.join(HERE, "fps_emul_check.json"), "w") as f:
        json.dump({"emulation": REF, "vs": "fps_*.npz (reference CUDA on gfx950)",
                   "cases": check}, f, indent=1)


if __name__ == "__main__":
    main()
