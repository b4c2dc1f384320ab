import ctypes, importlib, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
from oracle import oracle as O
L = pkg.lib()
L.pn2_fps_tune.restype = ctypes.c_int
L.pn2_fps_tune.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0"); st = torch.cuda.current_stream().cuda_stream
rng = np.random.default_rng(0)
g = np.stack(np.meshgrid(*[np.arange(16)] * 3, indexing="ij"), -1).reshape(-1, 3)
for N, M in [(64, 16), (256, 64), (1024, 256), (8192, 1024)]:
    for name, x in [("grid", np.stack([g[rng.integers(0, len(g), N)] for _ in range(4)]).astype(np.float32)),
                    ("uniform", pkg.synth.batch(range(4), N, "uniform")[0]),
                    ("scannet", pkg.synth.batch(range(4), N, "scannet")[0])]:
        x = np.ascontiguousarray(x); xt = torch.from_numpy(x).to(dev)
        ref = O.fps(x, M)
        res = {}
        for (v, bl, pp) in [(1, 64, 1), (2, 64, 1), (1, 256, 4), (2, 256, 4), (31, 256, 4), (32, 256, 4), (34, 256, 4), (34, 512, 16), (32, 512, 16), (2, 512, 16)]:
            if bl * pp < N or (bl*pp > 4*N and v < 30) : continue
            out = torch.zeros((4, M), dtype=torch.int32, device=dev)
            rc = L.pn2_fps_tune(xt.data_ptr(), 4, N, M, out.data_ptr(), None, v, bl, pp, st)
            torch.cuda.synchronize()
            o = out.cpu().numpy()
            bad = (o != ref)
            res[(v, bl, pp)] = (rc, int(bad.sum()), None if not bad.any() else (np.argwhere(bad)[0].tolist(), o[bad][:3].tolist(), ref[bad][:3].tolist()))
        print(N, name, res, flush=True)
