import ctypes, os, sys
import torch
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libubench.so"))
out = torch.zeros(4, dtype=torch.int64, device="cuda")
sink = torch.zeros(1024, device="cuda")
assert L.ubench_stamp(ctypes.c_void_p(out.data_ptr())) == 0
print("stamp back-to-back cycles:", out[0].item(), " clock64 back-to-back:", out[1].item())
iters = 2000
for mode, name in [(0, "barrier only"), (1, "+ lds atomic + read"), (2, "+ wave_max_u32"), (3, "+ dependent centre read")]:
    row = []
    for nt in (64, 128, 256, 512, 1024):
        for _ in range(2):
            assert L.ubench_tail(mode, nt, iters, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(sink.data_ptr())) == 0
        row.append(round(out[0].item() / iters, 1))
    print(f"mode {mode} ({name}): cycles/iter for 1,2,4,8,16 waves: {row}")

gidx = torch.zeros(8192, dtype=torch.int32, device="cuda")
for mode, name in [(0, "wave max + write/barrier/read + row16 + ballot"), (1, "+ centre read"), (2, "+ ring selects"), (3, "+ ring flush"), (4, "+ per-iter thread0 store (no ring)")]:
    row = []
    for nt in (64, 128, 256, 512, 1024):
        for _ in range(2):
            assert L.ubench_tail2(mode, nt, iters, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(gidx.data_ptr())) == 0
        row.append(round(out[0].item() / iters, 1))
    print(f"tail2 mode {mode} ({name}): cycles/iter for 1,2,4,8,16 waves: {row}")
