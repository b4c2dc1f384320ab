import os, torch
print("env GPU_MAX_HW_QUEUES =", os.environ.get("GPU_MAX_HW_QUEUES"))
ss = [torch.cuda.Stream() for _ in range(10)]
x = torch.ones(1 << 20, device="cuda")
for i, s in enumerate(ss):
    with torch.cuda.stream(s):
        for _ in range(3):
            x.mul_(1.0001)
torch.cuda.synchronize()
print("ok")
