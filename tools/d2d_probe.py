"""Device-to-device copy rate (design tool, GPU box): the practical ceiling for a kernel that
reads and writes each byte once (the incompressible paths), against the 8 TB/s HBM peak."""
import torch

n = 655360000
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty(n, dtype=torch.uint8, device="cuda")
a.fill_(1)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(10):
    s.record(); b.copy_(a); e.record(); e.synchronize(); ts.append(s.elapsed_time(e))
ms = min(ts)
print("D2D copy of %d B: %.3f ms, %.2f TB/s (read + write bytes)" % (n, ms, 2 * n / (ms * 1e-3) / 1e12))
