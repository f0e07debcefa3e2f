"""PCIe device-to-host bandwidth into pinned host memory (diagnostic)."""
import time
import torch
n = 4 << 30
d = torch.empty(n, dtype=torch.uint8, device="cuda")
d.fill_(1)
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
for chunk in (64 << 20, 512 << 20, n):
    torch.cuda.synchronize()
    t = time.time()
    for o in range(0, n, chunk):
        h[o:o + chunk].copy_(d[o:o + chunk], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.time() - t
    print("D2H pinned chunk %d MB: %.1f GB/s" % (chunk >> 20, n / dt / 1e9), flush=True)
hp = torch.empty(n, dtype=torch.uint8)
torch.cuda.synchronize()
t = time.time()
hp.copy_(d)
torch.cuda.synchronize()
print("D2H pageable: %.1f GB/s" % (n / (time.time() - t) / 1e9), flush=True)
