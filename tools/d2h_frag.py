"""Device-to-host copy rate of a fresh device buffer at process start and after device-memory churn
(diagnostic, GPU): does a buffer allocated late in a process (fragmented VRAM) copy out slower?"""
import time
import torch

GB = 1 << 30
h = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True)


def rate(x, reps=8):
    torch.cuda.synchronize()
    t0 = time.time()
    for i in range(reps):
        h.copy_(x[(i % 16) * (256 << 20):(i % 16 + 1) * (256 << 20)], non_blocking=True)
    torch.cuda.synchronize()
    return reps * (256 << 20) / (time.time() - t0) / 1e9


a = torch.empty(4 * GB, dtype=torch.uint8, device="cuda")
a.fill_(1)
print("fresh 4 GB buffer: %.1f GB/s" % rate(a), flush=True)
# churn: many buffers of mixed sizes allocated, half freed, caches emptied, repeated
keep = []
for r in range(6):
    bufs = [torch.empty(((k * 7919) % 509 + 1) << 20, dtype=torch.uint8, device="cuda") for k in range(300)]
    keep += bufs[::2]
    del bufs
    torch.cuda.empty_cache()
b = torch.empty(4 * GB, dtype=torch.uint8, device="cuda")
b.fill_(2)
print("after churn (%d live blocks, %.1f GB): new 4 GB buffer %.1f GB/s, first buffer %.1f GB/s"
      % (len(keep), sum(t.numel() for t in keep) / 1e9, rate(b), rate(a)), flush=True)
del keep
torch.cuda.empty_cache()
c = torch.empty(4 * GB, dtype=torch.uint8, device="cuda")
c.fill_(3)
print("churn freed: new 4 GB buffer %.1f GB/s" % rate(c), flush=True)
