#!/usr/bin/env python3
"""PCIe ceiling on this box: pinned host <-> HBM copies of 2 GB (torch), one
direction at a time and both at once on two streams."""
import time
import torch

n = 2 << 30
h = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
for _ in range(2):
    d.copy_(h, non_blocking=True)
    h2.copy_(d2, non_blocking=True)
torch.cuda.synchronize()
t = time.perf_counter()
d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
h2d = n / (time.perf_counter() - t) / 1e9
t = time.perf_counter()
h2.copy_(d2, non_blocking=True)
torch.cuda.synchronize()
d2h = n / (time.perf_counter() - t) / 1e9
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
t = time.perf_counter()
with torch.cuda.stream(s1):
    d.copy_(h, non_blocking=True)
with torch.cuda.stream(s2):
    h2.copy_(d2, non_blocking=True)
torch.cuda.synchronize()
both = 2 * n / (time.perf_counter() - t) / 1e9
print(f"pinned H2D {h2d:.1f} GB/s, D2H {d2h:.1f} GB/s, both directions at once {both:.1f} GB/s total")

# host side of the staging: pageable -> pinned copies, 1 and 16 threads
import threading
import numpy as np
src = np.random.default_rng(0).integers(0, 255, size=n, dtype=np.uint8)
dst = h.numpy()
for nt in (1, 4, 16):
    per = n // nt
    def work(i):
        dst[i * per:(i + 1) * per] = src[i * per:(i + 1) * per]
    work(0)
    t = time.perf_counter()
    ths = [threading.Thread(target=work, args=(i,)) for i in range(nt)]
    for x in ths:
        x.start()
    for x in ths:
        x.join()
    print(f"pageable -> pinned memcpy, {nt} threads: {n / (time.perf_counter() - t) / 1e9:.1f} GB/s")
