#!/usr/bin/env python3
"""PCIe probe (not product): pinned H2D alone, D2H alone, and both at once on two streams, plus
H2D of 2 buffers on 2 streams -- what bounds the host-inclusive rate on the GPU box."""
import time

import torch


def rate(fn, nbytes, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t) / 1e9


MB = 1 << 20
n = 64 * MB
h1 = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def h2d():
    d1.copy_(h1, non_blocking=True)


def d2h():
    h2.copy_(d2, non_blocking=True)


def both():
    with torch.cuda.stream(s1):
        d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)


def two_h2d():
    with torch.cuda.stream(s1):
        d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2):
        d2.copy_(h2, non_blocking=True)


print({"h2d_GBs": round(rate(h2d, n), 1), "d2h_GBs": round(rate(d2h, n), 1),
       "h2d+d2h_concurrent_GBs": round(rate(both, 2 * n), 1), "2xh2d_concurrent_GBs": round(rate(two_h2d, 2 * n), 1)})
