#!/usr/bin/env python3
"""EXPERIMENTS ONLY: do H2D and D2H copies overlap (PCIe full duplex)?
256 MiB each way, pinned host memory, separate streams; alone vs together."""
import time

import torch

torch.cuda.set_device(0)
n = 1 << 25
h1 = torch.rand(n, dtype=torch.float64).pin_memory()
h2 = torch.empty(n, dtype=torch.float64).pin_memory()
g1 = torch.empty(n, dtype=torch.float64, device="cuda")
g2 = torch.rand(n, dtype=torch.float64, device="cuda")
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def h2d():
    with torch.cuda.stream(sa):
        g1.copy_(h1, non_blocking=True)


def d2h():
    with torch.cuda.stream(sb):
        h2.copy_(g2, non_blocking=True)


def both():
    h2d()
    d2h()


for name, fn in (("H2D alone", h2d), ("D2H alone", d2h), ("H2D + D2H together", both)):
    t = timed(fn)
    moved = 2 * n * 8 if fn is both else n * 8
    print(f"{name:20s} {t * 1e3:6.2f} ms  {moved / t / 1e9:6.1f} GB/s total", flush=True)
