#!/usr/bin/env python3
"""EXPERIMENTS ONLY: does the relative placement of src vs dst (address offset
between the two streams) or a persistent 2-blocks/CU grid change the
256 MiB double-sum rate?  Interleaved rounds, kernel-stamped events."""
import ctypes
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

lib = pgamd.load()
torch.cuda.set_device(0)
N = 1 << 25
B = N * 8
pool = torch.empty(6 * B + (64 << 20), dtype=torch.uint8, device="cuda")
pool.view(torch.float64)[: (6 * B) // 8].uniform_(-1, 1)
base = pool.data_ptr()
sh = torch.cuda.current_stream().cuda_stream
ev = [(ctypes.c_void_p(), ctypes.c_void_p()) for _ in range(10)]
for a, b in ev:
    lib.pgk_event_create(ctypes.byref(a))
    lib.pgk_event_create(ctypes.byref(b))
variants = [("offset 0", 0, 0), ("offset 256 B", 256, 0), ("offset 4 KiB", 4096, 0), ("offset 64 KiB", 65536, 0),
            ("offset 1 MiB+4 KiB", (1 << 20) + 4096, 0), ("offset 32 MiB", 32 << 20, 0),
            ("grid 2/CU (persistent)", 0, 2), ("grid 4/CU", 0, 4)]
res = {v[0]: [] for v in variants}
k = 0
for rnd in range(10):
    for name, off, bpc in variants:
        lib.pgk_tune(bpc, 1)
        for i, (a, b) in enumerate(ev):
            slot = (k % 2) * 3 * B
            k += 1
            d = base + slot
            s = base + slot + B + (16 << 20) + off      # src after dst, 16 MiB gap + offset
            lib.pgk_reduce_timed(d, s, N, 1, 0, sh, a, b)
        torch.cuda.synchronize()
        for a, b in ev[2:]:
            ms = ctypes.c_float()
            lib.pgk_event_elapsed_ms(a, b, ctypes.byref(ms))
            res[name].append(ms.value * 1e3)
lib.pgk_tune(0, 1)
for name, v in res.items():
    med = statistics.median(v)
    print(f"{name:24s} {3 * B / med / 1e3:8.1f} GB/s  median {med:7.2f} us  min {min(v):7.2f}")
