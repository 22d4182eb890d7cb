#!/usr/bin/env python3
"""EXPERIMENTS ONLY: same process, interleaved rounds -- 256 MiB double-sum
chunks (a) as 4 separately allocated dst/src tensor pairs (bench.py layout),
(b) as blocks of one large allocation (the ring's layout: blocks of a send
buffer), (c) one allocation per operand (4 dst blocks | 4 src blocks)."""
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
sh = torch.cuda.current_stream().cuda_stream
sep_d = [torch.empty(N, dtype=torch.float64, device="cuda").uniform_(-1, 1) for _ in range(4)]
sep_s = [torch.empty(N, dtype=torch.float64, device="cuda").uniform_(-1, 1) for _ in range(4)]
pool = torch.empty(8 * N, dtype=torch.float64, device="cuda").uniform_(-1, 1)     # d0 s0 d1 s1 ...
dpool = torch.empty(4 * N, dtype=torch.float64, device="cuda").uniform_(-1, 1)
spool = torch.empty(4 * N, dtype=torch.float64, device="cuda").uniform_(-1, 1)
g = torch.Generator(device="cuda").manual_seed(1234)
bench_d = [torch.rand(N, dtype=torch.float64, device="cuda", generator=g) * 2 - 1 for _ in range(4)]
bench_s = [torch.rand(N, dtype=torch.float64, device="cuda", generator=g) * 2 - 1 for _ in range(4)]
pool8 = torch.empty(16 * N, dtype=torch.float64, device="cuda").uniform_(-1, 1)           # size-table layout
layouts = {
    "bench.py tensors (rand*2-1)": lambda i: (bench_d[i].data_ptr(), bench_s[i].data_ptr()),
    "4 GiB pool, 8 pairs": lambda i: (pool8.data_ptr() + 2 * (2 * i) * B, pool8.data_ptr() + (4 * i + 1) * B),
    "separate tensors (bench)": lambda i: (sep_d[i].data_ptr(), sep_s[i].data_ptr()),
    "one pool, d/s interleaved": lambda i: (pool.data_ptr() + 2 * i * B, pool.data_ptr() + (2 * i + 1) * B),
    "one pool per operand": lambda i: (dpool.data_ptr() + i * B, spool.data_ptr() + i * B),
}
ev = [(ctypes.c_void_p(), ctypes.c_void_p()) for _ in range(12)]
for a, b in ev:
    lib.pgk_event_create(ctypes.byref(a))
    lib.pgk_event_create(ctypes.byref(b))
res = {k: [] for k in layouts}
for rnd in range(10):
    for name, f in layouts.items():
        for i, (a, b) in enumerate(ev):
            d, s = f(i % 4)
            lib.pgk_reduce_timed(d, s, N, 1, 0, sh, a, b)
        torch.cuda.synchronize()
        for a, b in ev[2:]:
            ms = ctypes.c_float()
            lib.pgk_event_elapsed_ms(a, b, ctypes.byref(ms))
            res[name].append(ms.value * 1e3)
for name, v in res.items():
    med = statistics.median(v)
    print(f"{name:28s} {3 * B / med / 1e3:8.1f} GB/s  median {med:7.2f} us  min {min(v):7.2f}")
print("addresses:", [hex(t.data_ptr()) for t in sep_d + sep_s], hex(pool.data_ptr()))
