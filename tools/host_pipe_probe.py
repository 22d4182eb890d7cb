#!/usr/bin/env python3
"""EXPERIMENTS ONLY: pgx_reduce_host piece-size sweep (256 MiB double sum,
pageable and pinned host operands); PCIe GB/s counts 3*n*8 bytes."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

lib = pgamd.load()
torch.cuda.set_device(0)
n = 1 << 25
for kind in ("pageable", "pinned"):
    d = torch.rand(n, dtype=torch.float64)
    s = torch.rand(n, dtype=torch.float64)
    if kind == "pinned":
        d, s = d.pin_memory(), s.pin_memory()
    for piece_mib in (2, 4, 8, 16, 32, 64, 256):
        pc = piece_mib << 20
        pgamd.check(lib.pgx_reduce_host(d.data_ptr(), s.data_ptr(), n, 1, 0, pc), "warm")
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            pgamd.check(lib.pgx_reduce_host(d.data_ptr(), s.data_ptr(), n, 1, 0, pc), "run")
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        print(f"{kind:9s} piece {piece_mib:4d} MiB: {t * 1e3:7.2f} ms  {3 * n * 8 / t / 1e9:6.1f} GB/s", flush=True)
# one-direction references: plain hipMemcpy of 256 MiB each way
d = torch.rand(n, dtype=torch.float64)
g = torch.empty(n, dtype=torch.float64, device="cuda")
for name, fn in (("H2D 256 MiB pageable", lambda: g.copy_(d)), ("D2H 256 MiB pageable", lambda: d.copy_(g))):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / 5
    print(f"{name}: {t * 1e3:.2f} ms  {n * 8 / t / 1e9:.1f} GB/s", flush=True)
