#!/usr/bin/env python3
"""EXPERIMENTS ONLY: pgk_reduce_multi (the xgmi transport's and the eager
path's fold) on LOCAL sources: k sources of `size` bytes each, one output;
HBM traffic (k+1) * size per launch.  Interleaved rounds, kernel times from
HIP events around each launch (boundaries included)."""
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
stream = torch.cuda.current_stream()
sh = stream.cuda_stream
size = int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 128 << 20
n = size // 8
pool = torch.empty((9 + 9) * n, dtype=torch.float64, device="cuda").uniform_(-1, 1)   # two sets of 8 srcs + out
for k in (2, 4, 8):
    ts = []
    for rnd in range(10):
        base = pool.data_ptr() + (rnd % 2) * 9 * size
        srcs = (ctypes.c_void_p * k)(*[base + j * size for j in range(k)])
        out = base + 8 * size
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        pgamd.check(lib.pgk_reduce_multi(out, srcs, k, n, 1, 0, sh), "multi")
        b.record(stream)
        torch.cuda.synchronize()
        if rnd >= 2:
            ts.append(a.elapsed_time(b) * 1e3)
    med = statistics.median(ts)
    print(f"k={k}: {med:8.2f} us  {(k + 1) * size / med / 1e3:7.1f} GB/s  ({(k + 1) * size / med / 1e3 / 8000:.1%} of 8 TB/s)",
          flush=True)
