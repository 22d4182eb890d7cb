#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the burst fold's 64 MiB launches of one call alternated
between two streams, so that one launch's write burst and drain overlap the
next launch's reads (the pieces of a call write disjoint outputs).  Against the
same launches on one stream.  8 local sources, double sum; torch events around
the whole call (fork and join included), median of 9 calls.

    python tools/lab/burst_overlap_probe.py [MiB per source ...]     (default 128 256 512)
"""
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
POOL = 5 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1e-3, 1e-3)
base = pool.data_ptr()
VP = ctypes.c_void_p
PIECE = 64 << 20
K = 8
main = torch.cuda.current_stream()
side = [torch.cuda.Stream(), torch.cuda.Stream()]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
fork = torch.cuda.Event()
joins = [torch.cuda.Event(), torch.cuda.Event()]


def pieces(b0, size):
    for off in range(0, size, PIECE):
        srcs = (VP * K)(*[b0 + size * j + off for j in range(K)])
        yield b0 + K * size + off, srcs


def one_stream(b0, size):
    for out, srcs in pieces(b0, size):
        assert lib.pgk_reduce_multi(out, srcs, K, PIECE // 8, 1, 0, main.cuda_stream) == 0


def two_streams(b0, size):
    fork.record(main)
    for s in side:
        s.wait_event(fork)
    for i, (out, srcs) in enumerate(pieces(b0, size)):
        assert lib.pgk_reduce_multi(out, srcs, K, PIECE // 8, 1, 0, side[i & 1].cuda_stream) == 0
    for s, j in zip(side, joins):
        j.record(s)
        main.wait_event(j)


def check(size):
    n = size // 8
    two_streams(base, size)
    torch.cuda.synchronize()
    acc = pool[:n].clone()
    for j in range(1, K):
        acc += pool[j * n:(j + 1) * n]
    assert torch.equal(acc, pool[K * n:(K + 1) * n])


check(128 << 20)
print("two-stream call checked against torch", flush=True)
for mib in [int(a) for a in sys.argv[1:]] or [128, 256, 512]:
    size = mib << 20
    span = (K + 1) * size
    sets = max(1, POOL // span)
    res = {}
    for name, fn in (("one stream", one_stream), ("two streams", two_streams), ("one stream", one_stream),
                     ("two streams", two_streams)):
        ts = []
        for i in range(10):
            b0 = base + span * (i % sets)
            torch.cuda.synchronize()
            e0.record(main)
            fn(b0, size)
            e1.record(main)
            torch.cuda.synchronize()
            if i:
                ts.append(e0.elapsed_time(e1) * 1e3)
        res.setdefault(name, []).append(statistics.median(ts))
    for name, v in res.items():
        t = min(v)
        print(f"  8 x {mib:4d} MiB  {name:12s} {t:9.2f} us  {(K + 1) * size / t / 8e4:5.1f}%", flush=True)
