#!/usr/bin/env python3
"""EXPERIMENTS ONLY: is one large reduce slower than the same reduce cut into
several launches?  The size table shows 4 x 256 MiB launches (4 x 122.6 us)
beating one 1 GiB launch (501.6 us).  Here the SAME operands are reduced as
one pgk_reduce launch and as k back-to-back launches of n/k elements each,
bracketed by events on the launch stream, interleaved rounds, rotating over
an 8 GiB pool so every launch streams from HBM.

    python tools/lab/split_probe.py [total MiB per operand ...]   (default 256 512 1024 2048)
    python tools/lab/split_probe.py --shapes [total MiB ...]       one launch in every instantiated shape
                                                                   (is it the block count or the bytes?)
"""
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 8 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
SHAPES = "--shapes" in sys.argv
if SHAPES:
    sys.argv.remove("--shapes")
totals = [int(a) << 20 for a in sys.argv[1:]] or [m << 20 for m in (256, 512, 1024, 2048)]
ROUNDS = 10
for total in totals:
    n = total // 8
    pairs = POOL // (2 * total)
    splits = [k for k in (1, 2, 4, 8, 16) if total // k >= (64 << 20)]
    if SHAPES:      # (pieces, block, unroll); block 0 = the size-chosen shape
        splits = [(1, 0, 0), (2, 0, 0), (1, 1024, 1), (1, 512, 2), (1, 256, 4), (1, 256, 8)]
    else:
        splits = [(k, 0, 0) for k in splits]
    res = {k: [] for k in splits}
    i = 0
    for rnd in range(ROUNDS + 1):
        for key in splits:
            k, blk, unr = key
            pgamd.check(lib.pgk_tune_shape(blk, unr), "shape")
            d = base + 2 * total * (i % pairs)
            s = d + total
            i += 1
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            piece = n // k
            for j in range(k):
                off = j * piece * 8
                pgamd.check(lib.pgk_reduce(d + off, s + off, piece if j < k - 1 else n - piece * (k - 1), 1, 0, sh),
                            "reduce")
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[key].append(e0.elapsed_time(e1) * 1e3)
    pgamd.check(lib.pgk_tune_shape(0, 0), "shape")
    print(f"== {total >> 20} MiB per operand, {pairs} rotating pairs, medians of {ROUNDS} ==")
    for (k, blk, unr), v in res.items():
        med = statistics.median(v)
        shape = f"{blk}x{unr}" if blk else "by size"
        tile = (blk or 1024) * (unr or 1) * 16 if blk else None
        blocks = f"{total // k // tile:6d} blocks" if tile else ""
        print(f"  {k:2d} launch(es) of {total // k >> 20:5d} MiB, {shape:7s} {blocks:13s}: {med:9.2f} us  {3 * total / med / 1e3:7.1f} GB/s "
              f"({3 * total / med / 1e3 / 80:.1f}% of 8 TB/s)  min {min(v):9.2f}", flush=True)
