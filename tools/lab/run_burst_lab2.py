#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the burst fold of tools/lab/burst_lab.hip as it would ship:
a call is cut into launches of at most 64 MiB per source, and every launch is
ONE round (each wave folds all its tiles, then stores them), its tile count per
wave picked by the piece's size.  Against the shipped kernels, for 2..8 sources
and 8..256 MiB per source.  Events stamped on the first launch's start and the
last launch's end; GB/s counts (k + 1) x bytes per source.

    python tools/lab/run_burst_lab2.py
"""
import ctypes
import pathlib
import statistics
import subprocess
import sys

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

so = HERE / "libburstlab.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
                    str(HERE / "burst_lab.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
VP = ctypes.c_void_p
lab.burst_launch_k.argtypes = [ctypes.c_int] * 4 + [ctypes.c_uint, ctypes.c_uint, ctypes.c_int, VP, ctypes.POINTER(VP),
                                                    ctypes.c_size_t, VP, VP, VP]
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
PIECE = 64 << 20


def unroll_for(piece_bytes, blocks):
    """tiles per wave so that about `blocks` workgroups of 256 lanes cover the piece"""
    want = piece_bytes / (blocks * 256 * 16)
    return next(u for u in (2, 4, 8, 16, 32) if u >= want or u == 32)


def burst(k, srcs_at, out_at, size, e0, e1, blocks=512, inplace=False):
    """the call as single-round launches of <= 64 MiB per source"""
    off = 0
    while off < size:
        ln = min(PIECE, size - off)
        u = unroll_for(ln, blocks)
        srcs = (VP * 8)(*[srcs_at[min(j, k - 1)] + off for j in range(8)])
        first, last = off == 0, off + ln == size
        rc = lab.burst_launch_k(k, u, 256, 16, 0, 0, 0, out_at + off, srcs, ln // 8, sh, e0 if first else None,
                                e1 if last else None)
        assert rc == 0, (k, u, ln, rc)
        off += ln


def shipped(k, srcs_at, out_at, size, e0, e1):
    srcs = (VP * k)(*srcs_at[:k])
    assert lib.pgk_reduce_multi_timed(out_at, srcs, k, size // 8, 1, 0, sh, e0, e1) == 0


def shipped_inplace(k, srcs_at, out_at, size, e0, e1):     # k == 2, out == srcs[0]: the two-operand reduce
    assert lib.pgk_reduce_timed(out_at, srcs_at[1], size // 8, 1, 0, sh, e0, e1) == 0


# correctness: 2..8 sources, whole / ragged / multi-piece, out of place and over source 0
for k in (2, 3, 4, 5, 6, 7, 8):
    for size in (1 << 16, (4 << 20) + 4096 + 16, (72 << 20) + 32):
        n = size // 8
        for inplace in (False, True):
            want = pool[:n].clone()
            for j in range(1, k):
                want += pool[j * n:(j + 1) * n]
            keep = pool[:n].clone()
            at = [base + size * j for j in range(8)]
            out_at = at[0] if inplace else base + 8 * size
            burst(k, at, out_at, size, None, None)
            torch.cuda.synchronize()
            got = pool[:n] if inplace else pool[8 * n:9 * n]
            assert torch.equal(got, want), (k, size, inplace)
            pool[:n].copy_(keep)
print("burst launches checked against torch (2 .. 8 sources; ragged; several pieces; in place)", flush=True)


def measure(fn, k, size, inplace=False, **kw):
    span = (k + 1) * size
    sets = max(1, POOL // span)
    ts = []
    for i in range(13):
        b0 = base + span * (i % sets)
        at = [b0 + size * j for j in range(k)]
        out_at = at[0] if inplace else b0 + k * size
        fn(k, at, out_at, size, ev[0], ev[1], **kw)
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        pgamd.check(lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)), "elapsed")
        if i:
            ts.append(ms.value * 1e3)
    return statistics.median(ts)


def pct(k, size, us, inplace=False):
    return (k + (0 if inplace else 1) + (1 if inplace else 0)) * size / us / 8e4      # k reads + 1 write either way


print("== 8 sources: shipped pgk_reduce_multi against single-round burst launches (<= 64 MiB per source each) ==", flush=True)
print("   MiB/source   shipped us    %     burst(512 blocks) us    %     burst(1024 blocks) us    %", flush=True)
for mib in (4, 8, 16, 32, 64, 128, 256):
    size = mib << 20
    rows = []
    for rnd in range(2):
        rows.append((measure(shipped, 8, size), measure(burst, 8, size, blocks=512), measure(burst, 8, size, blocks=1024)))
    a, b, c = (min(r[i] for r in rows) for i in range(3))
    print(f"   {mib:6d}      {a:9.2f} {pct(8, size, a):6.1f}      {b:9.2f} {pct(8, size, b):13.1f}      {c:9.2f} {pct(8, size, c):14.1f}",
          flush=True)

print("== fewer sources, 64 and 256 MiB per source ==", flush=True)
for k in (2, 3, 4, 5, 6, 7):
    for mib in (16, 64, 256):
        size = mib << 20
        a = min(measure(shipped, k, size) for _ in range(2))
        b = min(measure(burst, k, size) for _ in range(2))
        print(f"   k={k} {mib:4d} MiB: shipped pgk_reduce_multi {a:8.2f} us {pct(k, size, a):5.1f}%   burst {b:8.2f} us {pct(k, size, b):5.1f}%",
              flush=True)
print("== the two-operand reduce in place (dst = dst + src): shipped pgk_reduce against the burst form ==", flush=True)
for mib in (16, 32, 64, 128, 256):
    size = mib << 20
    a = min(measure(shipped_inplace, 2, size, inplace=True) for _ in range(2))
    b = min(measure(burst, 2, size, inplace=True) for _ in range(2))
    c = min(measure(burst, 2, size, inplace=True, blocks=1024) for _ in range(2))
    print(f"   {mib:4d} MiB: shipped pgk_reduce {a:8.2f} us {3 * size / a / 8e4:5.1f}%   burst(512) {b:8.2f} us {3 * size / b / 8e4:5.1f}%"
          f"   burst(1024) {c:8.2f} us {3 * size / c / 8e4:5.1f}%", flush=True)
