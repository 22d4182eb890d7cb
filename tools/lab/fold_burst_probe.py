#!/usr/bin/env python3
"""The shipped fold with and without its burst form (pgk_tune_fold), through
the library: pgk_reduce_multi over 5..8 local sources, sizes on and off the
64 MiB launch boundary, both dtypes.  Events stamped on the call's first
launch's begin and its last one's end; share of 8000 GB/s counting
(k + 1) x bytes per source.  Every burst result is compared with the plain
form's, byte for byte.

    python tools/lab/fold_burst_probe.py
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
sh = torch.cuda.current_stream().cuda_stream
POOL = 5 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1e-3, 1e-3)
base = pool.data_ptr()
VP = ctypes.c_void_p
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")


def timed(k, size, dt, burst):
    lib.pgk_tune_fold(burst)
    es = 8 if dt == 1 else 4
    span = (k + 1) * size
    sets = max(1, POOL // span)
    ts = []
    for i in range(11):
        b0 = base + span * (i % sets)
        srcs = (VP * k)(*[b0 + size * j for j in range(k)])
        assert lib.pgk_reduce_multi_timed(b0 + k * size, srcs, k, size // es, dt, 0, sh, ev[0], ev[1]) == 0
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms))
        if i:
            ts.append(ms.value * 1e3)
    lib.pgk_tune_fold(1)
    return statistics.median(ts)


def same(k, size, dt):
    es = 8 if dt == 1 else 4
    srcs = (VP * k)(*[base + size * j for j in range(k)])
    outs = []
    for burst in (0, 1):
        lib.pgk_tune_fold(burst)
        o = torch.empty(size // 8, dtype=torch.float64, device="cuda")
        assert lib.pgk_reduce_multi(o.data_ptr(), srcs, k, size // es, dt, 0, sh) == 0
        torch.cuda.synchronize()
        outs.append(o)
    lib.pgk_tune_fold(1)
    return torch.equal(outs[0].view(torch.int64), outs[1].view(torch.int64))


print("   k  dtype  MiB/source   plain us    %     burst us    %   same bytes", flush=True)
for k in (5, 6, 7, 8):
    for dt in (1, 0):
        for mib in ((24, 32, 40, 48, 56, 64, 72, 80, 96, 112, 128, 160, 256, 512) if k == 8 and dt == 1 else (32, 64, 160)):
            size = mib << 20
            if (k + 1) * size > POOL:
                continue
            a = min(timed(k, size, dt, 0) for _ in range(2))
            b = min(timed(k, size, dt, 1) for _ in range(2))
            print(f"   {k}  {'f64' if dt else 'i32'}   {mib:6d}     {a:9.2f} {(k + 1) * size / a / 8e4:6.1f}   {b:9.2f} {(k + 1) * size / b / 8e4:6.1f}   "
                  f"{same(k, size, dt)}", flush=True)
