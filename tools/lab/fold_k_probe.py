#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the multi-source fold at k = 2 .. 8 sources
(pgk_reduce_multi, kernel-stamped, sources rotating over a 4 GiB pool, double
sum), beside pgk_reduce_out on the same operands at k = 2 (the tuned
two-operand kernel computes the same out = a op b).  GB/s counts (k+1) x size.

    python tools/lab/fold_k_probe.py [MiB per source ...]     (default 16 64 256)
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
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
VP = ctypes.c_void_p
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
for mib in [int(a) for a in sys.argv[1:]] or [16, 64, 256]:
    size = mib << 20
    n = size // 8
    print(f"== {mib} MiB per source (kernel-stamped us median; GB/s of (k+1) x size; share of 8000) ==", flush=True)
    for k in (2, 3, 4, 5, 6, 7, 8):
        if (k + 1) * size > POOL // 2:
            continue
        sets = POOL // ((k + 1) * size)
        ts = []
        for i in range(13):
            b0 = base + (k + 1) * size * (i % sets)
            srcs = (VP * k)(*[b0 + size * j for j in range(k)])
            assert lib.pgk_reduce_multi_timed(b0 + k * size, srcs, k, n, 1, 0, sh, ev[0], ev[1]) == 0
            torch.cuda.synchronize()
            ms = ctypes.c_float()
            lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms))
            if i:
                ts.append(ms.value * 1e3)
        m = statistics.median(ts)
        print(f"  k={k}: {m:9.2f} us  {(k + 1) * size / m / 1e3:8.1f} GB/s {(k + 1) * size / m / 8e4:5.1f}%", flush=True)
    # the two-operand kernel on a k = 2 shape: out = a op b, events around back-to-back launches
    sets = POOL // (3 * size)
    for name, call in (("pgk_reduce_out (two-operand kernel)", lambda b0: lib.pgk_reduce_out(b0 + 2 * size, b0, b0 + size, n, 1, 0, sh)),
                       ("pgk_reduce_multi k=2", lambda b0: lib.pgk_reduce_multi(b0 + 2 * size, (VP * 2)(b0, b0 + size), 2, n, 1, 0, sh))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(4):
            call(base + 3 * size * (i % sets))
        torch.cuda.synchronize()
        e0.record()
        for i in range(20):
            assert call(base + 3 * size * (i % sets)) == 0
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        print(f"  back-to-back, {name}: {us:9.2f} us  {3 * size / us / 8e4:5.1f}%", flush=True)
