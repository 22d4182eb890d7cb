#!/usr/bin/env python3
"""EXPERIMENTS ONLY: does the fold stream faster when its output overwrites
one of its sources?  The two-operand reduce writes dst over the dst it has just
read (two address streams) and runs at 82%; the fold writes a separate output
(k + 1 streams) and runs at 74-77% from k = 3 up.  Here: pgk_reduce_multi with
out = a separate region, out = srcs[0] (the first source read), out =
srcs[k-1] (the last).  Kernel-stamped, rotating over a 4 GiB pool, double sum;
GB/s counts (k+1) x size in every case.

    python tools/lab/fold_inplace_probe.py [MiB per source ...]     (default 16 64)
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
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1e-3, 1e-3)
base = pool.data_ptr()
VP = ctypes.c_void_p
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
for mib in [int(a) for a in sys.argv[1:]] or [16, 64]:
    size = mib << 20
    n = size // 8
    print(f"== {mib} MiB per source (kernel-stamped us median; share of 8000 GB/s counting (k+1) x size) ==", flush=True)
    for k in (3, 4, 8):
        sets = POOL // ((k + 1) * size)
        res = {}
        for rnd in range(3):
            for where in ("separate", "first", "last"):
                for i in range(7):
                    b0 = base + (k + 1) * size * ((rnd * 21 + i) % sets)
                    srcs = (VP * k)(*[b0 + size * j for j in range(k)])
                    out = {"separate": b0 + k * size, "first": b0, "last": b0 + (k - 1) * size}[where]
                    assert lib.pgk_reduce_multi_timed(out, srcs, k, n, 1, 0, sh, ev[0], ev[1]) == 0
                    torch.cuda.synchronize()
                    ms = ctypes.c_float()
                    lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms))
                    if i:
                        res.setdefault(where, []).append(ms.value * 1e3)
        line = "  ".join(f"out = {w}: {statistics.median(v):8.2f} us {(k + 1) * size / statistics.median(v) / 8e4:5.1f}%"
                         for w, v in res.items())
        print(f"  k={k}: {line}", flush=True)
