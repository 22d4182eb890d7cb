#!/usr/bin/env python3
"""EXPERIMENTS ONLY: wall time per step of K back-to-back 256 MiB double-sum
reduces, launched (a) plainly, (b) with kernel-stamped start/stop events
(pgk_reduce_timed), (c) between torch marker events; interleaved rounds."""
import ctypes
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

lib = pgamd.load()
torch.cuda.set_device(0)
N = 1 << 25
K = 50
dst = [torch.rand(N, dtype=torch.float64, device="cuda") for _ in range(4)]
src = [torch.rand(N, dtype=torch.float64, device="cuda") for _ in range(4)]
sh = torch.cuda.current_stream().cuda_stream
ev = []
for _ in range(K):
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    lib.pgk_event_create(ctypes.byref(a))
    lib.pgk_event_create(ctypes.byref(b))
    ev.append((a, b))
tev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
res = {"plain": [], "ext-events": [], "torch-events": []}
for rnd in range(5):
    for mode in res:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            d, s = dst[i % 4].data_ptr(), src[i % 4].data_ptr()
            if mode == "plain":
                lib.pgk_reduce(d, s, N, 1, 0, sh)
            elif mode == "ext-events":
                lib.pgk_reduce_timed(d, s, N, 1, 0, sh, ev[i][0], ev[i][1])
            else:
                tev[i][0].record()
                lib.pgk_reduce(d, s, N, 1, 0, sh)
                tev[i][1].record()
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) / K * 1e6)
for mode, v in res.items():
    print(f"{mode:13s} median {statistics.median(v):8.2f} us/step  min {min(v):8.2f}")
ms = ctypes.c_float()
ks = []
for a, b in ev:
    lib.pgk_event_elapsed_ms(a, b, ctypes.byref(ms))
    ks.append(ms.value * 1e3)
print(f"kernel (ext events) median {statistics.median(ks):.2f} us")
