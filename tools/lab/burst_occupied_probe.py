#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the fold while another kernel holds part of the GPU.  In
the direct exchange the fold runs beside the transport's communication
kernels; the burst form wants all its 512 workgroups resident at once (two per
CU at its ~220 VGPRs), so what happens when some CUs are partly taken?
tools/lab/occupy_lab.hip parks G workgroups of 256 lanes x 128 VGPRs for the
duration; the fold (8 local sources x 64 MiB, double sum) is stamped beside
them: the burst form for a GPU the fold has to itself, the burst form for a
shared GPU (PGK_FOLD_SHARED_GPU) and the plain form.

    python tools/lab/burst_occupied_probe.py
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

so = HERE / "liboccupylab.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
                    str(HERE / "occupy_lab.hip"), "-o", str(so)], check=True)
occ = ctypes.CDLL(str(so))
VP = ctypes.c_void_p
occ.occupy_launch.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_int, VP]
lib = pgamd.load()
torch.cuda.set_device(0)
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1e-3, 1e-3)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
K, SIZE = 8, 64 << 20
span = (K + 1) * SIZE
sets = POOL // span


def fold_us(occupied, burst, flags=0):
    lib.pgk_tune_fold(burst)
    ts = []
    for i in range(9):
        b0 = base + span * (i % sets)
        srcs = (VP * K)(*[b0 + SIZE * j for j in range(K)])
        torch.cuda.synchronize()
        if occupied:
            # parked for 400 us (40,000 ticks), looked at every ~1 us: ends by itself
            assert occ.occupy_launch(occupied, 40000, 2000, side.cuda_stream) == 0
        assert lib.pgk_fold_timed(b0 + K * SIZE, srcs, K, SIZE // 8, 1, 0, flags, main.cuda_stream, ev[0], ev[1]) == 0
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms))
        if i:
            ts.append(ms.value * 1e3)
    lib.pgk_tune_fold(1)
    return statistics.median(ts)


print("  parked workgroups      whole-GPU form (one 64 MiB launch)   shared-GPU form (two 32 MiB launches)   one tile per wave",
      flush=True)
for g in (0, 8, 16, 32, 64, 128, 256):
    b = min(fold_us(g, 1) for _ in range(2))
    sh = min(fold_us(g, 1, pgamd.FOLD_SHARED_GPU) for _ in range(2))
    p = min(fold_us(g, 0) for _ in range(2))
    pct = lambda t: (K + 1) * SIZE / t / 8e4
    print(f"  {g:6d}                 {b:9.2f} us {pct(b):5.1f}%                 {sh:9.2f} us {pct(sh):5.1f}%"
          f"                  {p:9.2f} us {pct(p):5.1f}%", flush=True)
