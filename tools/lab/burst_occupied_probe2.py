#!/usr/bin/env python3
"""EXPERIMENTS ONLY: how many workgroups may a burst launch have, when other
kernels hold part of the GPU?  The lab's burst kernel (tools/lab/burst_lab.hip,
8 sources, 32 tiles per wave) with 384 .. 1024 workgroups per launch and 16, 24 or 32 tiles per wave, beside G parked workgroups of 256 lanes x 128
VGPRs (tools/lab/occupy_lab.hip).  Kernel-stamped; share of 8000 GB/s.

    python tools/lab/burst_occupied_probe2.py
"""
import ctypes
import pathlib
import statistics
import sys

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

VP = ctypes.c_void_p
occ = ctypes.CDLL(str(HERE / "liboccupylab.so"))
occ.occupy_launch.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_int, VP]
lab = ctypes.CDLL(str(HERE / "libburstlab.so"))
lab.burst_launch_k.argtypes = [ctypes.c_int] * 4 + [ctypes.c_uint, ctypes.c_uint, ctypes.c_int, VP, ctypes.POINTER(VP),
                                                    ctypes.c_size_t, VP, VP, VP]
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
K = 8


def fold_us(blocks, unroll, occupied):
    size = blocks * 256 * unroll * 16
    span = (K + 1) * size
    sets = POOL // span
    ts = []
    for i in range(9):
        b0 = base + span * (i % sets)
        srcs = (VP * 8)(*[b0 + size * j for j in range(K)])
        torch.cuda.synchronize()
        if occupied:
            assert occ.occupy_launch(occupied, 40000, 2000, side.cuda_stream) == 0
        assert lab.burst_launch_k(K, unroll, 256, 16, 0, 0, 0, b0 + K * size, srcs, size // 8, main.cuda_stream,
                                  ev[0], ev[1]) == 0
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms))
        if i:
            ts.append(ms.value * 1e3)
    return (K + 1) * size / statistics.median(ts) / 8e4


GS = (0, 8, 32, 64, 128)
print("  workgroups x tiles per wave (MiB per source)   " + "".join(f"  G={g:<4d}" for g in GS), flush=True)
for blocks, unroll in ((512, 32), (480, 32), (448, 32), (384, 32), (1024, 16), (896, 16), (832, 16), (768, 16), (640, 16),
                       (512, 16), (456, 16), (768, 24), (640, 24), (576, 24), (512, 24)):
    row = "".join(f"  {max(fold_us(blocks, unroll, g) for _ in range(2)):5.1f}%" for g in GS)
    print(f"  {blocks:5d} x {unroll:2d} ({blocks * 256 * unroll * 16 >> 20:3d} MiB)                          {row}", flush=True)
