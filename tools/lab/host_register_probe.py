#!/usr/bin/env python3
"""EXPERIMENTS ONLY: what does pinning pageable host memory in place cost?
pgx_reduce_host reduces PINNED operands with one kernel across PCIe at ~80 GB/s
and stages PAGEABLE ones through HBM slots at 34-57 GB/s.  If hipHostRegister /
hipHostUnregister of a piece is cheap against the piece's transfer time, pageable
operands could be pinned piece by piece ahead of the kernel instead of copied.

    python tools/lab/host_register_probe.py
"""
import ctypes
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pgamd  # noqa: E402

lib = pgamd.load()
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
# the HIP runtime this process already uses (torch's and libpg_amd.so's), not a second copy
hip_path = next(line.split()[-1] for line in open("/proc/self/maps") if "libamdhip64" in line)
print("HIP runtime:", hip_path, flush=True)
hip = ctypes.CDLL(hip_path)
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
MAPPED = 0x02        # hipHostRegisterMapped

n = 1 << 25                                    # 256 MiB of doubles per operand


def aligned(seed):
    """n random doubles starting on a page boundary (pageable memory)."""
    raw = np.empty(n + 512, dtype=np.float64)
    off = (-raw.ctypes.data % 4096) // 8
    v = raw[off:off + n]
    v[:] = np.random.default_rng(seed).random(n)
    return v


a, b = aligned(1), aligned(2)
want = a + b
hip.hipGetErrorString.restype = ctypes.c_char_p
hip.hipGetErrorString.argtypes = [ctypes.c_int]
for flags in (0, 1, 2, 3):
    rc = hip.hipHostRegister(a.ctypes.data, 4 << 20, flags)
    print(f"hipHostRegister(numpy memory at {a.ctypes.data:#x}, 4 MiB, flags {flags}) -> {rc} {hip.hipGetErrorString(rc).decode()}",
          flush=True)
    if rc == 0:
        hip.hipHostUnregister(a.ctypes.data)
        MAPPED = flags
        break
else:
    import mmap
    m = mmap.mmap(-1, 8 << 20)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(m))
    rc = hip.hipHostRegister(addr, 4 << 20, 0)
    print(f"hipHostRegister(mmap memory at {addr:#x}) -> {rc} {hip.hipGetErrorString(rc).decode()}", flush=True)
    sys.exit(0)
for piece_mib in (4, 16, 64, 256):
    piece = piece_mib << 20
    reg, unreg = [], []
    for rep in range(3):
        for off in range(0, min(n * 8, 4 * piece), piece):
            p = a.ctypes.data + off
            t0 = time.perf_counter()
            rc = hip.hipHostRegister(p, piece, MAPPED)
            t1 = time.perf_counter()
            assert rc == 0, (rc, hex(p), piece)
            rc = hip.hipHostUnregister(p)
            t2 = time.perf_counter()
            assert rc == 0, rc
            reg.append((t1 - t0) * 1e3)
            unreg.append((t2 - t1) * 1e3)
    xfer = piece / 55e9 * 1e3
    print(f"{piece_mib:4d} MiB piece: register {statistics.median(reg):7.3f} ms (min {min(reg):.3f}), unregister "
          f"{statistics.median(unreg):7.3f} ms; one PCIe direction moves it in {xfer:.3f} ms", flush=True)

# end to end: register both operands whole, one kernel on the mapped pointers, unregister
for rep in range(3):
    d = aligned(0)
    d[:] = a
    t0 = time.perf_counter()
    assert hip.hipHostRegister(d.ctypes.data, n * 8, MAPPED) == 0
    assert hip.hipHostRegister(b.ctypes.data, n * 8, MAPPED) == 0
    t1 = time.perf_counter()
    pgamd.check(lib.pgx_reduce_host(d.ctypes.data, b.ctypes.data, n, 1, 0, 0), "reduce")
    t2 = time.perf_counter()
    hip.hipHostUnregister(d.ctypes.data)
    hip.hipHostUnregister(b.ctypes.data)
    t3 = time.perf_counter()
    assert d.tobytes() == want.tobytes()
    print(f"whole operands: register 2 x 256 MiB {1e3 * (t1 - t0):.2f} ms, reduce (kernel across PCIe) {1e3 * (t2 - t1):.2f} ms, "
          f"unregister {1e3 * (t3 - t2):.2f} ms, total {1e3 * (t3 - t0):.2f} ms", flush=True)
d = a.copy()
t0 = time.perf_counter()
pgamd.check(lib.pgx_reduce_host(d.ctypes.data, b.ctypes.data, n, 1, 0, 0), "reduce")
print(f"shipped pageable path (staged through HBM): {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
d = a.copy()
t0 = time.perf_counter()
pgamd.check(lib.pgx_reduce_host(d.ctypes.data, b.ctypes.data, n, 1, 0, 0), "reduce")
print(f"shipped pageable path, second call: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
