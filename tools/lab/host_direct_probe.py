#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the chunk reduce with both operands in PINNED host memory,
three ways:
  staged  pgx_reduce_host on pageable copies: pieces copied H2D, reduced in
          HBM, copied back D2H (SDMA engines, one direction at a time)
  pinned  pgx_reduce_host on the pinned buffers (the library detects them and
          reduces in place over PCIe)
  direct  pgk_reduce launched on the mapped device pointers by hand: the kernel
          reads dst and src across PCIe and writes dst back across PCIe itself,
          so both link directions carry data at once
Operands come from hipHostMalloc(hipHostMallocMapped) only: a kernel must never
touch pageable host memory (no XNACK on this pool).

    python tools/lab/host_direct_probe.py [MiB]
"""
import ctypes
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pgamd  # noqa: E402

HIP_HOST_MALLOC_MAPPED = 0x2


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = (mib << 20) // 8
    torch.cuda.init()
    lib = pgamd.load()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    bufs, dev = [], []
    for _ in range(2):
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), n * 8, HIP_HOST_MALLOC_MAPPED) == 0
        d = ctypes.c_void_p()
        assert hip.hipHostGetDevicePointer(ctypes.byref(d), p, 0) == 0
        bufs.append(p)
        dev.append(d)
    dst = np.ctypeslib.as_array(ctypes.cast(bufs[0], ctypes.POINTER(ctypes.c_double)), shape=(n,))
    src = np.ctypeslib.as_array(ctypes.cast(bufs[1], ctypes.POINTER(ctypes.c_double)), shape=(n,))
    rng = np.random.default_rng(1)
    d0 = rng.random(n) * 2 - 1
    src[:] = rng.random(n) * 2 - 1
    want = d0 + src
    sh = torch.cuda.current_stream().cuda_stream
    traffic = 3 * n * 8

    pd, ps = d0.copy(), src.copy()                 # pageable copies: the staged path
    for rep in range(3):
        pd[:] = d0
        t = time.perf_counter()
        pgamd.check(lib.pgx_reduce_host(pd.ctypes.data, ps.ctypes.data, n, pgamd.DT_DOUBLE, pgamd.OP_SUM, 0), "host")
        ms = (time.perf_counter() - t) * 1e3
        print(f"staged (pageable) {mib} MiB: {ms:8.2f} ms  {traffic / ms / 1e6:6.1f} GB/s  ok={np.array_equal(pd, want)}",
              flush=True)
    for rep in range(3):
        dst[:] = d0
        t = time.perf_counter()
        pgamd.check(lib.pgx_reduce_host(bufs[0].value, bufs[1].value, n, pgamd.DT_DOUBLE, pgamd.OP_SUM, 0), "host")
        ms = (time.perf_counter() - t) * 1e3
        print(f"pgx_reduce_host (pinned) {mib} MiB: {ms:8.2f} ms  {traffic / ms / 1e6:6.1f} GB/s  "
              f"ok={np.array_equal(dst, want)}", flush=True)
    for rep in range(3):
        dst[:] = d0
        torch.cuda.synchronize()
        t = time.perf_counter()
        pgamd.check(lib.pgk_reduce(dev[0].value, dev[1].value, n, pgamd.DT_DOUBLE, pgamd.OP_SUM, sh), "direct")
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        print(f"pgk_reduce on mapped pointers {mib} MiB: {ms:8.2f} ms  {traffic / ms / 1e6:6.1f} GB/s  ok={np.array_equal(dst, want)}",
              flush=True)
    for p in bufs:
        hip.hipHostFree(p)


if __name__ == "__main__":
    main()
