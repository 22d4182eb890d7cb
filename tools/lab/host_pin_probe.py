#!/usr/bin/env python3
"""EXPERIMENTS ONLY: could pageable host operands go faster through pinned
staging that the reduce kernel reads and writes across PCIe itself?

pgx_reduce_host moves pageable operands with hipMemcpy (the runtime stages
them, SDMA, one direction at a time: 12.8 ms per 256 MiB double sum), while
pinned operands let one kernel read and write across PCIe at once (10.0 ms).
The candidate: host threads copy pageable pieces into pinned slots, the kernel
reduces slot to slot across PCIe, host threads copy the result out.  This
times the three parts alone for 256 MiB per operand, with 1-16 copy threads:

  in   : dst and src pieces, pageable -> pinned (2 x 256 MiB)
  gpu  : pgk_reduce_out over the pinned pieces, device addresses (3 x 256 MiB over PCIe)
  out  : result pieces, pinned -> pageable (256 MiB)

and the three overlapped over a 3-slot pipeline (thread pools for in/out,
one stream for the kernels), against pgx_reduce_host on the same arrays.

    python tools/lab/host_pin_probe.py [piece MiB]      (default 16)
"""
import concurrent.futures as cf
import ctypes
import pathlib
import statistics
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

lib = pgamd.load()
torch.cuda.set_device(0)
N = 1 << 25                                  # 256 MiB of doubles per operand
PIECE = (int(sys.argv[1]) if len(sys.argv) > 1 else 16) << 20
PE = PIECE // 8
rng = np.random.default_rng(1)
dst0 = rng.uniform(-1, 1, N)
src = rng.uniform(-1, 1, N)
want = dst0 + src
SLOTS = 3
pin_a = [torch.empty(PE, dtype=torch.float64).pin_memory() for _ in range(SLOTS)]
pin_b = [torch.empty(PE, dtype=torch.float64).pin_memory() for _ in range(SLOTS)]
pin_o = [torch.empty(PE, dtype=torch.float64).pin_memory() for _ in range(SLOTS)]
stream = torch.cuda.Stream()
sh = stream.cuda_stream
hip = ctypes.CDLL("libamdhip64.so")


def devptr(t):
    """The device address of a pinned tensor (hipHostGetDevicePointer, as pg_host.c does)."""
    d = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(t.data_ptr()), 0) == 0 and d.value
    return d.value


dev_a, dev_b, dev_o = ([devptr(t) for t in pins] for pins in (pin_a, pin_b, pin_o))


def par_copy(pool, nthreads, dst, src_):
    """dst[:] = src_ in nthreads slices."""
    n = dst.size
    step = -(-n // nthreads)
    futs = [pool.submit(np.copyto, dst[i:i + step], src_[i:i + step]) for i in range(0, n, step)]
    for f in futs:
        f.result()


def parts(nthreads):
    pool = cf.ThreadPoolExecutor(nthreads)
    d = dst0.copy()
    t_in = t_gpu = t_out = 0.0
    for off in range(0, N, PE):
        a, b, o = pin_a[0].numpy(), pin_b[0].numpy(), pin_o[0].numpy()
        t = time.perf_counter()
        par_copy(pool, nthreads, a, d[off:off + PE])
        par_copy(pool, nthreads, b, src[off:off + PE])
        t_in += time.perf_counter() - t
        t = time.perf_counter()
        pgamd.check(lib.pgk_reduce_out(dev_o[0], dev_a[0], dev_b[0], PE, 1, 0, sh), "reduce")
        stream.synchronize()
        t_gpu += time.perf_counter() - t
        t = time.perf_counter()
        par_copy(pool, nthreads, d[off:off + PE], o)
        t_out += time.perf_counter() - t
    pool.shutdown()
    assert np.array_equal(d, want)
    return t_in * 1e3, t_gpu * 1e3, t_out * 1e3


def pipelined(nthreads):
    """piece k: copy in (pool A) -> kernel on slot k % 3 -> copy out (pool B)."""
    pin_pool = cf.ThreadPoolExecutor(nthreads)
    out_pool = cf.ThreadPoolExecutor(nthreads)
    d = dst0.copy()
    pieces = list(range(0, N, PE))
    evs = [torch.cuda.Event() for _ in range(SLOTS)]
    outs = [None] * SLOTS                            # futures of the copy-out using each slot
    t = time.perf_counter()

    def copy_in(k):
        s, off = k % SLOTS, pieces[k]
        par_copy(pin_pool, nthreads, pin_a[s].numpy(), d[off:off + PE])
        par_copy(pin_pool, nthreads, pin_b[s].numpy(), src[off:off + PE])

    def copy_out(k):
        s, off = k % SLOTS, pieces[k]
        evs[s].synchronize()
        par_copy(out_pool, nthreads, d[off:off + PE], pin_o[s].numpy())

    driver = cf.ThreadPoolExecutor(2)
    fin = driver.submit(copy_in, 0)
    for k in range(len(pieces)):
        s = k % SLOTS
        fin.result()
        if outs[s] is not None:
            outs[s].result()                         # slot's previous result copied out
        pgamd.check(lib.pgk_reduce_out(dev_o[s], dev_a[s], dev_b[s], PE, 1, 0, sh), "reduce")
        evs[s].record(stream)
        outs[s] = driver.submit(copy_out, k)
        if k + 1 < len(pieces):
            nxt = (k + 1) % SLOTS
            if outs[nxt] is not None:
                outs[nxt].result()                   # kernel k-2 (slot nxt) is done: its inputs may be refilled
            fin = driver.submit(copy_in, k + 1)
    for f in outs:
        if f is not None:
            f.result()
    ms = (time.perf_counter() - t) * 1e3
    for p in (pin_pool, out_pool, driver):
        p.shutdown()
    assert np.array_equal(d, want)
    return ms


def shipped():
    d = dst0.copy()
    t = time.perf_counter()
    pgamd.check(lib.pgx_reduce_host(d.ctypes.data, src.ctypes.data, N, 1, 0, 0), "pgx_reduce_host")
    ms = (time.perf_counter() - t) * 1e3
    assert np.array_equal(d, want)
    return ms


shipped()
print(f"256 MiB double sum, pageable operands, {PIECE >> 20} MiB pieces; ms (median of 3)")
print(f"  pgx_reduce_host (shipped)          {statistics.median([shipped() for _ in range(3)]):7.2f}", flush=True)
for nt in (1, 2, 4, 8, 16):
    r = [parts(nt) for _ in range(3)]
    med = [statistics.median(x[i] for x in r) for i in range(3)]
    pl = statistics.median([pipelined(nt) for _ in range(3)])
    print(f"  {nt:2d} threads: in {med[0]:6.2f}  gpu {med[1]:6.2f}  out {med[2]:6.2f}  (sum {sum(med):6.2f})  "
          f"pipelined {pl:6.2f}", flush=True)
