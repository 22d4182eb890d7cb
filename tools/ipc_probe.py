#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the HIP IPC behaviour the xgmi transport is built around
(csrc/pg_xport_xgmi.c), on one GPU with processes as ranks.

  --mode sizes   which device allocations can a second process map with
                 hipIpcOpenMemHandle, and how long does it take?  Each variant
                 runs in a fresh exporter/importer pair; a stalled import is
                 killed after --timeout seconds and reported as such.
                 Finding (MI355X, ROCm 7.2): sizes with bit 31 set (2 GiB,
                 2 GiB + 2 MiB, 3 GiB, 6 GiB) never open; others open in < 1 ms
                 -> ipc_size_ok / ipc_safe_size.
  --mode reuse   are HIP buffer ids / IPC handle bytes / base addresses reused
                 when an allocation is freed and another of the same size made?
                 Finding: the address and the handle bytes are reused, the
                 buffer id is not -> the export history (may_export).

    python tools/ipc_probe.py --mode sizes [--timeout 30] [--only prefix,...]
    python tools/ipc_probe.py --mode reuse
"""
import argparse
import ctypes
import multiprocessing as mp
import time


class Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def hiplib():
    import torch
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    hip.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    hip.hipMemGetAddressRange.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                          ctypes.c_void_p]
    return hip


GIB = 1 << 30
MIB = 1 << 20
VARIANTS = {
    # name: (how, bytes, cached bytes freed first)
    "hipMalloc 1.5 GiB": ("hip", 3 * GIB // 2, 0),
    "hipMalloc 2 GiB - 2 MiB": ("hip", 2 * GIB - 2 * MIB, 0),
    "hipMalloc 2 GiB + 2 MiB": ("hip", 2 * GIB + 2 * MIB, 0),
    "hipMalloc 3 GiB": ("hip", 3 * GIB, 0),
    "hipMalloc 5 GiB": ("hip", 5 * GIB, 0),
    "hipMalloc 6 GiB": ("hip", 6 * GIB, 0),
    "hipMalloc 8 GiB": ("hip", 8 * GIB, 0),
    "hipMalloc 12 GiB": ("hip", 12 * GIB, 0),
    "hipMalloc 1 GiB": ("hip", GIB, 0),
    "hipMalloc 2 GiB": ("hip", 2 * GIB, 0),
    "hipMalloc 4 GiB": ("hip", 4 * GIB, 0),
    "torch 256 MiB fresh": ("torch", 256 * MIB, 0),
    "torch 1 GiB fresh": ("torch", GIB, 0),
    "torch 2 GiB fresh": ("torch", 2 * GIB, 0),
    "torch 256 MiB carved from 512 MiB": ("torch", 256 * MIB, 512 * MIB),
    "torch 1 GiB carved from 2 GiB": ("torch", GIB, 2 * GIB),
    "torch 1 GiB carved from 1 GiB+2 MiB": ("torch", GIB, GIB + 2 * MIB),
}


def exporter(name, q_out, q_done):
    import torch
    hip = hiplib()
    how, nbytes, cached = VARIANTS[name]
    keep = None
    if how == "hip":
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), nbytes) == 0
        ptr = p.value
    else:
        if cached:
            tmp = torch.empty(cached, dtype=torch.uint8, device="cuda")
            del tmp                                   # stays in torch's cache
        keep = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        ptr = keep.data_ptr()
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(ptr))
    h = (ctypes.c_char * 64)()
    rc = hip.hipIpcGetMemHandle(h, base)
    q_out.put((rc, bytes(h), size.value, ptr - base.value))
    q_done.get(timeout=120)


def importer(q_in, q_res):
    hip = hiplib()
    rc, raw, size, off = q_in.get(timeout=120)
    if rc != 0:
        q_res.put(f"export rc={rc}")
        return
    m = ctypes.c_void_p()
    t0 = time.perf_counter()
    r = hip.hipIpcOpenMemHandle(ctypes.byref(m), Handle.from_buffer_copy(raw), 1)
    dt = time.perf_counter() - t0
    if r == 0:
        hip.hipIpcCloseMemHandle(m)
    q_res.put(f"open rc={r} in {dt * 1e3:.1f} ms (range {size >> 20} MiB, offset {off >> 20} MiB)")


def reuse():
    import torch
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipPointerGetAttribute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    buffer_id = 7     # hip/driver_types.h enum hipPointer_attribute: HIP_POINTER_ATTRIBUTE_BUFFER_ID

    def info(p):
        bid = ctypes.c_ulonglong()
        rc = hip.hipPointerGetAttribute(ctypes.byref(bid), buffer_id, p)
        h = (ctypes.c_char * 64)()
        rc2 = hip.hipIpcGetMemHandle(h, p)
        return rc, bid.value, rc2, bytes(h).hex()

    for size in (2 << 20, 256 << 20):
        seen = []
        for k in range(4):
            p = ctypes.c_void_p()
            hip.hipMalloc(ctypes.byref(p), size)
            rc, bid, rc2, h = info(p)
            seen.append((hex(p.value), bid, h[:48]))
            print(f"size {size >> 20} MiB alloc {k}: ptr {hex(p.value)} bid {bid} (rc {rc}) "
                  f"handle[0:24] {h[:48]} (rc {rc2})", flush=True)
            hip.hipFree(p)
        print("  same ptr reused:", len({s[0] for s in seen}) < len(seen),
              " bid reused:", len({s[1] for s in seen}) < len(seen),
              " handle reused:", len({s[2] for s in seen}) < len(seen), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("sizes", "reuse"), default="sizes")
    ap.add_argument("--timeout", type=float, default=30)
    ap.add_argument("--only", default="", help="comma-separated name prefixes")
    a = ap.parse_args()
    if a.mode == "reuse":
        reuse()
        return
    ctx = mp.get_context("spawn")
    for name in VARIANTS:
        if a.only and not any(name.startswith(p) for p in a.only.split(",")):
            continue
        q1, q2, q3 = ctx.Queue(), ctx.Queue(), ctx.Queue()
        pe = ctx.Process(target=exporter, args=(name, q1, q2))
        pi = ctx.Process(target=importer, args=(q1, q3))
        pe.start()
        pi.start()
        try:
            res = q3.get(timeout=a.timeout)
        except Exception:
            res = f"STALLED (> {a.timeout:.0f} s)"
        q2.put(1)
        for p in (pi, pe):
            p.join(10)
            if p.is_alive():
                p.kill()
                p.join()
        print(f"{name:40s} {res}", flush=True)


if __name__ == "__main__":
    main()
