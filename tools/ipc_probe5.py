#!/usr/bin/env python3
"""EXPERIMENTS ONLY: two exporter processes make same-size allocations (which
land at the same virtual address in each), fill them with their own rank, and
export; one importer opens both handles and reads back what each mapping holds.
Do handles from different processes collide?"""
import ctypes
import multiprocessing as mp
import os


class Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def hiplib():
    import torch
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    hip.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    return hip


def exporter(rank, q_out, q_done):
    hip = hiplib()
    p = ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(p), 2 << 20)
    hip.hipMemset(p, rank + 1, 2 << 20)
    h = (ctypes.c_char * 64)()
    hip.hipIpcGetMemHandle(h, p)
    q_out.put((rank, os.getpid(), hex(p.value), bytes(h)))
    q_done.get(timeout=120)


def importer(handles, q_res):
    hip = hiplib()
    out = []
    for rank, pid, va, raw in handles:
        m = ctypes.c_void_p()
        rc = hip.hipIpcOpenMemHandle(ctypes.byref(m), Handle.from_buffer_copy(raw), 1)
        b = (ctypes.c_ubyte * 4)()
        if rc == 0:
            hip.hipMemcpy(b, m, 4, 2)
        out.append((rank, pid, va, raw[:32].hex(), rc, hex(m.value or 0), list(b)))
    q_res.put(out)


def main():
    ctx = mp.get_context("spawn")
    q1, q2, q3 = ctx.Queue(), ctx.Queue(), ctx.Queue()
    ex = [ctx.Process(target=exporter, args=(r, q1, q2)) for r in range(2)]
    for p in ex:
        p.start()
    handles = sorted(q1.get(timeout=120) for _ in ex)
    imp = ctx.Process(target=importer, args=(handles, q3))
    imp.start()
    for row in q3.get(timeout=120):
        print("exporter rank %d pid %d va %s handle %s -> open rc %d at %s reads %s (expect %d)" % (*row, row[0] + 1),
              flush=True)
    for _ in ex:
        q2.put(1)
    for p in ex + [imp]:
        p.join(30)


if __name__ == "__main__":
    main()
