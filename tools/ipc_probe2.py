#!/usr/bin/env python3
"""Two processes: P1 imports P0's allocation, closes it, then allocates and
exports -- does a fresh allocation on a previously imported range export?"""
import ctypes
import multiprocessing as mp


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
    return hip


def p0(q_to1, q_from1):
    hip = hiplib()
    a = ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(a), 256 << 20)
    h = (ctypes.c_char * 64)()
    print("P0 export A", hip.hipIpcGetMemHandle(h, a), hex(a.value), flush=True)
    q_to1.put(bytes(h))
    q_from1.get(timeout=60)      # P1 done
    hip.hipFree(a)


def p1(q_from0, q_to0):
    try:
        hip = hiplib()
        raw = q_from0.get(timeout=60)
        h = Handle.from_buffer_copy(raw)
        m = ctypes.c_void_p()
        print("P1 import", hip.hipIpcOpenMemHandle(ctypes.byref(m), h, 1), hex(m.value or 0), flush=True)
        imp = m.value or 0
        print("P1 close", hip.hipIpcCloseMemHandle(m), flush=True)
        for sz in (256, 512, 128):
            b = ctypes.c_void_p()
            hip.hipMalloc(ctypes.byref(b), sz << 20)
            hh = (ctypes.c_char * 64)()
            print(f"P1 alloc {sz} MiB at {hex(b.value or 0)} (import was {hex(imp)}) export ->",
                  hip.hipIpcGetMemHandle(hh, b), flush=True)
    finally:
        q_to0.put(1)


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    a, b = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=p0, args=(a, b)), ctx.Process(target=p1, args=(a, b))]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=120)
