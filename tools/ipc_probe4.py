#!/usr/bin/env python3
"""EXPERIMENTS ONLY: are HIP buffer ids / IPC handle bytes / base addresses
reused when an allocation is freed and another one of the same size is made?
(The xgmi transport caches exports and imports by buffer id.)"""
import ctypes

import torch

torch.cuda.set_device(0)
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipPointerGetAttribute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
HIP_POINTER_ATTRIBUTE_BUFFER_ID = 7     # hip/driver_types.h enum hipPointer_attribute


def info(p):
    bid = ctypes.c_ulonglong()
    rc = hip.hipPointerGetAttribute(ctypes.byref(bid), HIP_POINTER_ATTRIBUTE_BUFFER_ID, p)
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
        print(f"size {size >> 20} MiB alloc {k}: ptr {hex(p.value)} bid {bid} (rc {rc}) handle[0:24] {h[:48]} (rc {rc2})",
              flush=True)
        hip.hipFree(p)
    print("  same ptr reused:", len({s[0] for s in seen}) < len(seen), " bid reused:", len({s[1] for s in seen}) < len(seen),
          " handle reused:", len({s[2] for s in seen}) < len(seen), flush=True)
