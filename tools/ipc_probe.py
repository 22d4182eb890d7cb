#!/usr/bin/env python3
"""Probe hipIpcGetMemHandle on fresh hipMalloc allocations of several sizes and
in several alloc/free orders (diagnostic for the xgmi exchange slots)."""
import ctypes
import sys

import torch  # loads the HIP runtime torch uses (the one libpg_amd.so binds to)

torch.cuda.set_device(0)
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipGetErrorString.restype = ctypes.c_char_p


def alloc(sz):
    p = ctypes.c_void_p()
    e = hip.hipMalloc(ctypes.byref(p), sz)
    return p, e


def get(p):
    h = (ctypes.c_char * 64)()
    e = hip.hipIpcGetMemHandle(h, p)
    return e


MiB = 1 << 20
print("independent allocations:")
for sz in (64, 128, 256, 384, 512, 768, 1024, 2048, 4096):
    p, e = alloc(sz * MiB)
    g = get(p)
    print(f"  {sz:5d} MiB  malloc={e} ipc={g} {hip.hipGetErrorString(g).decode()} addr={hex(p.value or 0)}")
    hip.hipFree(p)
print("keep A, then B:")
a, _ = alloc(256 * MiB)
print("  A ipc", get(a))
b, _ = alloc(512 * MiB)
print("  B ipc", get(b))
hip.hipFree(a)
c, _ = alloc(1024 * MiB)
print("  C ipc after free(A)", get(c))
hip.hipFree(b)
hip.hipFree(c)
print("after torch allocations:")
t = [torch.empty(s, dtype=torch.uint8, device="cuda") for s in (75 * MiB, 300 * MiB, 600 * MiB)]
for sz in (256, 512, 1024):
    p, e = alloc(sz * MiB)
    print(f"  {sz:5d} MiB ipc={get(p)}")
    hip.hipFree(p)
sys.stdout.flush()
