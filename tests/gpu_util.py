"""Helpers for the -m gpu tests: torch is plumbing (HBM allocations, copies,
stream handles); every computation under test goes through libpg_amd.so."""
import ctypes

import numpy as np

import pgamd


def to_dev(torch, a: np.ndarray):
    """Device copy of `a`.  Zero-length arrays get a 1-element allocation so
    the pointer is not NULL (a NULL buffer is an argument error, as in the
    reference src/pg.c:267); the view keeps the zero length."""
    if a.size == 0:
        t = torch.zeros(1, dtype=torch.from_numpy(a[:0]).dtype, device="cuda")
        t._logical_n = 0
        return t
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def to_host(torch, t) -> np.ndarray:
    torch.cuda.synchronize()
    out = t.cpu().numpy()
    n = getattr(t, "_logical_n", None)
    return out if n is None else out[:n]


def ptr(t) -> int:
    return t.data_ptr()


def stream(torch) -> int:
    return torch.cuda.current_stream().cuda_stream


def same_bits_nan_aware(got: np.ndarray, want: np.ndarray) -> bool:
    """Bit-identical, except that a NaN result only has to be a NaN (payload
    and sign of a NaN produced by the hardware are not part of the contract)."""
    if got.dtype != np.float64:
        return got.tobytes() == want.tobytes()
    gn, wn = np.isnan(got), np.isnan(want)
    if not np.array_equal(gn, wn):
        return False
    return got[~gn].tobytes() == want[~wn].tobytes()


def open_local(lib, rank, world, transport):
    h = ctypes.c_void_p()
    pgamd.check(lib.pg_connect_local(rank, world, transport, ctypes.byref(h)), "pg_connect_local")
    return h
