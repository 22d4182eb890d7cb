"""TEST INFRASTRUCTURE ONLY -- ctypes access to the CPU oracle.

  liboracle.so      : oracle/pg_oracle.c, the C restatement of the reference's
                      path (cites reference file:line per function).
  _ref/libpgref.so  : the reference's own src/pg.c path lines, compiled by
                      oracle/Makefile (container; travels prebuilt to the GPU box).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker or the timed CPU baseline.  Parity is
pinned: tests/golden/ fixtures come from _ref/libpgref.so (gen_golden.py), and
tests/test_oracle_golden.py checks the restatement against them.
"""
from __future__ import annotations

import ctypes
import pathlib

import numpy as np

ORACLE_DIR = pathlib.Path(__file__).resolve().parent
ORACLE_LIB = ORACLE_DIR / "liboracle.so"
REF_LIB = ORACLE_DIR / "_ref" / "libpgref.so"

DT_INT32, DT_DOUBLE = 0, 1
OP_SUM, OP_PROD = 0, 1
NP_DTYPE = {DT_INT32: np.int32, DT_DOUBLE: np.float64}

_VP, _SZ, _I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _ptr_array(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


class Oracle:
    """The C restatement (liboracle.so)."""

    def __init__(self, path: pathlib.Path = ORACLE_LIB):
        if not path.exists():
            raise RuntimeError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        lib = ctypes.CDLL(str(path))
        sig = {
            "orc_elem_size": (_SZ, [_I]),
            "orc_chunk_elems_from_bytes": (_SZ, [_SZ, _I]),
            "orc_chunk_offsets": (None, [_SZ, _SZ, _I, _SZ, ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
            "orc_rs_send_chunk_index": (_I, [_I, _I, _I]),
            "orc_rs_recv_chunk_index": (_I, [_I, _I, _I]),
            "orc_reduce_inplace": (None, [_VP, _VP, _SZ, _I, _I]),
            "orc_mock_reduce_scatter": (_I, [_I, _I, _SZ, _VP, _VP, _I, _I, _I]),
            "orc_mock_all_gather": (_I, [_I, _I, _VP, _VP, _I, _I]),
            "orc_mock_all_reduce": (_I, [_I, _I, _SZ, _VP, _VP, _I, _I, _I]),
            "orc_ring_reduce_scatter": (_I, [_I, ctypes.POINTER(_VP), ctypes.POINTER(_VP), _I, _I, _I, _I]),
            "orc_ring_step": (_I, [_I, _I, _I]),
            "orc_ring_all_gather": (_I, [_I, ctypes.POINTER(_VP), ctypes.POINTER(_VP), _I, _I]),
            "orc_ring_all_reduce": (_I, [_I, ctypes.POINTER(_VP), ctypes.POINTER(_VP), _I, _I, _I, _I]),
            "orc_ring_block": (None, [_SZ, _I, _I, ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
            "orc_fill": (None, [_VP, _SZ, _I, _I, ctypes.c_uint64]),
            "orc_time_reduce": (ctypes.c_double, [_VP, _VP, _SZ, _I, _I, _I]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        self.lib = lib

    # -- inputs ---------------------------------------------------------------
    def fill(self, n: int, dt: int, op: int, seed: int) -> np.ndarray:
        a = np.empty(n, dtype=NP_DTYPE[dt])
        if n:
            self.lib.orc_fill(_ptr(a), n, dt, op, seed & 0xFFFFFFFFFFFFFFFF)
        return a

    # -- the hot loop -----------------------------------------------------------
    def reduce(self, dst: np.ndarray, src: np.ndarray, dt: int, op: int) -> np.ndarray:
        out = np.array(dst, copy=True)
        if out.size:
            self.lib.orc_reduce_inplace(_ptr(out), _ptr(src), out.size, dt, op)
        return out

    # -- reference mock collectives (one rank) -------------------------------------
    def mock_reduce_scatter(self, rank, world, chunk_bytes, send, recv, dt, op):
        r = np.array(recv, copy=True)
        rc = self.lib.orc_mock_reduce_scatter(rank, world, chunk_bytes, _ptr(send), _ptr(r), send.size, dt, op)
        return rc, r

    def mock_all_gather(self, rank, world, send, recv, count, dt):
        r = np.array(recv, copy=True)
        rc = self.lib.orc_mock_all_gather(rank, world, _ptr(send), _ptr(r), count, dt)
        return rc, r

    # -- real-ring semantics ----------------------------------------------------------
    def ring_step(self, world, rings, g):
        return self.lib.orc_ring_step(world, rings, g)

    def ring_block(self, count, world, b):
        off, ln = _SZ(), _SZ()
        self.lib.orc_ring_block(count, world, b, ctypes.byref(off), ctypes.byref(ln))
        return off.value, ln.value

    # rings: 2 = the library default (PG_RINGS), 1 = one clockwise ring, 3 / 4 = rings of
    # step +3 / -3 added (include/pg_ext.h)
    def ring_reduce_scatter(self, sends, dt, op, rings=2):
        world, count = len(sends), sends[0].size
        outs = [np.zeros(self.ring_block(count, world, b)[1], dtype=NP_DTYPE[dt]) for b in range(world)]
        rc = self.lib.orc_ring_reduce_scatter(world, _ptr_array(sends), _ptr_array(outs), count, dt, op, rings)
        assert rc == 0
        return outs

    def ring_all_gather(self, sends, dt):
        world, count = len(sends), sends[0].size
        recvs = [np.zeros(count * world, dtype=NP_DTYPE[dt]) for _ in range(world)]
        rc = self.lib.orc_ring_all_gather(world, _ptr_array(sends), _ptr_array(recvs), count, dt)
        assert rc == 0
        return recvs

    def ring_all_reduce(self, sends, dt, op, rings=2):
        world, count = len(sends), sends[0].size
        recvs = [np.zeros(count, dtype=NP_DTYPE[dt]) for _ in range(world)]
        rc = self.lib.orc_ring_all_reduce(world, _ptr_array(sends), _ptr_array(recvs), count, dt, op, rings)
        assert rc == 0
        return recvs

    def time_reduce(self, dst, src, dt, op, reps) -> float:
        return self.lib.orc_time_reduce(_ptr(dst), _ptr(src), dst.size, dt, op, reps)


class Reference:
    """The reference's own path, compiled from /root/reference/src/pg.c (oracle/_ref)."""

    def __init__(self, path: pathlib.Path = REF_LIB):
        if not path.exists():
            raise RuntimeError(f"{path} missing: `make -C oracle ref` needs /root/reference")
        lib = ctypes.CDLL(str(path))
        sig = {
            "ref_elem_size": (_SZ, [_I]),
            "ref_chunk_elems_from_bytes": (_SZ, [_SZ, _I]),
            "ref_chunk_offsets": (None, [_SZ, _SZ, _I, _SZ, ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
            "ref_rs_send_chunk_index": (_I, [_I, _I, _I]),
            "ref_rs_recv_chunk_index": (_I, [_I, _I, _I]),
            "ref_reduce_inplace": (None, [_VP, _VP, _SZ, _I, _I]),
            "ref_reduce_scatter": (_I, [_I, _I, _SZ, _VP, _VP, _I, _I, _I]),
            "ref_all_gather": (_I, [_I, _I, _VP, _VP, _I, _I]),
            "ref_all_reduce": (_I, [_I, _I, _SZ, _VP, _VP, _I, _I, _I]),
            "ref_time_reduce": (ctypes.c_double, [_VP, _VP, _SZ, _I, _I, _I]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        self.lib = lib

    def reduce(self, dst, src, dt, op):
        out = np.array(dst, copy=True)
        if out.size:
            self.lib.ref_reduce_inplace(_ptr(out), _ptr(src), out.size, dt, op)
        return out

    def reduce_scatter(self, rank, world, chunk_bytes, send, recv, dt, op):
        r = np.array(recv, copy=True)
        rc = self.lib.ref_reduce_scatter(rank, world, chunk_bytes, _ptr(send), _ptr(r), send.size, dt, op)
        return rc, r

    def all_gather(self, rank, world, send, recv, count, dt):
        r = np.array(recv, copy=True)
        rc = self.lib.ref_all_gather(rank, world, _ptr(send), _ptr(r), count, dt)
        return rc, r

    def all_reduce(self, rank, world, chunk_bytes, send, recv, dt, op):
        r = np.array(recv, copy=True)
        s = r if send is None else send
        rc = self.lib.ref_all_reduce(rank, world, chunk_bytes, _ptr(s), _ptr(r), r.size, dt, op)
        return rc, r

    def time_reduce(self, dst, src, dt, op, reps) -> float:
        return self.lib.ref_time_reduce(_ptr(dst), _ptr(src), dst.size, dt, op, reps)


def splitmix64_numpy(seed: int, n: int) -> np.ndarray:
    """Vectorised splitmix64 (same stream as orc_splitmix64), for fixture checks."""
    with np.errstate(over="ignore"):
        k = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))
