"""ctypes binding of libpg_amd.so (include/pg.h, include/pg_ext.h, include/pgk.h).

This is how Python callers (tests, bench.py, __graft_entry__) reach the C-ABI;
a C/C++ caller links libpg_amd.so directly.  There is no Python or CPU
implementation of any collective or reduction here: if the shared library is
missing, `load()` raises.

PyTorch, when present, is imported before the library is opened so that both
resolve the same HIP runtime (libamdhip64.so.7 is matched by SONAME).
"""
from __future__ import annotations

import ctypes
import os
import pathlib

PKG_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libpg_amd.so"
REPO_ROOT = PKG_DIR.parent

# include/pg.h (reference pg.h:78-87)
DT_INT32, DT_DOUBLE = 0, 1
FOLD_REMOTE_SOURCES, FOLD_SHARED_GPU = 1, 2        # pgk_fold_timed flags (include/pgk.h)
OP_SUM, OP_PROD = 0, 1
# include/pg_ext.h
PG_TRANSPORT_RCCL, PG_TRANSPORT_LOOPBACK, PG_TRANSPORT_THREADS, PG_TRANSPORT_SELF, PG_TRANSPORT_XGMI = 0, 1, 2, 3, 4
PG_BUF_NONE, PG_BUF_SRC, PG_BUF_OUT, PG_BUF_STAGE0, PG_BUF_STAGE1 = 0, 1, 2, 3, 4
PG_COLL_REDUCE_SCATTER, PG_COLL_ALL_GATHER, PG_COLL_ALL_REDUCE = 0, 1, 2
# include/pgk.h
PGK_STAGED_MAX_BYTES = 16 << 20

ELEM_SIZE = {DT_INT32: 4, DT_DOUBLE: 8}


class PgStep(ctypes.Structure):
    """struct pg_step (include/pg_ext.h)."""
    _fields_ = [
        ("round", ctypes.c_int32), ("batch", ctypes.c_int32), ("seg", ctypes.c_int32),
        ("send_wait", ctypes.c_int32),
        ("send_buf", ctypes.c_int32), ("recv_buf", ctypes.c_int32),
        ("red_dst_buf", ctypes.c_int32), ("red_src_buf", ctypes.c_int32),
        ("send_peer", ctypes.c_int32), ("recv_peer", ctypes.c_int32),
        ("send_off", ctypes.c_int64), ("send_bytes", ctypes.c_int64),
        ("recv_off", ctypes.c_int64), ("recv_bytes", ctypes.c_int64),
        ("red_dst_off", ctypes.c_int64), ("red_src_off", ctypes.c_int64),
        ("red_elems", ctypes.c_int64),
        ("red_rev", ctypes.c_int32), ("red_fold", ctypes.c_int32),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class PgRedRange(ctypes.Structure):
    """struct pg_red_range (include/pg_ext.h)."""
    _fields_ = [("dst_buf", ctypes.c_int32), ("src_buf", ctypes.c_int32), ("rev", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("dst_off", ctypes.c_int64), ("src_off", ctypes.c_int64),
                ("elems", ctypes.c_int64)]


class PgStats(ctypes.Structure):
    """struct pg_stats (include/pg_ext.h)."""
    _fields_ = [
        ("wall_us", ctypes.c_double), ("h2d_us", ctypes.c_double), ("d2h_us", ctypes.c_double),
        ("ring_us", ctypes.c_double),
        ("reduce_launches", ctypes.c_int64), ("reduce_elems", ctypes.c_int64),
        ("bytes_sent", ctypes.c_int64), ("bytes_recv", ctypes.c_int64),
        ("sync_us", ctypes.c_double), ("copy_us", ctypes.c_double), ("barrier_us", ctypes.c_double),
        ("kernel_us", ctypes.c_double), ("zero_copy", ctypes.c_int32), ("retried", ctypes.c_int32),
        ("calls_redone", ctypes.c_int64), ("red_kernel_us", ctypes.c_double), ("red_kernel_bytes", ctypes.c_int64),
        ("transport", ctypes.c_int32), ("algo_direct", ctypes.c_int32), ("xgmi_push", ctypes.c_int32),
        ("xgmi_mode_auto", ctypes.c_int32), ("probe_read_gbs", ctypes.c_double), ("probe_write_gbs", ctypes.c_double),
    ]


class PgHead(ctypes.Structure):
    """Leading fields of struct pg (include/pg.h) -- what a reference harness reads/sets."""
    _fields_ = [
        ("rank", ctypes.c_int), ("world_size", ctypes.c_int),
        ("chunk_bytes", ctypes.c_size_t), ("eager_max", ctypes.c_size_t),
        ("inflight", ctypes.c_int),
        ("hosts", ctypes.POINTER(ctypes.c_char_p)), ("port", ctypes.c_int),
        ("device", ctypes.c_int), ("transport", ctypes.c_int), ("impl", ctypes.c_void_p),
    ]


_lib = None

_VP, _CVP, _SZ, _I = ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
_SIGS = {
    # include/pg.h
    "connect_process_group": (_I, [ctypes.c_char_p, ctypes.POINTER(_VP)]),
    "pg_close": (_I, [_VP]),
    "pg_all_reduce": (_I, [_VP, _VP, _I, _I, _I, _VP]),
    "pg_reduce_scatter": (_I, [_VP, _VP, _I, _I, _I, _VP]),
    "pg_all_gather": (_I, [_VP, _VP, _I, _I, _VP]),
    # include/pg_ext.h
    "pg_block_range": (_I, [_I, _I, _I, ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
    "pg_plan_reduce_scatter": (_I, [_I, _I, _I, _I, _SZ, _SZ, _I, _I, _I, ctypes.POINTER(PgStep), _I]),
    "pg_plan_direct_reduce_scatter": (_I, [_I, _I, _I, _I, _SZ, _I, _I, ctypes.POINTER(PgStep), _I]),
    "pg_plan_all_gather": (_I, [_I, _I, _I, _I, _I, _I, ctypes.POINTER(PgStep), _I]),
    "pg_block_part": (_I, [_SZ, _I, _I, ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
    "pg_plan_coalesce": (_I, [ctypes.POINTER(PgStep), ctypes.POINTER(_I), _I, _SZ, ctypes.POINTER(PgRedRange), _I]),
    "pg_ring_offset": (_I, [_I, _I, _I]),
    "pgx_xgmi_link_probe": (_I, [_VP, _SZ, _I, ctypes.POINTER(ctypes.c_double)]),
    "pgx_xgmi_mode": (_I, [_VP, ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "pg_connect_local": (_I, [_I, _I, _I, ctypes.POINTER(_VP)]),
    "pgx_sim_run": (_I, [_I, _I, ctypes.POINTER(_VP), ctypes.POINTER(_VP), _I, _I, _I, _SZ, _SZ, _I, _I]),
    "pg_get_stats": (_I, [_VP, ctypes.POINTER(PgStats)]),
    "pgx_reduce_host": (_I, [_VP, _CVP, _SZ, _I, _I, _SZ]),
    "pg_last_error": (ctypes.c_char_p, []),
    "pgx_boot_selftest": (_I, [ctypes.c_char_p, _I, _I, _I, ctypes.POINTER(_I)]),
    # include/pgk.h
    "pgk_reduce": (_I, [_VP, _CVP, _SZ, _I, _I, _VP]),
    "pgk_reduce_out": (_I, [_VP, _CVP, _CVP, _SZ, _I, _I, _VP]),
    "pgk_reduce_ranges": (_I, [ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.POINTER(_SZ),
                               _I, _I, _I, _VP, _VP, _VP]),
    "pgk_reduce_multi_timed": (_I, [_VP, ctypes.POINTER(_VP), _I, _SZ, _I, _I, _VP, _VP, _VP]),
    "pgk_fold_timed": (_I, [_VP, ctypes.POINTER(_VP), _I, _SZ, _I, _I, ctypes.c_uint, _VP, _VP, _VP]),
    "pgk_tune_fold": (_I, [_I]),
    "pgk_fold_geometry": (_I, [_SZ, _I, _I, ctypes.c_uint, ctypes.POINTER(_SZ), ctypes.POINTER(_I), _I,
                               ctypes.POINTER(_SZ)]),
    "pgk_reduce_multi": (_I, [_VP, ctypes.POINTER(_VP), _I, _SZ, _I, _I, _VP]),
    "pgk_fold_blocks": (_I, [_VP, ctypes.POINTER(_VP), _I, _SZ, _SZ, _I, _I, _I, _VP]),
    "pgk_gather": (_I, [ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.POINTER(_SZ), _I, _VP]),
    "pgk_all_reduce_staged": (_I, [ctypes.POINTER(_VP), ctypes.POINTER(_VP), _I, _SZ, _I, _I, _I, _VP]),
    "pgk_device_count": (_I, [ctypes.POINTER(_I)]),
    "pgk_set_device": (_I, [_I]),
    "pgk_synchronize": (_I, []),
    "pgk_tune": (_I, [_I, _I]),
    "pgk_tune_shape": (_I, [_I, _I]),
    "pgk_reduce_timed": (_I, [_VP, _CVP, _SZ, _I, _I, _VP, _VP, _VP]),
    "pgk_event_create": (_I, [ctypes.POINTER(_VP)]),
    "pgk_event_destroy": (_I, [_VP]),
    "pgk_event_elapsed_ms": (_I, [_VP, _VP, ctypes.POINTER(ctypes.c_float)]),
    "pgk_launch_geometry": (_I, [_SZ, _I, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_uint)]),
    "pgk_last_error": (ctypes.c_char_p, []),
    "pgk_version": (ctypes.c_char_p, []),
}


def load() -> ctypes.CDLL:
    """Open libpg_amd.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `make -C rdma-ring-collectives_amd` "
            "or __graft_entry__.build(); there is no fallback implementation")
    try:  # share torch's HIP runtime if torch is used in this process
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    lib = load()
    msg = lib.pg_last_error() or b""
    kmsg = lib.pgk_last_error() or b""
    return (msg or kmsg).decode(errors="replace")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {last_error()}")


def block_range(count: int, world: int, block: int) -> tuple[int, int]:
    lib = load()
    off, ln = ctypes.c_size_t(), ctypes.c_size_t()
    check(lib.pg_block_range(count, world, block, ctypes.byref(off), ctypes.byref(ln)), "pg_block_range")
    return off.value, ln.value


def block_part(length: int, rings: int, part: int) -> tuple[int, int]:
    """(offset, length) of ring part `part` of a block (include/pg_ext.h)."""
    lib = load()
    off, ln = ctypes.c_size_t(), ctypes.c_size_t()
    check(lib.pg_block_part(length, rings, part, ctypes.byref(off), ctypes.byref(ln)), "pg_block_part")
    return off.value, ln.value


def ring_offset(world: int, rings: int, part: int) -> int:
    """Step d of ring `part` (send to rank+d, receive from rank-d; include/pg_ext.h)."""
    return load().pg_ring_offset(world, rings, part)


def plan_reduce_scatter(rank, world, count, dt, chunk_bytes, eager_max=4096, inflight=4, alias=0, rings=2):
    lib = load()
    n = lib.pg_plan_reduce_scatter(rank, world, count, dt, chunk_bytes, eager_max, inflight, rings, alias, None, 0)
    if n < 0:
        raise ValueError("pg_plan_reduce_scatter: bad arguments")
    arr = (PgStep * max(n, 1))()
    m = lib.pg_plan_reduce_scatter(rank, world, count, dt, chunk_bytes, eager_max, inflight, rings, alias, arr, n)
    assert m == n
    return [arr[i].as_dict() for i in range(n)]


def plan_direct_reduce_scatter(rank, world, count, dt, chunk_bytes, inflight=4, rings=2):
    lib = load()
    n = lib.pg_plan_direct_reduce_scatter(rank, world, count, dt, chunk_bytes, inflight, rings, None, 0)
    if n < 0:
        raise ValueError("pg_plan_direct_reduce_scatter: bad arguments")
    arr = (PgStep * max(n, 1))()
    m = lib.pg_plan_direct_reduce_scatter(rank, world, count, dt, chunk_bytes, inflight, rings, arr, n)
    assert m == n
    return [arr[i].as_dict() for i in range(n)]


def plan_all_gather(rank, world, count, dt, uniform=1, rings=2):
    lib = load()
    n = lib.pg_plan_all_gather(rank, world, count, dt, uniform, rings, None, 0)
    if n < 0:
        raise ValueError("pg_plan_all_gather: bad arguments")
    arr = (PgStep * max(n, 1))()
    lib.pg_plan_all_gather(rank, world, count, dt, uniform, rings, arr, n)
    return [arr[i].as_dict() for i in range(n)]


def plan_coalesce(steps, es):
    """pg_plan_coalesce on a list of step dicts (as the plan_* helpers return
    them): the ranges one reduce launch over those steps covers, as dicts."""
    lib = load()
    n = len(steps)
    arr = (PgStep * max(n, 1))()
    for i, s in enumerate(steps):
        for name, _ in PgStep._fields_:
            setattr(arr[i], name, s.get(name, 0))
    idx = (ctypes.c_int * max(n, 1))(*range(n))
    out = (PgRedRange * max(n, 1))()
    k = lib.pg_plan_coalesce(arr, idx, n, es, out, n)
    if k < 0:
        raise ValueError("pg_plan_coalesce: bad arguments")
    return [{name: getattr(out[i], name) for name, _ in PgRedRange._fields_} for i in range(k)]


def head(handle) -> PgHead:
    """View the public leading fields of a struct pg handle."""
    return PgHead.from_address(handle if isinstance(handle, int) else handle.value)


def stats(handle) -> dict:
    lib = load()
    st = PgStats()
    check(lib.pg_get_stats(handle, ctypes.byref(st)), "pg_get_stats")
    return {name: getattr(st, name) for name, _ in PgStats._fields_}


def header_symbols() -> list[str]:
    """Every function declared in include/*.h (for the ABI export test)."""
    import re
    names = []
    for h in sorted((REPO_ROOT / "include").glob("*.h")):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", text, flags=re.M):
            name = m.group(1)
            if name not in ("if", "for", "while", "return", "sizeof") and not name.isupper():
                names.append(name)
    return sorted(set(names))
