"""The TCP bootstrap star (pg_boot.c) and the node-local shm barrier across
real processes, no GPU: rank 0
relays every rank's value to all (the path that carries the RCCL unique id
and the xgmi IPC handles), late joiners are retried, and a rank outside the
list is rejected."""
import ctypes
import multiprocessing as mp
import pathlib
import socket
import sys
import time

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, delay, q):
    sys.path[:0] = [str(ROOT / "rdma-ring-collectives_amd")]
    import pgamd
    lib = pgamd.load()
    time.sleep(delay)
    out = (ctypes.c_int * world)()
    hosts = " ".join(["127.0.0.1"] * world).encode()
    rc = lib.pgx_boot_selftest(hosts, rank, port, 1000 + rank * rank, out)
    q.put((rank, rc, list(out), pgamd.last_error()))


@pytest.mark.parametrize("world", [1, 2, 5])
def test_star_allgather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    # rank 0 starts last: the others must retry until its listener is up
    procs = [ctx.Process(target=_rank, args=(r, world, port, 1.0 if r == 0 else 0.0, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    want = [1000 + r * r for r in range(world)]
    for rank, rc, out, err in res:
        assert rc == 0, err
        assert out == want


def test_bad_rank(lib):
    out = (ctypes.c_int * 2)()
    assert lib.pgx_boot_selftest(b"a b", 5, 1, 0, out) == -1
    assert lib.pgx_boot_selftest(None, 0, 1, 0, out) == -1
