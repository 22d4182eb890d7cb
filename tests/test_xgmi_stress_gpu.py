"""PG_TRANSPORT=xgmi (and rccl, below) under a long random sequence of collectives in one process
lifetime per rank: reduce-scatter / all-gather / all-reduce, int32 / double,
sum / prod, sizes from 0 to 8 MiB, device / host / mixed buffers, in place,
inputs that stay allocated across calls, fresh ones, and fresh allocations
after torch.cuda.empty_cache() (which land at recycled addresses: the reuse
hazard: a new allocation at a freed one's address exports the same IPC handle bytes).  Every rank draws the same sequence from one seed
and checks every call bit for bit against the oracle's ring simulator.

This is the shape of the config-5 sequence (tools/xgmi_cfg5_probe.py) that
exposed the stale-mapping and desynchronisation bugs, widened to every call
form and buffer kind."""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]
COUNTS = (0, 1, 5, 64, 1000, 4099, 65539, 300001, (1 << 20) + 7)
CALLS = int(os.environ.get("XGMI_STRESS_CALLS", "120"))    # a soak run sets more


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sequence(seed, world):
    rng = np.random.default_rng(seed)
    seq = []
    for i in range(CALLS):
        coll = ("rs", "ag", "ar")[rng.integers(3)]
        dt, op = int(rng.integers(2)), int(rng.integers(2))
        count = int(COUNTS[rng.integers(len(COUNTS))])
        mem = ("dev", "dev", "dev", "host", "mixed")[rng.integers(5)]
        in_place = coll != "rs" and rng.random() < 0.2
        keep = rng.random() < 0.4            # reuse the previous call's input allocation if it fits
        flush = rng.random() < 0.15          # torch.cuda.empty_cache() before this call
        seq.append((i, coll, dt, op, count, mem, in_place, keep, flush))
    return seq


def _worker(rank, world, port, q, mode, seed, rings, transport="xgmi", tune=None):
    os.environ.update(PG_TRANSPORT=transport, PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_CONNECT_TIMEOUT_MS="120000", PG_BARRIER_TIMEOUT_MS="60000", PG_RINGS=str(rings))
    os.environ.update(tune or {})
    if transport == "xgmi":
        os.environ["PG_XGMI_MODE"] = mode
    else:        # the RCCL transport on one GPU: one host id per rank, hops over RCCL's socket transport
        os.environ.update(PG_ALGO=mode, NCCL_HOSTID=f"pg-stress-{port}-rank{rank}", NCCL_SOCKET_IFNAME="lo",
                          NCCL_IB_DISABLE="1")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    fails = []
    try:
        import ctypes

        import torch

        import pgamd
        from oracle.pyoracle import Oracle
        torch.cuda.set_device(0)
        lib = pgamd.load()
        orc = Oracle()
        h = ctypes.c_void_p()
        if lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) != 0:
            q.put((rank, ["connect: " + pgamd.last_error()]))
            return
        NP = {0: np.int32, 1: np.float64}
        TD = {0: torch.int32, 1: torch.float64}
        pool = None                                  # a kept device input allocation
        zc = 0                                       # calls whose inputs peers read in place
        for i, coll, dt, op, count, mem, in_place, keep, flush in _sequence(seed, world):
            if flush:
                pool = None
                torch.cuda.empty_cache()
            on_dev = mem == "dev" or (mem == "mixed" and rank % 2 == 0)
            xs = [orc.fill(count, dt, op, 9000 + 31 * i + r) for r in range(world)]
            if coll == "rs":
                want = orc.ring_reduce_scatter(xs, dt, op, rings)[rank]
                recv = np.zeros(max(want.size, 1), NP[dt])
            elif coll == "ag":
                want = orc.ring_all_gather(xs, dt)[rank]
                recv = np.zeros(max(count * world, 1), NP[dt])
                if in_place:
                    recv[rank * count:(rank + 1) * count] = xs[rank]
            else:
                want = orc.ring_all_reduce(xs, dt, op, rings)[rank]
                recv = xs[rank].copy() if in_place else np.zeros(max(count, 1), NP[dt])
                if recv.size == 0:
                    recv = np.zeros(1, NP[dt])
            send = xs[rank] if count else np.zeros(1, NP[dt])
            if on_dev:
                nbytes = send.nbytes
                if keep and pool is not None and pool.numel() * pool.element_size() >= nbytes + 4096:
                    # the same allocation as an earlier call, at an offset
                    S = pool.view(torch.uint8)[4096:4096 + nbytes].view(TD[dt])
                    S.copy_(torch.from_numpy(send))
                else:
                    pool = torch.empty((nbytes + 4096) // 4 + 1, dtype=torch.int32, device="cuda")
                    S = pool.view(torch.uint8)[4096:4096 + nbytes].view(TD[dt])
                    S.copy_(torch.from_numpy(send))
                R = torch.from_numpy(recv.copy()).cuda()
                torch.cuda.synchronize()
                sp, rp = S.data_ptr(), R.data_ptr()
            else:
                S, R = send.copy(), recv.copy()
                sp, rp = S.ctypes.data, R.ctypes.data
            if coll == "rs":
                rc = lib.pg_reduce_scatter(sp, rp, count, dt, op, h)
            elif coll == "ag":
                rc = lib.pg_all_gather(None if in_place else sp, rp, count, dt, h)
            else:
                rc = lib.pg_all_reduce(rp if in_place else sp, rp, count, dt, op, h)
            if rc != 0:
                fails.append((i, coll, count, mem, "rc", pgamd.last_error()))
                break
            zc += pgamd.stats(h)["zero_copy"]
            got = R.cpu().numpy() if on_dev else R
            if got[:want.size].tobytes() != want.tobytes():
                fails.append((i, coll, dt, op, count, mem, in_place, keep, flush))
        lib.pg_close(h)
        if transport == "xgmi" and mode == "read" and zc == 0:
            fails.append("no call read its inputs in place: zero-copy never exercised")
    except Exception as e:  # report, never hang the parent
        fails.append(("exception", repr(e)))
    q.put((rank, fails))


@pytest.mark.parametrize("world,mode,seed,rings", [(4, "read", 1, 2), (3, "push", 2, 2), (8, "read", 3, 2),
                                                   (5, "read", 4, 2), (8, "push", 5, 4), (5, "read", 6, 3)])
def test_xgmi_random_sequence(gpu, world, mode, seed, rings):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode, seed, rings)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=420))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, fails in results:
        assert not fails, (rank, fails)
    assert all(p.exitcode == 0 for p in procs)


SMALL_GROUPS = {"PG_CHUNK_BYTES": "65536", "PG_INFLIGHT": "2"}     # many transport groups per round


@pytest.mark.parametrize("world,algo,seed,rings,tune", [
    (3, "direct", 11, 2, None), (4, "ring", 12, 2, None), (2, "direct", 13, 1, None), (4, "direct", 14, 4, None),
    (4, "ring", 15, 2, dict(SMALL_GROUPS, PG_REDUCE_BYTES="393216")), (3, "ring", 16, 4, dict(SMALL_GROUPS, PG_REDUCE_BYTES="0")),
    (4, "direct", 17, 2, dict(SMALL_GROUPS, PG_REDUCE_BYTES="262144"))])
def test_rccl_random_sequence(gpu, world, algo, seed, rings, tune):
    """The same random sequence over the RCCL transport (ring and direct
    schedules; eager sizes, host / device / mixed buffers, in place, recycled
    allocations), every call against the oracle ring.  tune: small segments, so
    that a round is many transport groups, with the reduce launch taken per
    group (PG_REDUCE_BYTES=0) or once a few groups are pending."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, algo, seed, rings, "rccl", tune)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=420))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, fails in results:
        assert not fails, (rank, fails)
    assert all(p.exitcode == 0 for p in procs)
