"""PG_TRANSPORT=rccl -- the RCCL point-to-point ring (csrc/pg_xport_rccl.c, the
replacement of the reference's RC-QP ring, src/RDMA_api.c:93-309 and
src/pg_net.c:721-783, at the hop sites src/pg.c:287,317) -- with REAL separate
processes on the one GPU of the test box.

RCCL refuses two ranks on one device ("Duplicate GPU detected"), and that check
compares (host hash, bus id).  Giving every rank its own NCCL_HOSTID makes RCCL
treat the ranks as separate nodes, so the communicator comes up and every hop
travels over RCCL's socket network transport on loopback instead of xGMI.  The
rates are meaningless; what runs is exactly our path: the unique-id relay, the
communicator, ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd per batch
(both rings of a W=2 ring target the same peer inside one group), the recv
events that gate the reduce stream, and the red events that gate forwarding.
Every rank checks its output bit for bit against the oracle's ring simulator.

Without the NCCL_HOSTID split the same launch must fail cleanly: both ranks get
-1 from connect_process_group, neither hangs.
"""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]

CASES = [  # coll, dt, op, count, on_dev, in_place
    ("rs", 1, 0, 1000, True, False), ("rs", 0, 1, 4099, False, False), ("rs", 1, 1, 1, True, False),
    ("rs", 0, 0, 0, True, False), ("rs", 1, 0, (1 << 20) + 3, True, False),
    ("ag", 1, 0, 257, True, False), ("ag", 0, 0, 64, False, False), ("ag", 1, 0, 33, True, True),
    ("ag", 1, 0, 300001, True, False),
    ("ar", 1, 0, 100003, True, False), ("ar", 0, 1, 999, False, False), ("ar", 1, 1, 4096, True, True),
    ("ar", 0, 0, 7, False, True), ("ar", 1, 0, 300001, True, False), ("ar", 0, 1, 524288, False, True),
    # BASELINE config 1 at its exact shape: int32 sum, count 1,048,576 (reference src/pg.c:264-291)
    ("rs", 0, 0, 1 << 20, True, False), ("ar", 0, 0, 1 << 20, True, False),
    ("rs", 0, 0, 1 << 20, False, False), ("ar", 0, 0, 1 << 20, True, True),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rccl_env(rank, port, split_hosts):
    env = dict(PG_TRANSPORT="rccl", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
               PG_CONNECT_TIMEOUT_MS="60000", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    if split_hosts:
        env["NCCL_HOSTID"] = f"pg-rccl-test-{port}-rank{rank}"
    return env


def _worker(rank, world, port, q, rings, chunk_bytes, inflight, cases, algo, env_extra=None):
    os.environ.update(_rccl_env(rank, port, True), PG_RINGS=str(rings), PG_CHUNK_BYTES=str(chunk_bytes),
                      PG_INFLIGHT=str(inflight))
    os.environ.update(env_extra or {})
    if algo:
        os.environ["PG_ALGO"] = algo
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
        hosts = " ".join(["127.0.0.1"] * world).encode()
        if lib.connect_process_group(hosts, ctypes.byref(h)) != 0:
            q.put((rank, ["connect: " + pgamd.last_error()]))
            return
        hd = pgamd.head(h)
        assert (hd.rank, hd.world_size, hd.transport) == (rank, world, pgamd.PG_TRANSPORT_RCCL)
        assert (hd.chunk_bytes, hd.inflight) == (chunk_bytes, inflight)
        NP = {0: np.int32, 1: np.float64}
        for i, (coll, dt, op, count, on_dev, in_place) in enumerate(cases):
            xs = [orc.fill(count, dt, op, 900 + 17 * i + r) for r in range(world)]
            if coll == "rs":
                want = orc.ring_reduce_scatter(xs, dt, op, rings)[rank]
                recv = np.zeros(max(want.size, 1), NP[dt])
            elif coll == "ag":
                want = orc.ring_all_gather(xs, dt)[rank]
                recv = np.zeros(count * world, NP[dt])
                if in_place:
                    recv[rank * count:(rank + 1) * count] = xs[rank]
            else:
                want = orc.ring_all_reduce(xs, dt, op, rings)[rank]
                recv = xs[rank].copy() if in_place else np.zeros(count, NP[dt])
            send = xs[rank] if xs[rank].size else np.zeros(1, NP[dt])
            if on_dev:
                S = torch.from_numpy(send.copy()).cuda()
                R = torch.from_numpy(recv.copy() if recv.size else np.zeros(1, NP[dt])).cuda()
                sp, rp = S.data_ptr(), R.data_ptr()
            else:
                S, R = send.copy(), recv.copy() if recv.size else np.zeros(1, NP[dt])
                sp, rp = S.ctypes.data, R.ctypes.data
            if coll == "rs":
                rc = lib.pg_reduce_scatter(sp, rp, count, dt, op, h)
            elif coll == "ag":
                rc = lib.pg_all_gather(None if in_place else sp, rp, count, dt, h)
            else:
                rc = lib.pg_all_reduce(rp if in_place else sp, rp, count, dt, op, h)
            if rc != 0:
                fails.append((i, "rc", pgamd.last_error()))
                break
            got = R.cpu().numpy() if on_dev else R
            if got[:want.size].tobytes() != want.tobytes():
                fails.append((i, coll, dt, op, count, on_dev, in_place))
        lib.pg_close(h)
    except Exception as e:  # report, never hang the parent
        fails.append(("exception", repr(e)))
    q.put((rank, fails))


def _run(world, target, args_of, timeout=300):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args_of(r)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=timeout))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return results, procs


@pytest.mark.parametrize("world,rings,chunk_bytes,inflight,algo", [
    (2, 2, 4 << 20, 4, "ring"), (2, 1, 1 << 16, 2, "ring"), (3, 2, 1 << 18, 4, "ring"), (4, 4, 1 << 16, 3, "ring"),
    (4, 1, 4 << 20, 1, "ring"),
    (2, 2, 4 << 20, 4, None), (3, 2, 1 << 16, 2, "direct"), (4, 4, 1 << 18, 3, "direct"), (4, 1, 1 << 16, 1, None)])
def test_rccl_ring_multiprocess(gpu, world, rings, chunk_bytes, inflight, algo):
    """The RCCL transport at W = 2, 3, 4 with 1, 2 and 4 rings, small and default
    segments, against the oracle ring -- every collective form, host and device
    buffers, in place, the eager one-shot sizes and config 1's exact shape.
    algo: PG_ALGO=ring (the W-1 round ring), direct (one hop per block over
    every link, csrc/pg_direct.c), None (the default: direct, one host)."""
    cases = CASES if world == 2 else [c for c in CASES if c[3] != 1 << 20]
    results, procs = _run(world, _worker, lambda r: (rings, chunk_bytes, inflight, cases, algo))
    for rank, fails in results:
        assert not fails, (rank, fails)
    assert all(p.exitcode == 0 for p in procs)


def _dup_worker(rank, world, port, q):
    os.environ.update(_rccl_env(rank, port, False))
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    try:
        import ctypes
        import time

        import torch

        import pgamd
        torch.cuda.set_device(0)
        lib = pgamd.load()
        h = ctypes.c_void_p()
        t0 = time.monotonic()
        rc = lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h))
        took = time.monotonic() - t0
        err = pgamd.last_error()
        if rc == 0:
            lib.pg_close(h)
        q.put((rank, (rc, took, err)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, ("exception", repr(e))))


def test_rccl_duplicate_device_refused_cleanly(gpu):
    """Two ranks on one device with one host id: RCCL refuses the communicator,
    and connect_process_group returns -1 on BOTH ranks (no rank hangs waiting
    for the other) well inside PG_CONNECT_TIMEOUT_MS."""
    results, procs = _run(2, _dup_worker, lambda r: (), timeout=180)
    for rank, res in results:
        assert res[0] == -1, (rank, res)
        assert res[1] < 60.0, (rank, res)
        assert "Duplicate" in res[2] or "invalid usage" in res[2].lower() or "ncclCommInitRank" in res[2], (rank, res)
    assert all(p.exitcode == 0 for p in procs)


def _native_worker(rank, world, port, q, store_port):
    """Our collectives against RCCL's own (torch.distributed, backend nccl =
    RCCL) on the same inputs: an implementation the oracle's author did not
    write.  int32 sum and product: bit-exact for reduce-scatter, all-gather and
    all-reduce (two's-complement wrap is order-independent).  double sum: our
    result is bit-exact against the oracle ring and within the survey's bound of
    RCCL's (different fold order)."""
    os.environ.update(_rccl_env(rank, port, True))
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    fails = []
    try:
        import ctypes

        import torch
        import torch.distributed as dist

        import pgamd
        from oracle.pyoracle import Oracle
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{store_port}", rank=rank, world_size=world)
        lib = pgamd.load()
        orc = Oracle()
        h = ctypes.c_void_p()
        if lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) != 0:
            q.put((rank, ["connect: " + pgamd.last_error()]))
            return
        for count in (world * 1000, world * 65536 + 0):
            for op in (0, 1):
                xs = [orc.fill(count, 0, op, 4242 + 7 * r + op) for r in range(world)]
                x = torch.from_numpy(xs[rank]).cuda()
                rop = dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.PRODUCT
                ln = count // world
                ours = torch.empty(ln, dtype=torch.int32, device="cuda")
                nat = torch.empty(ln, dtype=torch.int32, device="cuda")
                assert lib.pg_reduce_scatter(x.data_ptr(), ours.data_ptr(), count, 0, op, h) == 0, pgamd.last_error()
                dist.reduce_scatter_tensor(nat, x, op=rop)
                torch.cuda.synchronize()
                if not torch.equal(ours, nat):
                    fails.append(("rs", count, op))
                ar = torch.empty(count, dtype=torch.int32, device="cuda")
                assert lib.pg_all_reduce(x.data_ptr(), ar.data_ptr(), count, 0, op, h) == 0, pgamd.last_error()
                nat_ar = x.clone()
                dist.all_reduce(nat_ar, op=rop)
                torch.cuda.synchronize()
                if not torch.equal(ar, nat_ar):
                    fails.append(("ar", count, op))
            ag = torch.empty(count * world, dtype=torch.int32, device="cuda")
            assert lib.pg_all_gather(x.data_ptr(), ag.data_ptr(), count, 0, h) == 0, pgamd.last_error()
            nat_ag = torch.empty_like(ag)
            dist.all_gather_into_tensor(nat_ag, x)
            torch.cuda.synchronize()
            if not torch.equal(ag, nat_ag):
                fails.append(("ag", count))
        # double sum: bit-exact against the oracle's ring, within the bound of RCCL's
        count = world * 100003
        xs = [orc.fill(count, 1, 0, 5151 + r) for r in range(world)]
        want = orc.ring_reduce_scatter(xs, 1, 0, 2)[rank]
        x = torch.from_numpy(xs[rank]).cuda()
        ours = torch.empty(count // world, dtype=torch.float64, device="cuda")
        nat = torch.empty_like(ours)
        sabs = torch.empty_like(ours)
        assert lib.pg_reduce_scatter(x.data_ptr(), ours.data_ptr(), count, 1, 0, h) == 0, pgamd.last_error()
        dist.reduce_scatter_tensor(nat, x)
        dist.reduce_scatter_tensor(sabs, x.abs())
        torch.cuda.synchronize()
        if ours.cpu().numpy().tobytes() != want.tobytes():
            fails.append(("f64 vs oracle",))
        g = (world - 1) * 2.0 ** -53
        tol = 2 * g / (1 - g) * sabs
        if not bool(((ours - nat).abs() <= tol).all()):
            fails.append(("f64 vs rccl", float((ours - nat).abs().max())))
        # double product: bit-exact against the oracle's ring, and within
        # 2g/(1-g) of RCCL's product relative to it (each order is within g of
        # the exact product; inputs 1 + U[-2^-10, 2^-10) stay normal)
        xs = [orc.fill(count, 1, 1, 6161 + r) for r in range(world)]
        want = orc.ring_reduce_scatter(xs, 1, 1, 2)[rank]
        x = torch.from_numpy(xs[rank]).cuda()
        assert lib.pg_reduce_scatter(x.data_ptr(), ours.data_ptr(), count, 1, 1, h) == 0, pgamd.last_error()
        dist.reduce_scatter_tensor(nat, x, op=dist.ReduceOp.PRODUCT)
        torch.cuda.synchronize()
        if ours.cpu().numpy().tobytes() != want.tobytes():
            fails.append(("f64 prod vs oracle",))
        if not bool(((ours - nat).abs() <= 2 * g / (1 - 2 * g) * nat.abs()).all()):
            fails.append(("f64 prod vs rccl", float(((ours - nat).abs() / nat.abs()).max())))
        lib.pg_close(h)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        fails.append(("exception", repr(e)))
    q.put((rank, fails))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_collectives_match_rccl_native(gpu, world):
    """An independent pin for the W > 1 output contract: RCCL's own
    reduce-scatter / all-gather / all-reduce on the same int32 inputs give the
    same bits (sum and product), and the double sum stays within the survey's
    tolerance of RCCL's ((W-1) * 2^-53 * sum|x| per fold order) while matching the oracle exactly."""
    store_port = _free_port()
    results, procs = _run(world, _native_worker, lambda r: (store_port,))
    for rank, fails in results:
        assert not fails, (rank, fails)
    assert all(p.exitcode == 0 for p in procs)


def _fallback_worker(rank, world, port, q, fail_reach, forced):
    """Default transport choice (no PG_TRANSPORT) on one host, with the xgmi
    reach check made to fail on one rank (test hook PG_XGMI_FAIL_REACH)."""
    env = _rccl_env(rank, port, True)
    env.pop("PG_TRANSPORT")
    os.environ.pop("PG_TRANSPORT", None)
    os.environ.update(env, PG_XGMI_FAIL_REACH=str(fail_reach))
    if forced:
        os.environ["PG_TRANSPORT"] = "xgmi"
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    out = {}
    try:
        import ctypes

        import torch

        import pgamd
        from oracle.pyoracle import Oracle
        torch.cuda.set_device(0)
        lib = pgamd.load()
        orc = Oracle()
        h = ctypes.c_void_p()
        out["rc"] = lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h))
        out["err"] = pgamd.last_error()
        if out["rc"] == 0:
            out["transport"] = pgamd.head(h).transport
            count = 100003
            xs = [orc.fill(count, 1, 0, 7700 + r) for r in range(world)]
            want = orc.ring_reduce_scatter(xs, 1, 0, 2)[rank]
            S = torch.from_numpy(xs[rank]).cuda()
            R = torch.zeros(want.size, dtype=torch.float64, device="cuda")
            out["call"] = lib.pg_reduce_scatter(S.data_ptr(), R.data_ptr(), count, 1, 0, h)
            out["match"] = R.cpu().numpy().tobytes() == want.tobytes()
            lib.pg_close(h)
    except Exception as e:  # noqa: BLE001
        out["exception"] = repr(e)
    q.put((rank, out))


@pytest.mark.parametrize("world,fail_reach", [(2, 1), (3, 0), (2, -1)])
def test_default_transport_falls_back_to_rccl(gpu, world, fail_reach):
    """The server list says "one host", so xgmi is the default; when some rank
    cannot map a peer's device memory every rank learns it at connect and all
    of them come up on the RCCL transport instead, with the same results."""
    import pgamd
    results, procs = _run(world, _fallback_worker, lambda r: (fail_reach, False))
    for rank, out in results:
        assert out.get("rc") == 0, (rank, out)
        assert out["transport"] == pgamd.PG_TRANSPORT_RCCL, (rank, out)
        assert out["call"] == 0 and out["match"], (rank, out)
    assert all(p.exitcode == 0 for p in procs)


def test_forced_xgmi_without_reach_fails_on_every_rank(gpu):
    """PG_TRANSPORT=xgmi is the caller's choice: no silent fallback, and every
    rank gets -1 from connect_process_group together."""
    results, procs = _run(2, _fallback_worker, lambda r: (1, True), timeout=180)
    for rank, out in results:
        assert out.get("rc") == -1, (rank, out)
        assert "cannot map a peer" in out["err"], (rank, out)
    assert all(p.exitcode == 0 for p in procs)


def test_direct_exchange_falls_back_to_ring_when_its_gather_area_cannot_grow(gpu, tmp_path):
    """The direct exchange's gather area is as large as the whole input.  When
    one rank cannot allocate it (test hook PG_TEST_FAIL_STAGE_ALLOC), every rank
    runs that call on the ring instead: same bits, nobody hangs, and later calls
    agree again on whether the area has to grow."""
    cases = [("rs", 1, 0, 300001, True, False), ("ar", 0, 1, 524288, True, False), ("rs", 1, 0, (1 << 20) + 3, True, False),
             ("ar", 1, 0, 100003, False, False), ("rs", 0, 0, 4099, True, False)]
    prefix = str(tmp_path / "trace")
    results, procs = _run(3, _worker, lambda r: (2, 1 << 18, 2, cases, "direct",
                                                 {"PG_TEST_FAIL_STAGE_ALLOC": "1", "PG_TRACE_FILE": prefix}))
    for rank, fails in results:
        assert not fails, (rank, fails)
    assert all(p.exitcode == 0 for p in procs)
    traces = "".join(f.read_text() for f in tmp_path.glob("trace.*"))
    assert traces.count("falling back to the ring") >= 3 * 4      # 3 ranks x the 4 calls above eager size


@pytest.mark.parametrize("algo,red_bytes", [("ring", 0), ("ring", 1 << 18), ("direct", 0), ("direct", 3 << 17)])
def test_rccl_reduce_launch_sizes(gpu, algo, red_bytes):
    """PG_REDUCE_BYTES over RCCL with real processes: 64 KiB segments, 2 in
    flight, 3 ranks, two rings; the arrived segments are reduced per group (0)
    or once a few groups are pending, host and device buffers, in place: the
    oracle ring's bits either way."""
    cases = [c for c in CASES if c[3] != 1 << 20]
    results, procs = _run(3, _worker, lambda r: (2, 1 << 16, 2, cases, algo, {"PG_REDUCE_BYTES": str(red_bytes)}))
    for rank, fails in results:
        assert not fails, (rank, fails)
    assert all(p.exitcode == 0 for p in procs)
