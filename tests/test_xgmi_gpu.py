"""PG_TRANSPORT=xgmi with REAL separate processes (one rank per process) on the
one GPU of the test box: IPC-mapped exchange buffers, the bootstrap star, the
multi-source fold kernel and the public pg_* calls, end to end.  Every rank
checks its results bit for bit against the oracle's ring simulator (same fold
order as the RCCL ring)."""
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
    ("ar", 1, 0, 100003, True, False), ("ar", 0, 1, 999, False, False), ("ar", 1, 1, 4096, True, True),
    ("ar", 0, 0, 7, False, True), ("rs", 1, 0, 5000, True, False), ("ar", 1, 0, 300001, True, False),
    ("ar", 0, 1, 524288, False, True),
    # BASELINE config 1's exact shape (int32 sum, count 1,048,576; reference src/pg.c:264-291)
    ("rs", 0, 0, 1 << 20, True, False), ("ar", 0, 0, 1 << 20, True, False),
    # "mixed": even ranks pass device buffers, odd ranks host buffers -> every
    # rank must agree to fall back from zero-copy to the slot copy
    ("rs", 1, 0, 77777, "mixed", False), ("ar", 0, 0, 300000, "mixed", False), ("ag", 1, 0, 999, "mixed", False),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, oneshot_max, zero_copy="1", rings=2, mode="read", extra_env=None):
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_CONNECT_TIMEOUT_MS="120000", PG_ONESHOT_MAX=str(oneshot_max), PG_XGMI_ZERO_COPY=zero_copy,
                      PG_RINGS=str(rings), PG_XGMI_MODE=mode, PG_BARRIER_TIMEOUT_MS="60000")
    for k, v in (extra_env or {}).items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
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
        assert (hd.rank, hd.world_size, hd.transport) == (rank, world, pgamd.PG_TRANSPORT_XGMI)
        if os.environ.get("PG_XGMI_MODE") is None:        # auto: chosen at connect by the link probe
            push, rg, wg = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
            assert lib.pgx_xgmi_mode(h, ctypes.byref(push), ctypes.byref(rg), ctypes.byref(wg)) == 0
            assert push.value in (0, 1) and rg.value > 0 and wg.value > 0
            assert push.value == (wg.value >= 1.15 * rg.value)
        NP = {0: np.int32, 1: np.float64}
        for i, (coll, dt, op, count, on_dev, in_place) in enumerate(CASES):
            if on_dev == "mixed":
                on_dev = rank % 2 == 0
            xs = [orc.fill(count, dt, op, 700 + 13 * i + r) for r in range(world)]
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


@pytest.mark.parametrize("world,oneshot_max,zero_copy,rings,mode", [
    (2, 1 << 20, "1", 2, "read"), (3, 1 << 20, "1", 2, "read"), (4, 1 << 20, "1", 2, "read"),
    (8, 1 << 20, "1", 2, "read"), (2, 0, "1", 2, "read"), (5, 0, "1", 2, "read"), (4, 1 << 40, "1", 2, "read"),
    (3, 1 << 20, "0", 2, "read"), (4, 0, "0", 2, "read"), (4, 1 << 20, "1", 1, "read"), (3, 1 << 40, "0", 1, "read"),
    (2, 1 << 20, "1", 2, "push"), (4, 0, "1", 2, "push"), (8, 1 << 20, "1", 2, "push"), (3, 0, "1", 1, "push"),
    (5, 0, "0", 2, "push"), (8, 1 << 20, "1", 4, "read"), (5, 0, "1", 3, "push"), (4, 1 << 40, "1", 4, "read")])
def test_xgmi_multiprocess(gpu, world, oneshot_max, zero_copy, rings, mode):
    """oneshot_max selects the all-reduce form: 0 = always reduce-scatter +
    gather, 2^40 = always the one-shot fold, 1 MiB = the default split.
    zero_copy "0" forces the slot copy for every input.  rings: PG_RINGS (the
    fold order of each block's second half).  mode: PG_XGMI_MODE (push: the
    reduce-scatter writes each block to its owner; host, mixed and in-place
    cases fall back to the read path on every rank together)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, oneshot_max, zero_copy, rings, mode))
             for r in range(world)]
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


def _run_workers(world, args, timeout=420):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q) + args) for r in range(world)]
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
    for rank, fails in results:
        assert not fails, (rank, fails)
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_push_without_shm_page_reads(gpu, world):
    """PG_XGMI_MODE=push with PG_NO_SHM_BARRIER=1: push keeps its per-call
    flags in the shared-memory page, so without it every rank takes the read
    path (TCP barrier) instead of dereferencing a missing page.  All cases
    against the oracle."""
    _run_workers(world, (1 << 20, "1", 2, "push", {"PG_NO_SHM_BARRIER": "1"}))


@pytest.mark.parametrize("world", [2, 4])
def test_default_transport_is_xgmi_on_one_node(gpu, world):
    """No PG_TRANSPORT and no PG_XGMI_MODE, every server-list entry the same
    host, W <= 16: the xgmi transport (pg_default_transport) with the mode the
    connect-time link probe chose (PG_XGMI_MODE=auto); the worker asserts the
    transport and the probe's rule, and runs every case against the oracle."""
    _run_workers(world, (1 << 20, "1", 2, "read", {"PG_TRANSPORT": None, "PG_XGMI_MODE": None}))


def _grow_worker(rank, world, port, q):
    """Exchange slots grow (64 MiB granule, doubling) inside a sequence of
    calls; results checked against a closed form on the device."""
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port))
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    fails = []
    try:
        import ctypes

        import torch

        import pgamd
        torch.cuda.set_device(0)
        lib = pgamd.load()
        h = ctypes.c_void_p()
        assert lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) == 0
        for count in (1 << 10, 9 << 20, 30 << 20, 1 << 12, 9 << 20):     # doubles: 8 KiB .. 240 MiB
            i = torch.arange(count, device="cuda", dtype=torch.int64)
            x = ((i % 1000) + rank).to(torch.float64)
            want = ((i % 1000) * world + world * (world - 1) // 2).to(torch.float64)
            y = torch.empty(count, dtype=torch.float64, device="cuda")
            if lib.pg_all_reduce(x.data_ptr(), y.data_ptr(), count, 1, 0, h) != 0:
                fails.append((count, pgamd.last_error()))
                break
            if not torch.equal(y, want):
                fails.append((count, "mismatch"))
            off, ln = pgamd.block_range(count, world, rank)
            z = torch.empty(max(ln, 1), dtype=torch.float64, device="cuda")
            if lib.pg_reduce_scatter(x.data_ptr(), z.data_ptr(), count, 1, 0, h) != 0 or \
                    not torch.equal(z[:ln], want[off:off + ln]):
                fails.append((count, "rs", pgamd.last_error()))
            del i, x, y, z, want
            torch.cuda.empty_cache()
        lib.pg_close(h)
    except Exception as e:
        fails.append(("exception", repr(e)))
    q.put((rank, fails))


@pytest.mark.parametrize("world", [2, 3])
def test_xgmi_slot_growth(gpu, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grow_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=300))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, fails in results:
        assert not fails, (rank, fails)


def _bit31_worker(rank, world, port, q):
    """Allocations whose size has bit 31 set stall hipIpcOpenMemHandle on
    ROCm 7.2 (tools/ipc_probe.py --mode sizes).  600 MiB calls need 1 GiB slots, i.e. a
    2 GiB two-slot region that the transport must pad: (a) a fresh input is
    read in place and the all-reduce grows the result region; (b) an input
    that lives in a 2 GiB allocation cannot be shared in place, so every rank
    falls back to the slot copy together and grows the contribution region."""
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_BARRIER_TIMEOUT_MS="60000")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    fails = []
    try:
        import ctypes

        import torch

        import pgamd
        torch.cuda.set_device(0)
        lib = pgamd.load()
        h = ctypes.c_void_p()
        assert lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) == 0
        big = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")          # exactly 2 GiB
        for label, count in (("fresh input", (600 << 20) // 8), ("input in 2 GiB", (600 << 20) // 8)):
            i = torch.arange(count, device="cuda", dtype=torch.int64)
            if label == "input in 2 GiB":
                x = big[:count * 8].view(torch.float64)
                x.copy_(((i % 1000) + rank).to(torch.float64))
            else:
                x = ((i % 1000) + rank).to(torch.float64)
            want = ((i % 1000) * world + world * (world - 1) // 2).to(torch.float64)
            off, ln = pgamd.block_range(count, world, rank)
            z = torch.empty(max(ln, 1), dtype=torch.float64, device="cuda")
            if lib.pg_reduce_scatter(x.data_ptr(), z.data_ptr(), count, 1, 0, h) != 0 or \
                    not torch.equal(z[:ln], want[off:off + ln]):
                fails.append((label, "rs", pgamd.last_error()))
            y = torch.empty(count, dtype=torch.float64, device="cuda")
            if lib.pg_all_reduce(x.data_ptr(), y.data_ptr(), count, 1, 0, h) != 0 or not torch.equal(y, want):
                fails.append((label, "ar", pgamd.last_error()))
            del i, x, y, z, want
            torch.cuda.empty_cache()
        lib.pg_close(h)
    except Exception as e:
        fails.append(("exception", repr(e)))
    q.put((rank, fails))


def test_xgmi_ipc_bit31_sizes(gpu):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bit31_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=150))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, fails in results:
        assert not fails, (rank, fails)


def _release_worker(rank, world, port, q, push=False):
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_BARRIER_TIMEOUT_MS="60000", PG_XGMI_MODE="push" if push else "read")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    res = {}
    try:
        import ctypes

        import torch

        import pgamd
        torch.cuda.set_device(0)
        lib = pgamd.load()
        h = ctypes.c_void_p()
        assert lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) == 0
        small = torch.ones(1 << 16, dtype=torch.float64, device="cuda")
        sout = torch.empty(1 << 16, dtype=torch.float64, device="cuda")

        def sync_all():          # a collective: every rank has passed the previous call
            assert lib.pg_all_reduce(small.data_ptr(), sout.data_ptr(), 1 << 16, 1, 0, h) == 0, pgamd.last_error()

        sync_all()
        torch.cuda.synchronize()
        res["free0"] = torch.cuda.mem_get_info()[0]
        sync_all()
        if not push:
            count = 1 << 29                               # 4 GiB of doubles, read in place by the peers
            x = torch.full((count,), float(rank + 1), dtype=torch.float64, device="cuda")
            off, ln = pgamd.block_range(count, world, rank)
            out = torch.empty(ln, dtype=torch.float64, device="cuda")
            assert lib.pg_reduce_scatter(x.data_ptr(), out.data_ptr(), count, 1, 0, h) == 0, pgamd.last_error()
            res["zero_copy"] = pgamd.stats(h)["zero_copy"]
            res["ok"] = bool((out == world * (world + 1) / 2).all())
        else:
            # push mode: an all-gather still READS its peers' inputs (and caches the
            # mappings of a 1 GiB allocation here; 2 GiB ones are never exported, their
            # size has bit 31 set); the calls after it are pushed
            count = 1 << 27
            x = torch.full((count,), float(rank + 1), dtype=torch.float64, device="cuda")
            out = torch.empty(count * world, dtype=torch.float64, device="cuda")
            assert lib.pg_all_gather(x.data_ptr(), out.data_ptr(), count, 1, h) == 0, pgamd.last_error()
            res["zero_copy"] = pgamd.stats(h)["zero_copy"]
            res["ok"] = all(bool((out[q * count:(q + 1) * count] == q + 1).all()) for q in range(world))
        del x, out
        torch.cuda.empty_cache()                          # the caller frees its large input
        if not push:
            for kind in ("in place", "slot copy"):        # the next calls read other inputs
                y = torch.full((1 << 20,), 2.0, dtype=torch.float64, device="cuda")
                z = y if kind == "slot copy" else torch.empty(1 << 20, dtype=torch.float64, device="cuda")
                assert lib.pg_all_reduce(y.data_ptr(), z.data_ptr(), 1 << 20, 1, 0, h) == 0, pgamd.last_error()
                res["ok"] &= bool((z == 2.0 * world).all())
                del y, z
        else:
            for _ in range(2):                            # pushed calls: no peer input is read at all
                n = 1 << 21
                y = torch.full((n,), 2.0, dtype=torch.float64, device="cuda")
                o2, l2 = pgamd.block_range(n, world, rank)
                z = torch.empty(l2, dtype=torch.float64, device="cuda")
                assert lib.pg_reduce_scatter(y.data_ptr(), z.data_ptr(), n, 1, 0, h) == 0, pgamd.last_error()
                res["ok"] &= bool((z == 2.0 * world).all()) and pgamd.stats(h)["zero_copy"] == 0
                del y, z
        sync_all()
        torch.cuda.synchronize()
        res["free1"] = torch.cuda.mem_get_info()[0]
        sync_all()
        lib.pg_close(h)
    except Exception as e:
        res["exception"] = repr(e)
    q.put((rank, res))


@pytest.mark.parametrize("push", [False, True])
def test_xgmi_freed_large_input_is_released(gpu, push):
    """A peer's mapping of a caller's large input (4 GiB; 1 GiB per rank in the
    push case) must not keep that HBM alive once the caller has freed it and moved
    on: the next call closes large mappings it does not read, whether it reads
    other inputs in place, takes the slot copy, or (push mode, where an
    all-gather cached the mapping) pushes and reads no peer input at all.  Both
    ranks share the one GPU, so device free memory after the sequence must be
    back to where it was before the large inputs (within 1 GiB of small
    allocations)."""
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_release_worker, args=(r, world, port, q, push)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=240))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, res in results:
        assert "exception" not in res, res
        assert res["ok"] and res["zero_copy"] == 1, res
        assert res["free1"] > res["free0"] - (1 << 30), (rank, res["free0"] >> 20, res["free1"] >> 20)


def _probe_worker(rank, world, port, q):
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_BARRIER_TIMEOUT_MS="60000")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    out = {}
    try:
        import ctypes

        import torch

        import pgamd
        torch.cuda.set_device(0)
        lib = pgamd.load()
        h = ctypes.c_void_p()
        assert lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) == 0
        g = (ctypes.c_double * 4)()
        out["rc"] = lib.pgx_xgmi_link_probe(h, 64 << 20, 3, g)
        out["gbs"] = list(g)
        out["bad_rc"] = lib.pgx_xgmi_link_probe(h, 1000, 3, g)          # not a multiple of 4 KiB
        lib.pg_close(h)
    except Exception as e:
        out["exception"] = repr(e)
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 3])
def test_xgmi_link_probe(gpu, world):
    """pgx_xgmi_link_probe: the four copy phases run collectively and report
    positive rates (on the one-GPU box every "link" is the same device)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_probe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=150))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, out in results:
        assert "exception" not in out, out
        assert out["rc"] == 0 and all(v > 0 for v in out["gbs"]), (rank, out)
        assert out["bad_rc"] == -1


def _realloc_worker(rank, world, port, q):
    """A rank frees its input allocation and makes a new one, which lands at the
    same address (hipMalloc reuses it for equal sizes); the IPC handle of the
    new allocation is byte-identical to the old one's (tools/ipc_probe.py --mode reuse), so
    a peer that kept its mapping of the old allocation would be handed that
    stale mapping back by hipIpcOpenMemHandle and fold freed data."""
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_BARRIER_TIMEOUT_MS="60000")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    out = {"fails": [], "same_va": None}
    try:
        import ctypes

        import torch

        import pgamd
        torch.cuda.set_device(0)
        lib = pgamd.load()
        hip = ctypes.CDLL("libamdhip64.so.7")
        hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        hip.hipFree.argtypes = [ctypes.c_void_p]
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        h = ctypes.c_void_p()
        assert lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) == 0
        count = 8 << 20                                            # 64 MiB of doubles
        off, ln = pgamd.block_range(count, world, rank)
        vas = []
        for trial in range(3):
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), count * 8) == 0
            vas.append(p.value)
            x = (np.arange(count, dtype=np.float64) % 97) + 1000 * trial + rank
            assert hip.hipMemcpy(p, x.ctypes.data, count * 8, 1) == 0      # hipMemcpyHostToDevice
            y = torch.empty(ln, dtype=torch.float64, device="cuda")
            if lib.pg_reduce_scatter(p.value, y.data_ptr(), count, 1, 0, h) != 0:
                out["fails"].append((trial, pgamd.last_error()))
            out.setdefault("zero_copy", []).append(pgamd.stats(h)["zero_copy"])
            i = np.arange(off, off + ln)
            want = world * (i % 97) + world * 1000 * trial + world * (world - 1) // 2
            if not np.array_equal(y.cpu().numpy(), want.astype(np.float64)):
                out["fails"].append((trial, "stale or wrong data"))
            hip.hipFree(p)
        out["same_va"] = len(set(vas)) < len(vas)
        out["vas"] = vas
        lib.pg_close(h)
    except Exception as e:
        out["fails"].append(("exception", repr(e)))
    q.put((rank, out))


def test_xgmi_input_reallocated_at_same_address(gpu):
    import torch.multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_realloc_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=150))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, out in results:
        assert not out["fails"], (rank, out)
    assert any(out["same_va"] for _, out in results), "no address was reused: the test did not set up the hazard"
    # trial t is shared in place unless some rank's allocation recycles an address it exported before
    # (then every rank takes the slot copy: the choice is collective)
    trials = len(results[0][1]["vas"])
    for t in range(trials):
        recycled = any(out["vas"][t] in out["vas"][:t] for _, out in results)
        for rank, out in results:
            assert out["zero_copy"][t] == (0 if recycled else 1), (t, rank, out)


def _mismatch_worker(rank, world, port, q, mode):
    """Rank 1 passes a different count than the others.  Every rank must fail
    that call (the descriptors carry each rank's byte count) before any peer
    memory is read with the wrong extent, and the ranks must stay in step: the
    next, well-formed call succeeds everywhere with the right answer."""
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_BARRIER_TIMEOUT_MS="60000", PG_XGMI_MODE=mode)
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    out = {"rcs": [], "fails": []}
    try:
        import ctypes

        import torch

        import pgamd
        torch.cuda.set_device(0)
        lib = pgamd.load()
        h = ctypes.c_void_p()
        assert lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) == 0
        x = torch.full((4096,), rank + 1, dtype=torch.int32, device="cuda")
        y = torch.zeros(4096, dtype=torch.int32, device="cuda")
        bad = 512 if rank == 1 else 256
        out["rcs"].append(lib.pg_reduce_scatter(x.data_ptr(), y.data_ptr(), bad, 0, 0, h))
        out["err"] = pgamd.last_error()
        out["rcs"].append(lib.pg_all_reduce(x.data_ptr(), y.data_ptr(), bad, 0, 0, h))
        out["rcs"].append(lib.pg_reduce_scatter(x.data_ptr(), y.data_ptr(), 3000, 0, 0, h))
        off, ln = pgamd.block_range(3000, world, rank)
        if not torch.equal(y[:ln].cpu(), torch.full((ln,), world * (world + 1) // 2, dtype=torch.int32)):
            out["fails"].append("wrong result after the failed calls")
        lib.pg_close(h)
    except Exception as e:
        out["fails"].append(repr(e))
    q.put((rank, out))


@pytest.mark.parametrize("mode", ["read", "push"])
def test_xgmi_count_mismatch_fails_on_every_rank(gpu, mode):
    import torch.multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mismatch_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=150))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, out in results:
        assert not out["fails"] and out["rcs"] == [-1, -1, 0], (rank, out)
        assert "counts must agree" in out["err"], (rank, out)


def _retry_worker(rank, world, port, q):
    """Rank 1's second IPC open fails (test hook PG_XGMI_FAIL_IMPORT=2).  Every
    rank must learn of it at the call's closing barrier and redo that call with
    the slot copy: every call returns 0 with the oracle's bits."""
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_BARRIER_TIMEOUT_MS="60000", PG_XGMI_FAIL_IMPORT="2" if rank == 1 else "0")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    out = {"fails": [], "errs": []}
    try:
        import ctypes

        import torch

        import pgamd
        from oracle.pyoracle import Oracle
        torch.cuda.set_device(0)
        lib = pgamd.load()
        orc = Oracle()
        h = ctypes.c_void_p()
        assert lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) == 0
        for i, coll in enumerate(("rs", "ar", "ag", "rs")):
            count = 100003
            xs = [orc.fill(count, 1, 0, 300 + 7 * i + r) for r in range(world)]
            x = torch.from_numpy(xs[rank]).cuda()
            if coll == "rs":
                want = orc.ring_reduce_scatter(xs, 1, 0)[rank]
                y = torch.zeros(want.size, dtype=torch.float64, device="cuda")
                rc = lib.pg_reduce_scatter(x.data_ptr(), y.data_ptr(), count, 1, 0, h)
            elif coll == "ar":
                want = orc.ring_all_reduce(xs, 1, 0)[rank]
                y = torch.zeros(count, dtype=torch.float64, device="cuda")
                rc = lib.pg_all_reduce(x.data_ptr(), y.data_ptr(), count, 1, 0, h)
            else:
                want = orc.ring_all_gather(xs, 1)[rank]
                y = torch.zeros(count * world, dtype=torch.float64, device="cuda")
                rc = lib.pg_all_gather(x.data_ptr(), y.data_ptr(), count, 1, h)
            out["errs"].append(pgamd.last_error())
            out.setdefault("retried", []).append(pgamd.stats(h)["retried"])
            if rc != 0 or y.cpu().numpy().tobytes() != want.tobytes():
                out["fails"].append((i, coll, rc, pgamd.last_error()))
        lib.pg_close(h)
    except Exception as e:
        out["fails"].append(("exception", repr(e)))
    q.put((rank, out))


def test_xgmi_failed_import_is_redone_with_copy(gpu):
    import torch.multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_retry_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=150))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, out in results:
        assert not out["fails"], (rank, out)
    errs = dict(results)[1]["errs"]
    assert "hipIpcOpenMemHandle" in errs[0], errs       # the injected failure happened, and was absorbed
    for rank, out in results:                           # by every rank redoing the first call, only that one
        assert out["retried"] == [1, 0, 0, 0], (rank, out["retried"])


def _probe_fail_worker(rank, world, port, q):
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_BARRIER_TIMEOUT_MS="120000", PG_XGMI_MODE="auto", PG_XGMI_FAIL_PROBE="1")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    out = {}
    try:
        import ctypes
        import time

        import torch

        import pgamd
        torch.cuda.set_device(0)
        lib = pgamd.load()
        h = ctypes.c_void_p()
        t0 = time.monotonic()
        out["rc"] = lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h))
        out["took"] = time.monotonic() - t0
        out["err"] = pgamd.last_error()
        if out["rc"] == 0:
            lib.pg_close(h)
    except Exception as e:  # noqa: BLE001
        out["exception"] = repr(e)
    q.put((rank, out))


def test_xgmi_probe_failure_fails_connect_on_every_rank_together(gpu):
    """The connect-time link probe of the auto mode: when one rank's probe launch
    fails (test hook PG_XGMI_FAIL_PROBE), that rank keeps meeting the others at
    the probe's barriers and the outcome is agreed at its end, so every rank's
    connect_process_group returns -1 within seconds -- nobody sits in a barrier
    until PG_BARRIER_TIMEOUT_MS (120 s here)."""
    import torch.multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_probe_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            results.append(q.get(timeout=200))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, out in results:
        assert out.get("rc") == -1, (rank, out)
        assert out["took"] < 60.0, (rank, out)
        assert "probe" in out["err"], (rank, out)
