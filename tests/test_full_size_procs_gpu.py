"""The W > 1 transports at BASELINE's full sizes with REAL processes (one rank
per process, all on the test box's one GPU): the default one-node transport
(PG_TRANSPORT=xgmi) and the RCCL transport (its direct exchange, the one-node
default, and the two-ring P2P ring; RCCL carries the hops over its socket
transport here, one NCCL_HOSTID per rank, as in tests/test_rccl_gpu.py):

  config 3: 4 ranks, int32 sum, 1 GiB per rank (count 2^28)
  config 4: 8 ranks, double sum, 4 GiB per rank (count 2^29)
  config 5: 8 ranks, double / int32 product, 4 KiB calls around 2 GiB calls
  the API's largest count: 2 ranks, int32 sum, INT_MAX elements (8 GiB per rank)
  pg_all_reduce at configs 3 and 4's sizes, on both transports

xgmi in the auto mode (the library's default: read or push, chosen at connect
by the link probe) and with push forced.  At these sizes the C oracle would need
minutes, so each rank computes its expected block on the GPU from the same
inputs, in the fold order the oracle restates (orc_ring_step, part g of block
b: x[b+d] op x[b+2d] op ... op x[b]), one IEEE operation per element and step,
as tests/test_full_size_gpu.py does for the ring executor.  Every rank makes
every rank's input from a counter-based formula of (rank, index), so no input
crosses processes except through the transport.  The doubles carry full
53-bit mantissas, so a different fold order would change their bits.

That GPU-side expectation is itself a restatement, so it is pinned to the C
oracle where the oracle is affordable: for every checked block, windows at the
start and the end of every ring part (the part boundaries included) are folded
on the host by the oracle's own reduce loop (orc_reduce_inplace, the
restatement of reference src/pg.c:151-159) in the ring order orc_ring_step
gives, from inputs regenerated for just those windows, and compared with the
transport's output bit for bit."""
import os
import pathlib
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]
CHUNK = 1 << 26          # elements generated per step (bounds the int64 index temporaries)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fill(torch, out, q, off, dt, op):
    """out[k] = rank q's input at index off + k (deterministic, chunked)."""
    n = out.numel()
    for lo in range(0, n, CHUNK):
        hi = min(n, lo + CHUNK)
        i = torch.arange(off + lo, off + hi, dtype=torch.int64, device="cuda")
        h1 = (i * 2654435761 + (q + 1) * 40503) & 0xFFFFFFFF
        h2 = (i * 2246822519 + (q + 7) * 97) & 0xFFFFFFFF
        if dt == 0:                           # int32: the full range, wrapping sums and products
            out[lo:hi] = (h1 - (h1 >= 2**31).to(torch.int64) * 2**32).to(torch.int32)
        elif op == 0:                         # double sum: full mantissas in [-1, 1)
            out[lo:hi] = (h1.double() / 2**31 - 1) * (1 + h2.double() / 2**33)
        else:                                 # double product: 1 + [-2^-10, 2^-10), normal over 8 factors
            out[lo:hi] = 1 + (h1.double() / 2**31 - 1) * (1 + h2.double() / 2**33) * 2.0**-10
        del i, h1, h2


def _expected(torch, world, rank, count, dt, op, rings, ring_step, block_range):
    off, ln = block_range(count, world, rank)
    tdt = torch.int32 if dt == 0 else torch.float64
    parts = [torch.empty(ln, dtype=tdt, device="cuda") for _ in range(world)]
    for q in range(world):
        _fill(torch, parts[q], q, off, dt, op)
    out = torch.empty(ln, dtype=tdt, device="cuda")
    for g in range(rings):
        lo, hi = -(-g * ln // rings), -(-(g + 1) * ln // rings)
        if lo == hi:
            continue
        d = ring_step(world, rings, g) % world
        acc = parts[(rank + d) % world][lo:hi].clone()
        for j in range(2, world + 1):
            src = parts[(rank + j * d) % world][lo:hi]
            if op == 0:
                acc.add_(src)
            else:
                acc.mul_(src)
        out[lo:hi] = acc
        del acc
    del parts
    return out


WINDOW = 1 << 15         # elements per oracle-checked window


def _oracle_windows(ln, rings):
    """(lo, hi, ring part) windows of a block of ln elements: the first and the
    last WINDOW elements of every ring part."""
    wins = []
    for g in range(rings):
        lo, hi = -(-g * ln // rings), -(-(g + 1) * ln // rings)
        if lo == hi:
            continue
        wins.append((lo, min(hi, lo + WINDOW), g))
        if hi - lo > WINDOW:
            wins.append((hi - WINDOW, hi, g))
    return wins


def _oracle_check(torch, orc, got_block, world, b, boff, bln, dt, op, rings):
    """Windows of block b of the transport's output against the C oracle's fold
    of the same windows of every rank's input.  Returns the windows that differ."""
    tdt = torch.int32 if dt == 0 else torch.float64
    bad = []
    for lo, hi, g in _oracle_windows(bln, rings):
        d = orc.ring_step(world, rings, g) % world
        win = torch.empty(hi - lo, dtype=tdt, device="cuda")
        acc = None
        for j in range(1, world + 1):                  # x[b+d] op x[b+2d] op ... op x[b]
            _fill(torch, win, (b + j * d) % world, boff + lo, dt, op)
            xq = win.cpu().numpy()
            acc = xq.copy() if acc is None else orc.reduce(acc, xq, dt, op)
        if got_block[lo:hi].cpu().numpy().tobytes() != acc.tobytes():
            bad.append((lo, hi, g))
    return bad


def _env(transport, rank, port, mode=None, algo=None):
    env = dict(PG_TRANSPORT=transport, PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
               PG_CONNECT_TIMEOUT_MS="120000", PG_BARRIER_TIMEOUT_MS="120000", PG_XGMI_MODE=mode, PG_ALGO=algo)
    if transport == "rccl":
        env.update(NCCL_HOSTID=f"pg-full-size-{port}-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    return env


def _worker(rank, world, port, q, calls, transport, mode, algo):
    for k, v in _env(transport, rank, port, mode, algo).items():
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
        if lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) != 0:
            q.put((rank, ["connect: " + pgamd.last_error()]))
            return
        rings = int(os.environ.get("PG_RINGS", "2"))
        for i, call in enumerate(calls):
            coll, (dt, op, count) = (call[0], call[1:]) if isinstance(call[0], str) else ("rs", call)
            tdt = torch.int32 if dt == 0 else torch.float64
            x = torch.empty(count, dtype=tdt, device="cuda")
            _fill(torch, x, rank, 0, dt, op)
            off, ln = pgamd.block_range(count, world, rank)
            out = torch.empty(max(ln, 1) if coll == "rs" else count, dtype=tdt, device="cuda")
            torch.cuda.synchronize()
            fn = lib.pg_reduce_scatter if coll == "rs" else lib.pg_all_reduce
            if fn(x.data_ptr(), out.data_ptr(), count, dt, op, h) != 0:
                fails.append((i, "rc", pgamd.last_error()))
                break
            del x
            # reduce-scatter: this rank's block; all-reduce: every block, in its own ring order
            for b in ([rank] if coll == "rs" else range(world)):
                boff, bln = pgamd.block_range(count, world, b)
                want = _expected(torch, world, b, count, dt, op, rings, orc.ring_step, pgamd.block_range)
                got = out[:bln] if coll == "rs" else out[boff:boff + bln]
                bad_windows = _oracle_check(torch, orc, got, world, b, boff, bln, dt, op, rings)
                if bad_windows:
                    fails.append((i, coll, dt, op, count, b, "differs from the C oracle in windows", bad_windows))
                if dt == 1:                          # bits, not values (-0.0 == 0.0)
                    got, want = got.view(torch.int64), want.view(torch.int64)
                if not torch.equal(got, want):
                    bad = int((got != want).sum())
                    fails.append((i, coll, dt, op, count, b, f"{bad} of {bln} elements differ"))
                del want, got
            st = pgamd.stats(h)
            if st["calls_redone"]:
                fails.append((i, "call redone with the slot copy"))
            del out
            torch.cuda.empty_cache()
        lib.pg_close(h)
    except Exception as e:  # report, never hang the parent
        fails.append(("exception", repr(e)))
    q.put((rank, fails))


def _run(world, calls, mode=None, transport="xgmi", algo=None, timeout=280):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, calls, transport, mode, algo)) for r in range(world)]
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


@pytest.mark.parametrize("mode", [None, "push"])
def test_xgmi_config3_full_size(gpu, mode):
    _run(4, [(0, 0, 1 << 28)], mode)


@pytest.mark.parametrize("mode", [None, "push"])
def test_xgmi_config4_full_size(gpu, mode):
    _run(8, [(1, 0, 1 << 29)], mode)


@pytest.mark.parametrize("transport", ["xgmi", "rccl"])
def test_all_reduce_full_size(gpu, transport):
    """pg_all_reduce at configs 3 and 4's sizes (1 GiB int32 over 4 ranks, 4 GiB
    double over 8): every rank checks every block of its result, each block in
    its own ring order (the order the reduce-scatter folds it in)."""
    _run(4, [("ar", 0, 0, 1 << 28)], transport=transport)
    _run(8, [("ar", 1, 0, 1 << 29)], transport=transport)


def test_xgmi_config5_sequence(gpu):
    """double and int32 products: 4 KiB (eager size), 2 GiB, 4 KiB, on one handle per process."""
    calls = []
    for dt, big in ((1, 1 << 28), (0, 1 << 29)):
        small = 4096 // (8 if dt == 1 else 4)
        calls += [(dt, 1, small), (dt, 1, big), (dt, 1, small)]
    _run(8, calls)


def test_xgmi_maximum_count(gpu):
    """INT_MAX int32 elements per rank (8 GiB): every offset past 2^31 and 2^32
    bytes, the ragged second block (one element shorter)."""
    _run(2, [(0, 0, (1 << 31) - 1)])


@pytest.mark.parametrize("algo", [None, "ring"])
def test_rccl_config3_full_size(gpu, algo):
    """config 3 over RCCL: the direct exchange (default) and the two-ring P2P ring."""
    _run(4, [(0, 0, 1 << 28)], transport="rccl", algo=algo)


def test_rccl_config4_full_size(gpu):
    """config 4 over RCCL's direct exchange (the one-node default)."""
    _run(8, [(1, 0, 1 << 29)], transport="rccl")
