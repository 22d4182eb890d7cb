"""BASELINE configs 3 and 4 at their full sizes through the real ring executor
and the direct exchange (PG_ALGO=direct, the rccl transport's default on one
node) -- W virtual ranks on the one test GPU: PG_TRANSPORT_THREADS keeps the
plan, executor, streams, events, staging and the gfx950 kernels of the RCCL
path and replaces only the hop by a device copy.

At these sizes the C oracle would need minutes, so the expected blocks are
computed on the GPU with torch from the same inputs, in the fold order the
oracle restates (orc_ring_step, part g of block b: x[b+d] op x[b+2d] op ...
op x[b]): one IEEE operation per element and step, so double results are
compared bit for bit; int32 wraps in two's complement on both sides.

  config 3: 4 ranks, int32 sum, 1 GiB per rank, 256 MiB blocks
  config 4: 8 ranks, double sum, 4 GiB per rank, 512 MiB blocks (2 and 4 rings)
  config 5: 8 ranks, int32 / double product, 4 KiB calls around 2 GiB calls
"""
import ctypes

import pytest

import pgamd
from gpu_util import ptr

pytestmark = pytest.mark.gpu


def _expected_block(torch, xs, b, off, ln, rings, world, op, oracle):
    out = torch.empty(ln, dtype=xs[0].dtype, device="cuda")
    for g in range(rings):
        lo, hi = -(-g * ln // rings), -(-(g + 1) * ln // rings)
        if lo == hi:
            continue
        d = oracle.ring_step(world, rings, g) % world
        acc = xs[(b + d) % world][off + lo:off + hi].clone()
        for j in range(2, world + 1):
            src = xs[(b + j * d) % world][off + lo:off + hi]
            if op == pgamd.OP_SUM:
                acc.add_(src)
            else:
                acc.mul_(src)
        out[lo:hi] = acc
    return out


@pytest.mark.parametrize("world,dt,count,rings,algo", [
    (4, pgamd.DT_INT32, 1 << 28, 2, "ring"),        # config 3
    (8, pgamd.DT_DOUBLE, 1 << 29, 2, "ring"),       # config 4
    (8, pgamd.DT_DOUBLE, 1 << 29, 4, "ring"),       # config 4 over four rings
    (4, pgamd.DT_INT32, 1 << 28, 2, "direct"),      # config 3, direct exchange
    (8, pgamd.DT_DOUBLE, 1 << 29, 2, "direct"),     # config 4, direct exchange
])
def test_baseline_config_full_size(gpu, lib, oracle, monkeypatch, world, dt, count, rings, algo):
    monkeypatch.setenv("PG_ALGO", algo)
    torch = gpu
    g = torch.Generator(device="cuda").manual_seed(31 * world + rings)
    if dt == pgamd.DT_INT32:
        xs = [torch.randint(-2**31, 2**31 - 1, (count,), dtype=torch.int32, device="cuda", generator=g)
              for _ in range(world)]
    else:
        xs = [torch.rand(count, dtype=torch.float64, device="cuda", generator=g) * 2 - 1 for _ in range(world)]
    outs = []
    for r in range(world):
        _, ln = pgamd.block_range(count, world, r)
        outs.append(torch.empty(max(ln, 1), dtype=xs[0].dtype, device="cuda"))
    torch.cuda.synchronize()
    sp = (ctypes.c_void_p * world)(*[ptr(x) for x in xs])
    rp = (ctypes.c_void_p * world)(*[ptr(o) for o in outs])
    rc = lib.pgx_sim_run(world, pgamd.PG_COLL_REDUCE_SCATTER, sp, rp, count, dt, pgamd.OP_SUM, 4 << 20, 4096, 4,
                         rings)
    assert rc == 0, pgamd.last_error()
    for r in range(world):
        off, ln = pgamd.block_range(count, world, r)
        want = _expected_block(torch, xs, r, off, ln, rings, world, pgamd.OP_SUM, oracle)
        got = outs[r][:ln]
        if dt == pgamd.DT_DOUBLE:                 # bits, not values (-0.0 == 0.0)
            got, want = got.view(torch.int64), want.view(torch.int64)
        assert torch.equal(got, want), (world, dt, rings, r)
        del want
    del xs, outs
    torch.cuda.empty_cache()


@pytest.mark.parametrize("algo", ["ring", "direct"])
def test_baseline_config5_sequence(gpu, lib, oracle, monkeypatch, algo):
    """config 5: 8 ranks, int32 and double products, eager-size calls (4 KiB)
    interleaved with 2 GiB calls on one set of handles (pgx_sim_run opens
    fresh ones per call; the eager one-shot path and the ring or the direct
    exchange both run)."""
    monkeypatch.setenv("PG_ALGO", algo)
    torch = gpu
    world = 8
    g = torch.Generator(device="cuda").manual_seed(55)
    for dt, big in ((pgamd.DT_DOUBLE, 1 << 28), (pgamd.DT_INT32, 1 << 29)):
        small = 4096 // pgamd.ELEM_SIZE[dt]
        for count in (small, big, small):
            if dt == pgamd.DT_INT32:
                xs = [torch.randint(-2**31, 2**31 - 1, (count,), dtype=torch.int32, device="cuda", generator=g)
                      for _ in range(world)]
            else:   # 1 + U[-2^-10, 2^-10): stays normal over 8 factors
                xs = [1 + (torch.rand(count, dtype=torch.float64, device="cuda", generator=g) * 2 - 1) * 2.0**-10
                      for _ in range(world)]
            outs = [torch.empty(max(pgamd.block_range(count, world, r)[1], 1), dtype=xs[0].dtype, device="cuda")
                    for r in range(world)]
            torch.cuda.synchronize()
            sp = (ctypes.c_void_p * world)(*[ptr(x) for x in xs])
            rp = (ctypes.c_void_p * world)(*[ptr(o) for o in outs])
            rc = lib.pgx_sim_run(world, pgamd.PG_COLL_REDUCE_SCATTER, sp, rp, count, dt, pgamd.OP_PROD, 4 << 20,
                                 4096, 4, 2)
            assert rc == 0, pgamd.last_error()
            for r in range(world):
                off, ln = pgamd.block_range(count, world, r)
                want = _expected_block(torch, xs, r, off, ln, 2, world, pgamd.OP_PROD, oracle)
                got = outs[r][:ln]
                if dt == pgamd.DT_DOUBLE:
                    got, want = got.view(torch.int64), want.view(torch.int64)
                assert torch.equal(got, want), (dt, count, r)
            del xs, outs
            torch.cuda.empty_cache()


@pytest.mark.parametrize("algo", ["ring", "direct"])
def test_maximum_count_ring(gpu, lib, oracle, monkeypatch, algo):
    """The API's largest count (INT_MAX int32 elements, 8 GiB per rank) through
    the 2-rank ring and the direct exchange: every byte offset of the plan and
    executor past 2^31 and 2^32, the ragged second block (one element
    shorter), both rings."""
    monkeypatch.setenv("PG_ALGO", algo)
    torch = gpu
    world, count = 2, (1 << 31) - 1
    g = torch.Generator(device="cuda").manual_seed(77)
    xs = [torch.randint(-2**31, 2**31 - 1, (count,), dtype=torch.int32, device="cuda", generator=g)
          for _ in range(world)]
    outs = [torch.empty(pgamd.block_range(count, world, r)[1], dtype=torch.int32, device="cuda")
            for r in range(world)]
    torch.cuda.synchronize()
    sp = (ctypes.c_void_p * world)(*[ptr(x) for x in xs])
    rp = (ctypes.c_void_p * world)(*[ptr(o) for o in outs])
    rc = lib.pgx_sim_run(world, pgamd.PG_COLL_REDUCE_SCATTER, sp, rp, count, pgamd.DT_INT32, pgamd.OP_SUM,
                         64 << 20, 4096, 4, 2)
    assert rc == 0, pgamd.last_error()
    for r in range(world):
        off, ln = pgamd.block_range(count, world, r)
        want = _expected_block(torch, xs, r, off, ln, 2, world, pgamd.OP_SUM, oracle)
        assert torch.equal(outs[r], want), r
    del xs, outs
    torch.cuda.empty_cache()
