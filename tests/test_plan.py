"""The library's ring schedule (pg_plan.c, via its C-ABI), checked on CPU.

The plans are executed by tests/plan_sim.py (numpy, FIFO channels) and the
results compared bit-exact with the oracle's ring simulator, which is built on
the reference's own index functions and reduce loop (oracle/pg_oracle.c)."""
import itertools

import numpy as np
import pytest

import pgamd
from plan_sim import ring_all_gather, ring_all_reduce, ring_reduce_scatter


def inputs(oracle, world, count, dt, op, seed):
    return [oracle.fill(count, dt, op, seed * 131 + r) for r in range(world)]


def test_block_range_matches_oracle(oracle):
    for world in range(1, 10):
        for count in (0, 1, 2, 7, 8, 9, 100, 1001):
            for b in range(world):
                assert pgamd.block_range(count, world, b) == oracle.ring_block(count, world, b)


def test_plan_rejects_bad_arguments(lib):
    assert lib.pg_plan_reduce_scatter(0, 0, 8, 0, 16, 0, 1, 0, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(2, 2, 8, 0, 16, 0, 1, 0, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(0, 2, -1, 0, 16, 0, 1, 0, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(0, 2, 8, 9, 16, 0, 1, 0, None, 0) == -1
    assert lib.pg_plan_all_gather(0, 2, 8, 9, 1, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(0, 1, 8, 0, 16, 0, 1, 0, None, 0) == 0


def test_plan_shape():
    # W=4, count=4096 int32, 1 KiB segments, no eager: 3 rounds x 1 segment... block=1024 elems=4 KiB -> 4 segs
    st = pgamd.plan_reduce_scatter(1, 4, 4096, 0, 1024, 0, 2)
    assert [s["round"] for s in st] == [0] * 4 + [1] * 4 + [2] * 4
    assert [s["batch"] for s in st] == [0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5]
    assert all(s["send_wait"] == (s["round"] > 0) for s in st)
    last = [s for s in st if s["round"] == 2]
    assert all(s["recv_buf"] == pgamd.PG_BUF_OUT for s in last)
    # rank 1 ends with block 1: last round receives block (1-2-2) % 4 = 1
    assert all(s["red_src_off"] == 1024 * 4 + s["recv_off"] for s in last)
    # eager: a block <= eager_max bytes is one segment
    st = pgamd.plan_reduce_scatter(0, 4, 4096, 0, 1024, 1 << 20, 4)
    assert len(st) == 3


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
def test_plan_edges_pair_up(world):
    for count, dt, cb, eager, infl in itertools.product((0, 1, 9, 1000, 4099), (0, 1), (8, 100, 4096), (0, 4096), (1, 3)):
        plans = [pgamd.plan_reduce_scatter(r, world, count, dt, cb, eager, infl) for r in range(world)]
        for r in range(world):
            sends = [s["send_bytes"] for s in plans[r] if s["send_bytes"]]
            recvs = [s["recv_bytes"] for s in plans[(r + 1) % world] if s["recv_bytes"]]
            assert sends == recvs, (world, r, count, dt, cb)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_plan_reduce_scatter_matches_oracle(oracle, world):
    for dt, op, count, cb, infl in itertools.product((0, 1), (0, 1), (0, 1, 5, 64, 1001), (8, 24, 4096), (1, 4)):
        xs = inputs(oracle, world, count, dt, op, count + world)
        want = oracle.ring_reduce_scatter(xs, dt, op)
        if world == 1:
            continue
        got, _ = ring_reduce_scatter(xs, dt, op, cb, eager_max=0, inflight=infl)
        for r in range(world):
            assert got[r].tobytes() == want[r].tobytes(), (world, r, dt, op, count, cb)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_plan_all_reduce_in_place_matches_oracle(oracle, world):
    for dt, op, count in itertools.product((0, 1), (0, 1), (1, 7, 100, 1001)):
        xs = inputs(oracle, world, count, dt, op, 99 + count)
        want = oracle.ring_all_reduce(xs, dt, op)
        got = ring_all_reduce(xs, dt, op, chunk_bytes=40, eager_max=0, inflight=2)
        for r in range(world):
            assert got[r].tobytes() == want[r].tobytes(), (world, r, dt, op, count)


@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_plan_all_gather_matches_oracle(oracle, world):
    for dt, count in itertools.product((0, 1), (0, 1, 13, 512)):
        xs = inputs(oracle, world, count, dt, 0, 7 + count)
        want = oracle.ring_all_gather(xs, dt)
        got = ring_all_gather(xs, dt)
        for r in range(world):
            assert got[r].tobytes() == want[r].tobytes()
