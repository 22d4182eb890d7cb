"""The library's ring schedule (pg_plan.c, via its C-ABI), checked on CPU.

The plans are executed by tests/plan_sim.py (numpy, FIFO channels) and the
results compared bit-exact with the oracle's ring simulator, which is built on
the reference's own index functions and reduce loop (oracle/pg_oracle.c)."""
import itertools

import numpy as np
import pytest

import pgamd
from plan_sim import direct_reduce_scatter, ring_all_gather, ring_all_reduce, ring_reduce_scatter


def inputs(oracle, world, count, dt, op, seed):
    return [oracle.fill(count, dt, op, seed * 131 + r) for r in range(world)]


def test_block_range_matches_oracle(oracle):
    for world in range(1, 10):
        for count in (0, 1, 2, 7, 8, 9, 100, 1001):
            for b in range(world):
                assert pgamd.block_range(count, world, b) == oracle.ring_block(count, world, b)


def test_plan_rejects_bad_arguments(lib):
    assert lib.pg_plan_reduce_scatter(0, 0, 8, 0, 16, 0, 1, 2, 0, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(2, 2, 8, 0, 16, 0, 1, 2, 0, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(0, 2, -1, 0, 16, 0, 1, 2, 0, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(0, 2, 8, 9, 16, 0, 1, 2, 0, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(0, 2, 8, 0, 16, 0, 1, 5, 0, None, 0) == -1      # rings 1 .. 4
    assert lib.pg_plan_reduce_scatter(0, 2, 8, 0, 16, 0, 1, 0, 0, None, 0) == -1
    assert lib.pg_plan_all_gather(0, 2, 8, 9, 1, 2, None, 0) == -1
    assert lib.pg_plan_all_gather(0, 2, 8, 0, 1, 5, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(0, 1, 8, 0, 16, 0, 1, 2, 0, None, 0) == 0


def test_block_parts():
    for ln in (0, 1, 2, 3, 7, 8, 1001):
        assert pgamd.block_part(ln, 1, 0) == (0, ln)
        h = (ln + 1) // 2
        assert pgamd.block_part(ln, 2, 0) == (0, h)
        assert pgamd.block_part(ln, 2, 1) == (h, ln - h)
        for rings in (3, 4):
            parts = [pgamd.block_part(ln, rings, g) for g in range(rings)]
            assert parts[0][0] == 0 and sum(p[1] for p in parts) == ln
            assert all(a[0] + a[1] == b[0] for a, b in zip(parts, parts[1:]))     # contiguous
            assert parts[0][1] == -(-ln // rings) and all(p[1] <= parts[0][1] for p in parts)


def test_ring_offsets(oracle):
    # +1, -1, then +3, -3 where coprime with the world and new mod world; else repeat
    want = {2: [1, -1, 1, -1], 3: [1, -1, 1, -1], 4: [1, -1, 1, -1], 5: [1, -1, 3, -3],
            6: [1, -1, 1, -1], 7: [1, -1, 3, -3], 8: [1, -1, 3, -3], 9: [1, -1, 5, -5], 16: [1, -1, 3, -3]}
    for world, offs in want.items():
        assert [pgamd.ring_offset(world, 4, g) for g in range(4)] == offs, world
    for world in range(1, 17):
        for rings in range(1, 5):
            for g in range(rings):
                d = pgamd.ring_offset(world, rings, g)
                assert d == oracle.ring_step(world, rings, g)
                assert world == 1 or np.gcd(d % world, world) == 1


def test_plan_shape():
    # W=4, count=4096 int32, 1 KiB segments, no eager, one ring: block=1024 elems=4 KiB -> 4 segs
    st = pgamd.plan_reduce_scatter(1, 4, 4096, 0, 1024, 0, 2, rings=1)
    assert [s["round"] for s in st] == [0] * 4 + [1] * 4 + [2] * 4
    assert [s["batch"] for s in st] == [0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5]
    assert all(s["send_wait"] == (s["round"] > 0) for s in st)
    last = [s for s in st if s["round"] == 2]
    assert all(s["recv_buf"] == pgamd.PG_BUF_OUT for s in last)
    # rank 1 ends with block 1: last round receives block (1-2-2) % 4 = 1
    assert all(s["red_src_off"] == 1024 * 4 + s["recv_off"] for s in last)
    # eager: a block <= eager_max bytes is one segment
    st = pgamd.plan_reduce_scatter(0, 4, 4096, 0, 1024, 1 << 20, 4, rings=1)
    assert len(st) == 3


def test_plan_shape_two_rings():
    # same shape, two rings: each 4 KiB block splits into two 2 KiB parts of 2 segments each;
    # a batch carries 2 segment indices of each ring, clockwise first
    st = pgamd.plan_reduce_scatter(1, 4, 4096, 0, 1024, 0, 2, rings=2)
    assert len(st) == 3 * 4
    assert [s["send_peer"] for s in st[:4]] == [1, 1, -1, -1]
    assert all(s["recv_peer"] == -s["send_peer"] for s in st)
    assert [s["batch"] for s in st] == [0] * 4 + [1] * 4 + [2] * 4
    cw = [s for s in st if s["send_peer"] == 1]
    ccw = [s for s in st if s["send_peer"] == -1]
    # round 0: clockwise sends part 0 of block 0 (rank-1), counter-clockwise part 1 of block 2 (rank+1)
    assert [s["send_off"] for s in cw if s["round"] == 0] == [0, 1024]
    assert [s["send_off"] for s in ccw if s["round"] == 0] == [2 * 4096 + 2048, 2 * 4096 + 3072]
    # ring 1 stages at ceil(B/2) elements into the staging block; events do not collide
    assert all(s["recv_off"] >= 2048 for s in ccw if s["round"] == 0)
    assert {s["seg"] for s in cw}.isdisjoint({s["seg"] for s in ccw})
    # the last round lands both parts of block 1 in OUT: [0, 2 KiB) and [2 KiB, 4 KiB)
    assert sorted(s["recv_off"] for s in st if s["round"] == 2) == [0, 1024, 2048, 3072]
    assert all(s["recv_buf"] == pgamd.PG_BUF_OUT for s in st if s["round"] == 2)


@pytest.mark.parametrize("rings", [1, 2, 3, 4])
@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
def test_plan_edges_pair_up(world, rings):
    """Per directed edge, the sizes one rank sends equal, in order, the sizes its peer receives."""
    for count, dt, cb, eager, infl in itertools.product((0, 1, 9, 1000, 4099), (0, 1), (8, 100, 4096), (0, 4096), (1, 3)):
        plans = [pgamd.plan_reduce_scatter(r, world, count, dt, cb, eager, infl, rings=rings) for r in range(world)]
        for r in range(world):
            for q in range(world):
                sends = [s["send_bytes"] for s in plans[r] if s["send_bytes"] and (r + s["send_peer"]) % world == q]
                recvs = [s["recv_bytes"] for s in plans[q] if s["recv_bytes"] and (q + s["recv_peer"]) % world == r]
                assert sends == recvs, (world, r, q, count, dt, cb)


@pytest.mark.parametrize("rings", [1, 2, 3, 4])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
def test_plan_reduce_scatter_matches_oracle(oracle, world, rings):
    for dt, op, count, cb, infl in itertools.product((0, 1), (0, 1), (0, 1, 5, 64, 1001), (8, 24, 4096), (1, 4)):
        xs = inputs(oracle, world, count, dt, op, count + world)
        want = oracle.ring_reduce_scatter(xs, dt, op, rings)
        if world == 1:
            continue
        got, _ = ring_reduce_scatter(xs, dt, op, cb, eager_max=0, inflight=infl, rings=rings)
        for r in range(world):
            assert got[r].tobytes() == want[r].tobytes(), (world, r, dt, op, count, cb)


def test_two_rings_fold_order_differs_for_double(oracle):
    """Rings change which neighbour is folded first in the second half of each
    block: for doubles that is visible in the bits (so every transport must use
    the same PG_RINGS), for int32 it is not (two's complement is associative)."""
    # magnitudes spread over 2^-20 .. 2^20, so partial sums round (oracle.fill's
    # U[-1,1) multiples of 2^-52 add exactly in either order up to the last step)
    rng = np.random.default_rng(5)
    xs = [rng.standard_normal(4000) * np.exp2(rng.integers(-20, 21, 4000)) for _ in range(4)]
    a, b = oracle.ring_reduce_scatter(xs, 1, 0, 1), oracle.ring_reduce_scatter(xs, 1, 0, 2)
    assert all(x[:len(x) // 2].tobytes() == y[:len(y) // 2].tobytes() for x, y in zip(a, b))
    assert any(x.tobytes() != y.tobytes() for x, y in zip(a, b))
    bound = 2 * 3 * 2.0**-53 * sum(np.abs(v) for v in xs)       # 2 * (W-1) u * sum|x|, element-wise
    for blk, (x, y) in enumerate(zip(a, b)):
        off = blk * 1000
        assert np.all(np.abs(x - y) <= bound[off:off + 1000])
    xi = inputs(oracle, 4, 4000, 0, 1, 6)
    ai, bi = oracle.ring_reduce_scatter(xi, 0, 1, 1), oracle.ring_reduce_scatter(xi, 0, 1, 2)
    assert all(x.tobytes() == y.tobytes() for x, y in zip(ai, bi))


@pytest.mark.parametrize("rings", [1, 2, 4])
@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
def test_plan_all_reduce_in_place_matches_oracle(oracle, world, rings):
    for dt, op, count in itertools.product((0, 1), (0, 1), (1, 7, 100, 1001)):
        xs = inputs(oracle, world, count, dt, op, 99 + count)
        want = oracle.ring_all_reduce(xs, dt, op, rings)
        got = ring_all_reduce(xs, dt, op, chunk_bytes=40, eager_max=0, inflight=2, rings=rings)
        for r in range(world):
            assert got[r].tobytes() == want[r].tobytes(), (world, r, dt, op, count)


@pytest.mark.parametrize("rings", [1, 2, 3, 4])
@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_plan_all_gather_matches_oracle(oracle, world, rings):
    for dt, count in itertools.product((0, 1), (0, 1, 13, 512)):
        xs = inputs(oracle, world, count, dt, 0, 7 + count)
        want = oracle.ring_all_gather(xs, dt)
        got = ring_all_gather(xs, dt, rings)
        for r in range(world):
            assert got[r].tobytes() == want[r].tobytes()


@pytest.mark.parametrize("rings", [1, 2, 4])
def test_in_place_last_round_keeps_arrival_first(rings):
    """Only the in-place all-reduce's last round folds into SRC's own block;
    it is marked red_rev so the executor computes arrival op own like every
    other round (the left operand decides the payload of NaN op NaN)."""
    world = 5
    for alias in (0, 1):
        st = pgamd.plan_reduce_scatter(2, world, 10007, 1, 1 << 12, 0, 3, alias, rings)
        for s in st:
            last = s["round"] == world - 2
            assert s["red_rev"] == (1 if alias and last and s["red_elems"] else 0), s
            if s["red_rev"]:
                assert s["red_dst_buf"] == pgamd.PG_BUF_OUT and s["red_src_buf"] in (pgamd.PG_BUF_STAGE0,
                                                                                      pgamd.PG_BUF_STAGE1)


@pytest.mark.parametrize("rings", [1, 2, 3, 4])
@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
def test_direct_plan_matches_oracle(oracle, world, rings):
    """pg_plan_direct_reduce_scatter (PG_ALGO=direct) executed for every rank
    at once in numpy: one hop per block, every rank's groups pair up (run_plans
    asserts no deadlock and no unconsumed message) and the ring-order folds give
    the oracle ring's bits, ragged and tiny counts included."""
    for dt, op, count, cb, infl in ((0, 0, 1000, 64, 2), (1, 0, 4099, 256, 4), (1, 1, 77, 8, 1), (0, 1, 3, 4, 3),
                                    (1, 0, world * 8 + 1, 16, 1), (0, 0, 65537, 4096, 4)):
        xs = [oracle.fill(count, dt, op, 7000 + 13 * r + count) for r in range(world)]
        want = oracle.ring_reduce_scatter(xs, dt, op, rings)
        got = direct_reduce_scatter(xs, dt, op, cb, infl, rings)
        for r in range(world):
            assert got[r].tobytes() == want[r].tobytes(), (world, rings, dt, op, count, cb, infl, r)


def test_direct_plan_shape():
    """Every batch of a direct plan: transfers to/from the same peer offset,
    sends from SRC, receives into STAGE0 slot q, then the batch's folds; the
    bytes a rank sends equal its input minus its own block."""
    world, count, es = 4, 1000, 8
    for r in range(world):
        st = pgamd.plan_direct_reduce_scatter(r, world, count, 1, 64 * es, 2, 2)
        off, ln = pgamd.block_range(count, world, r)
        assert sum(s["send_bytes"] for s in st) == (count - ln) * es
        assert sum(s["recv_bytes"] for s in st) == ln * (world - 1) * es
        assert sum(s["red_elems"] for s in st if s["red_fold"]) == ln
        for s in st:
            if s["red_fold"]:
                assert not s["send_bytes"] and not s["recv_bytes"] and s["red_dst_buf"] == pgamd.PG_BUF_OUT
            else:
                assert s["send_peer"] == s["recv_peer"] and 1 <= s["send_peer"] < world
                q = (r + s["recv_peer"]) % world
                if s["recv_bytes"]:
                    assert s["recv_buf"] == pgamd.PG_BUF_STAGE0
                    assert q * 250 * es <= s["recv_off"] < (q + 1) * 250 * es


def test_plans_refuse_absurd_step_counts(lib):
    """A 4-byte segment over 2^30 elements would need billions of steps (an
    int); both planners refuse it instead of overflowing, and the collective
    reports it as a plan error."""
    assert lib.pg_plan_reduce_scatter(0, 8, (1 << 30) + 1, 0, 4, 0, 1, 2, 0, None, 0) == -1
    assert lib.pg_plan_direct_reduce_scatter(0, 8, (1 << 30) + 1, 0, 4, 1, 2, None, 0) == -1
    assert lib.pg_plan_reduce_scatter(0, 8, (1 << 30) + 1, 0, 4 << 20, 0, 4, 2, 0, None, 0) > 0
    assert lib.pg_plan_direct_reduce_scatter(0, 8, (1 << 30) + 1, 0, 4 << 20, 4, 2, None, 0) > 0


@pytest.mark.parametrize("rings", [1, 2, 4])
@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_deferred_reduce_launches_match_oracle(oracle, world, rings):
    """The executor's rule for its reduce launches (csrc/pg_exec.c,
    PG_REDUCE_BYTES), run in numpy over the library's own plans and its own
    pg_plan_coalesce: a transport group's reduce steps wait until red_bytes per
    operand are pending, or the round ends, and are reduced range by range.
    Whatever the threshold -- every group on its own, a few groups, the whole
    round -- the bits are the oracle ring's, in place too, and a larger
    threshold never means more launches."""
    for dt, op, count in itertools.product((0, 1), (0, 1), (7, 1001, 4099)):
        xs = inputs(oracle, world, count, dt, op, 500 + count)
        want_rs = oracle.ring_reduce_scatter(xs, dt, op, rings)
        want_ar = oracle.ring_all_reduce(xs, dt, op, rings)
        counts = []
        for red_bytes in (0, 96, 1000, 1 << 30):
            n = [0] * world
            got, _ = ring_reduce_scatter(xs, dt, op, 24, eager_max=0, inflight=2, rings=rings, red_bytes=red_bytes,
                                         launches_out=n)
            for r in range(world):
                assert got[r].tobytes() == want_rs[r].tobytes(), (world, rings, r, dt, op, count, red_bytes)
            counts.append(sum(n))
            got = ring_all_reduce(xs, dt, op, 24, eager_max=0, inflight=2, rings=rings, red_bytes=red_bytes)
            for r in range(world):
                assert got[r].tobytes() == want_ar[r].tobytes(), (world, rings, r, dt, op, count, red_bytes, "in place")
        assert counts == sorted(counts, reverse=True), counts
        # the whole round in one launch: at most one launch per round and rank
        assert counts[-1] <= world * (world - 1)


def test_coalesce_lists_one_range_per_ring():
    """pg_plan_coalesce on one round of a two-ring plan: the segments of each
    ring over consecutive transport groups are neighbours, so the round's
    reduce steps become at most one range per ring, covering every element once."""
    world, count, dt, es = 4, 40000, 1, 8
    plan = pgamd.plan_reduce_scatter(1, world, count, dt, 1024, 0, 2, rings=2)
    for k in range(world - 1):
        steps = [s for s in plan if s["round"] == k and s["red_elems"]]
        assert len(steps) > 8
        ranges = pgamd.plan_coalesce(list(reversed(steps)), es)          # any order in
        # one range per ring; a single one where the two rings' parts happen to be
        # neighbours in both operands (at W = 4 both rings fold the same block in rounds 0 and 2)
        assert len(ranges) == (2 if k == 1 else 1)
        assert sum(g["elems"] for g in ranges) == sum(s["red_elems"] for s in steps)
        for g in ranges:
            mine = [s for s in steps if g["dst_off"] <= s["red_dst_off"] < g["dst_off"] + g["elems"] * es
                    and s["red_dst_buf"] == g["dst_buf"]]
            assert sum(s["red_elems"] for s in mine) == g["elems"]
            assert {s["red_rev"] for s in mine} == {g["rev"]}
    assert pgamd.plan_coalesce([], es) == []
