"""pgk_all_reduce_staged (include/pgk.h): the all-reduce of pgx_sim_run for
callers that cannot allocate.  Its exchange area is a fixed device array
inside the library; the existing entry point allocates one per handle.  The
two must agree bit for bit (integer and double alike: both fold every block in
its ring's order), and both must equal the oracle ring.

Collected last (file name) so that a failure here cannot hide another test.
"""
import ctypes

import numpy as np
import pytest

import pgamd
from gpu_util import ptr, stream, to_dev, to_host

pytestmark = pytest.mark.gpu
NP = {0: np.int32, 1: np.float64}


def _staged(lib, torch, xs, count, dt, op, rings, in_place):
    world = len(xs)
    S = [to_dev(torch, x) for x in xs]
    R = S if in_place else [to_dev(torch, np.full(max(count, 1), 77, NP[dt])) for _ in xs]
    sp = (ctypes.c_void_p * world)(*[ptr(s) for s in S])
    rp = (ctypes.c_void_p * world)(*[ptr(r) for r in R])
    rc = lib.pgk_all_reduce_staged(sp, rp, world, count, rings, dt, op, stream(torch))
    assert rc == 0, pgamd.last_error()
    return [to_host(torch, r)[:count] for r in R]


def _existing(lib, torch, xs, count, dt, op, rings, in_place):
    world = len(xs)
    S = [to_dev(torch, x) for x in xs]
    R = S if in_place else [to_dev(torch, np.zeros(max(count, 1), NP[dt])) for _ in xs]
    sp = (ctypes.c_void_p * world)(*[ptr(s) for s in S])
    rp = (ctypes.c_void_p * world)(*[ptr(r) for r in R])
    rc = lib.pgx_sim_run(world, pgamd.PG_COLL_ALL_REDUCE, sp, rp, count, dt, op, 1 << 16, 4096, 4, rings)
    assert rc == 0, pgamd.last_error()
    return [to_host(torch, r)[:count] for r in R]


# two calls in a row on the shared array, the second smaller than the first
SEQUENCES = [  # world, dt, op, rings, (count of call 1, count of call 2)
    (4, 1, 0, 2, (100003, 4099)),
    (8, 0, 0, 2, (65536 + 3, 1000)),
    (3, 1, 1, 1, (4099, 7)),
    (8, 1, 0, 4, (262144, 511)),      # 8 x 2 MiB: the whole 16 MiB array, then 4 KiB
    (16, 0, 1, 3, (1001, 5)),         # count < world on the second call: empty blocks
    (2, 1, 0, 2, (1, 1)),
    (1, 1, 0, 2, (1000, 10)),         # one rank: a copy
]


@pytest.mark.parametrize("in_place", [False, True])
@pytest.mark.parametrize("seq", SEQUENCES)
def test_staged_all_reduce_matches_existing_entry_point(gpu, lib, oracle, seq, in_place):
    world, dt, op, rings, counts = seq
    for call, count in enumerate(counts):
        xs = [oracle.fill(count, dt, op, 9000 + 13 * r + count + call) for r in range(world)]
        got = _staged(lib, gpu, xs, count, dt, op, rings, in_place)
        ref = _existing(lib, gpu, xs, count, dt, op, rings, in_place)
        want = oracle.ring_all_reduce(xs, dt, op, rings)
        for r in range(world):
            assert got[r].tobytes() == ref[r].tobytes(), (seq, call, r, "vs pgx_sim_run")
            assert got[r].tobytes() == want[r].tobytes(), (seq, call, r, "vs oracle")


def test_staged_limits_and_arguments(gpu, lib):
    torch = gpu
    x = torch.zeros(16, dtype=torch.float64, device="cuda")
    one = (ctypes.c_void_p * 1)(ptr(x))
    two = (ctypes.c_void_p * 2)(ptr(x), ptr(x))
    cap = pgamd.PGK_STAGED_MAX_BYTES

    def kernel_lib_error():                     # this entry point reports through pgk_last_error()
        return (lib.pgk_last_error() or b"").decode()
    # a set-up call: count 0, no buffers needed
    assert lib.pgk_all_reduce_staged(None, None, 4, 0, 2, 1, 0, None) == 0
    # one element more than the array holds, and a world that multiplies past it
    assert lib.pgk_all_reduce_staged(one, one, 1, cap // 8 + 1, 1, 1, 0, None) == -1
    assert "exchange area" in kernel_lib_error()
    assert lib.pgk_all_reduce_staged(two, two, 2, cap // 8, 1, 1, 0, None) == -1
    assert "exchange area" in kernel_lib_error()
    assert lib.pgk_all_reduce_staged(two, two, 2, 2**61, 1, 1, 0, None) == -1
    # bad enums, world, rings, NULL lists
    assert lib.pgk_all_reduce_staged(one, one, 1, 4, 1, 2, 0, None) == -1
    assert lib.pgk_all_reduce_staged(one, one, 1, 4, 1, 1, 2, None) == -1
    assert lib.pgk_all_reduce_staged(one, one, 0, 4, 1, 1, 0, None) == -1
    assert lib.pgk_all_reduce_staged(one, one, 17, 4, 1, 1, 0, None) == -1
    assert lib.pgk_all_reduce_staged(one, one, 1, 4, 5, 1, 0, None) == -1
    assert lib.pgk_all_reduce_staged(None, one, 1, 4, 1, 1, 0, None) == -1
    torch.cuda.synchronize()


def test_staged_exact_capacity_and_free_memory(gpu, lib, oracle):
    """The largest call the array takes (1 rank x 16 MiB), on a side stream,
    with the device's free memory unchanged across the call."""
    torch = gpu
    count = pgamd.PGK_STAGED_MAX_BYTES // 4
    xs = [oracle.fill(count, 0, 0, 424242)]
    S = to_dev(torch, xs[0])
    R = torch.zeros(count, dtype=torch.int32, device="cuda")
    sp, rp = (ctypes.c_void_p * 1)(ptr(S)), (ctypes.c_void_p * 1)(ptr(R))
    side = torch.cuda.Stream()
    # a stream's first launch is where the HIP runtime sets the stream up, and that can take device memory
    # (2 MiB went at that moment in one run of the suite, whoever launches first): one small call on the
    # stream first, then the measured one
    assert lib.pgk_all_reduce_staged(sp, rp, 1, 16, 2, 0, 0, side.cuda_stream) == 0, pgamd.last_error()
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    with torch.cuda.stream(side):
        assert lib.pgk_all_reduce_staged(sp, rp, 1, count, 2, 0, 0, side.cuda_stream) == 0, pgamd.last_error()
    side.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert free1 == free0
    assert to_host(torch, R).tobytes() == xs[0].tobytes()


def test_staged_all_reduce_captured_in_hip_graph(gpu, lib, oracle):
    """What the entry point is for: captured into a hipGraph (torch.cuda.CUDAGraph
    is hipGraph on ROCm; only kernel launches are recorded, no memset nodes) and
    replayed.  The graph holds an in-place all-reduce of four buffers; every
    replay must equal the eager call on the same inputs, with eager calls of the
    same entry point (other sizes, so the shared array holds other contents) and
    synchronisations between the replays."""
    torch = gpu
    world, count, dt, op, rings = 4, 50001, 1, 0, 2
    xs = [oracle.fill(count, dt, op, 31000 + r) for r in range(world)]
    bufs = [to_dev(torch, x) for x in xs]
    ps = (ctypes.c_void_p * world)(*[ptr(b) for b in bufs])
    assert lib.pgk_all_reduce_staged(None, None, world, 0, rings, dt, op, None) == 0     # set-up, outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            sh = torch.cuda.current_stream().cuda_stream
            assert lib.pgk_all_reduce_staged(ps, ps, world, count, rings, dt, op, sh) == 0
    state = [x.copy() for x in xs]
    for rep in range(4):
        for b, v in zip(bufs, state):                 # this replay's inputs
            b.copy_(torch.from_numpy(v))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        want = oracle.ring_all_reduce(state, dt, op, rings)
        for r in range(world):
            assert to_host(torch, bufs[r]).tobytes() == want[r].tobytes(), (rep, r)
        # eager work of the program's own between the replays, on the same shared array
        small = [oracle.fill(777 + rep, 0, 1, 32000 + 5 * rep + r) for r in range(3)]
        got = _staged(lib, torch, small, 777 + rep, 0, 1, 1, False)
        ref = oracle.ring_all_reduce(small, 0, 1, 1)
        for r in range(3):
            assert got[r].tobytes() == ref[r].tobytes(), (rep, r, "eager between replays")
        state = [oracle.fill(count, dt, op, 33000 + 10 * rep + r) for r in range(world)]


def test_staged_all_reduce_special_values_match_existing_entry_point(gpu, lib, oracle):
    """NaNs with payloads, infinities, signed zeros, denormals and DBL_MAX
    scattered through every rank's input, sum and product, 1-4 rings: the bits
    (NaN payloads included: both entry points fold every block in the same
    order, the arrival on the left) equal pgx_sim_run's, and the int32
    wrap cases equal the oracle's."""
    rng = np.random.default_rng(99)
    specials = np.array([0x7FF8000000000001, 0xFFF800000000BEEF, 0x7FF0000000000000, 0xFFF0000000000000,
                         0x0000000000000000, 0x8000000000000000, 0x0000000000000001, 0x800FFFFFFFFFFFFF,
                         0x7FEFFFFFFFFFFFFF, 0xFFEFFFFFFFFFFFFF, 0x3FF0000000000000, 0xBFF0000000000000], dtype=np.uint64)
    for world, count, rings in ((4, 4099, 2), (8, 1001, 4), (3, 77, 1), (5, 300, 3)):
        for op in (0, 1):
            xs = []
            for r in range(world):
                x = oracle.fill(count, 1, op, 41000 + r).view(np.uint64).copy()
                where = rng.random(count) < 0.3
                x[where] = rng.choice(specials, int(where.sum()))
                xs.append(x.view(np.float64))
            got = _staged(lib, gpu, xs, count, 1, op, rings, True)
            ref = _existing(lib, gpu, xs, count, 1, op, rings, True)
            for r in range(world):
                assert got[r].tobytes() == ref[r].tobytes(), (world, count, rings, op, r)
    big = np.array([2**31 - 1, -2**31, 65536, -123456789, 987654, 1, -1, 0] * 64, dtype=np.int32)
    xs = [np.roll(big, 3 * r).copy() for r in range(4)]
    for op in (0, 1):
        got = _staged(lib, gpu, xs, big.size, 0, op, 2, False)
        want = oracle.ring_all_reduce(xs, 0, op, 2)
        for r in range(4):
            assert got[r].tobytes() == want[r].tobytes(), (op, r)
