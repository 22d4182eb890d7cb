"""gfx950 reduction kernel (include/pgk.h) against the reference's own outputs.

Golden vectors come from the reference's compiled reduce_inplace
(src/pg.c:151-159, tests/golden/); larger inputs are checked against the CPU
oracle (a restatement pinned to the same vectors).  int32 and double:
bit-exact, NaN results included (measured: gfx950 produces the same default
NaN 0xfff8000000000000 for inf-inf / 0*inf as x86 SSE and propagates NaN
payloads the same way)."""
import hashlib
import itertools

import numpy as np
import pytest

import pgamd
from gpu_util import ptr, same_bits_nan_aware, stream, to_dev, to_host

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run(lib, torch, d0, s, dt, op):
    d, sd = to_dev(torch, d0), to_dev(torch, s)
    assert lib.pgk_reduce(ptr(d), ptr(sd), d0.size, dt, op, stream(torch)) == 0
    return to_host(torch, d)


def test_kernel_kats(gpu, lib, golden, oracle):
    man, arr = golden
    for c in man["kernel"]:
        d0 = oracle.fill(c["n"], c["dt"], c["op"], c["seed_dst"])
        s = oracle.fill(c["n"], c["dt"], c["op"], c["seed_src"])
        assert sha(d0) == c["sha_dst0"]
        out = run(lib, gpu, d0, s, c["dt"], c["op"])
        assert sha(out) == c["sha_out"], c
        if c["stored"]:
            assert out.tobytes() == arr[c["key"] + "_out"].tobytes()


def test_special_values(gpu, lib, golden):
    man, arr = golden
    for c in man["specials"]:
        k = c["key"]
        out = run(lib, gpu, arr[k + "_dst0"], arr[k + "_src"], c["dt"], c["op"])
        assert same_bits_nan_aware(out, arr[k + "_out"]), k      # NaN-ness first, for a readable failure
        assert out.tobytes() == arr[k + "_out"].tobytes(), k      # then every bit, NaNs included
        if c["dt"] == 1:  # denormals must survive (no flush-to-zero)
            want = arr[k + "_out"]
            sub = (want != 0) & (np.abs(want) < np.finfo(np.float64).tiny)
            assert sub.any() and np.array_equal(out[sub], want[sub])


@pytest.mark.parametrize("dt", [0, 1])
@pytest.mark.parametrize("op", [0, 1])
def test_offsets_and_ragged_lengths(gpu, lib, oracle, dt, op):
    """Head/tail peeling (pointers congruent mod 16 B) and the scalar path
    (not congruent), for every small offset pair and ragged length."""
    torch = gpu
    base = 4096 + 9
    d_all = oracle.fill(base + 8, dt, op, 11)
    s_all = oracle.fill(base + 8, dt, op, 12)
    D, S = to_dev(torch, d_all), to_dev(torch, s_all)
    es = 4 if dt == 0 else 8
    for od in range(4):
        for os_ in range(4):
            for n in (0, 1, 2, 3, 5, 17, 255, 1024, 4099):
                D.copy_(torch.from_numpy(d_all))
                assert lib.pgk_reduce(ptr(D) + od * es, ptr(S) + os_ * es, n, dt, op, stream(torch)) == 0
                got = to_host(torch, D)
                want = d_all.copy()
                want[od:od + n] = oracle.reduce(d_all[od:od + n], s_all[os_:os_ + n], dt, op)
                assert got.tobytes() == want.tobytes(), (od, os_, n)


def test_reduce_out_and_aliasing(gpu, lib, oracle):
    torch = gpu
    for dt in (0, 1):
        for op in (0, 1):
            n = 100003
            a, b = oracle.fill(n, dt, op, 5), oracle.fill(n, dt, op, 6)
            want = oracle.reduce(a, b, dt, op)
            A, B, O = to_dev(torch, a), to_dev(torch, b), to_dev(torch, np.zeros_like(a))
            assert lib.pgk_reduce_out(ptr(O), ptr(A), ptr(B), n, dt, op, stream(torch)) == 0
            assert to_host(torch, O).tobytes() == want.tobytes()
            assert to_host(torch, A).tobytes() == a.tobytes()          # inputs untouched
            assert lib.pgk_reduce_out(ptr(B), ptr(A), ptr(B), n, dt, op, stream(torch)) == 0   # out == b
            assert to_host(torch, B).tobytes() == want.tobytes()
    # dst == src: d = d op d
    x = oracle.fill(4097, 1, 0, 9)
    X = to_dev(torch, x)
    assert lib.pgk_reduce(ptr(X), ptr(X), x.size, 1, 0, stream(torch)) == 0
    assert to_host(torch, X).tobytes() == oracle.reduce(x, x, 1, 0).tobytes()


@pytest.mark.parametrize("blocks_per_cu,nt,shape", [(0, 0, (256, 4)), (0, 1, (512, 2)), (4, 0, (1024, 1)),
                                                    (8, 1, (256, 8)), (1, 1, (256, 2)), (3, 1, (512, 2))])
def test_tuning_variants_agree(gpu, lib, oracle, blocks_per_cu, nt, shape):
    torch = gpu
    try:
        assert lib.pgk_tune(blocks_per_cu, nt) == 0
        assert lib.pgk_tune_shape(*shape) == 0
        for n in ((1 << 20) + 3, 4099, 77):
            for dt in (0, 1):
                a, b = oracle.fill(n, dt, 0, 21), oracle.fill(n, dt, 0, 22)
                assert run(lib, torch, a, b, dt, 0).tobytes() == oracle.reduce(a, b, dt, 0).tobytes()
    finally:
        lib.pgk_tune(0, 1)
        lib.pgk_tune_shape(0, 0)
    assert lib.pgk_tune_shape(256, 3) == -1


def test_timed_launch_events(gpu, lib, oracle):
    import ctypes
    torch = gpu
    n = 1 << 22
    a, b = oracle.fill(n, 1, 0, 41), oracle.fill(n, 1, 0, 42)
    A, B = to_dev(torch, a), to_dev(torch, b)
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.pgk_event_create(ctypes.byref(e0)) == 0 and lib.pgk_event_create(ctypes.byref(e1)) == 0
    assert lib.pgk_reduce_timed(ptr(A), ptr(B), n, 1, 0, stream(torch), e0, e1) == 0
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    assert lib.pgk_event_elapsed_ms(e0, e1, ctypes.byref(ms)) == 0 and 0 < ms.value < 100
    assert to_host(torch, A).tobytes() == oracle.reduce(a, b, 1, 0).tobytes()
    lib.pgk_event_destroy(e0)
    lib.pgk_event_destroy(e1)


def test_full_size_config2(gpu, lib, oracle):
    """BASELINE config 2 size: 256 MiB double sum (and int32 prod at 256 MiB),
    compared element-for-element with the oracle."""
    torch = gpu
    for dt, op, n in ((1, 0, 1 << 25), (0, 1, 1 << 26)):
        a, b = oracle.fill(n, dt, op, 31), oracle.fill(n, dt, op, 32)
        got = run(lib, torch, a, b, dt, op)
        assert got.tobytes() == oracle.reduce(a, b, dt, op).tobytes()
        del got
        torch.cuda.empty_cache()


@pytest.mark.parametrize("nbytes", [512 << 20, (512 << 20) + 8, (1 << 30) + 24])
def test_split_launches(gpu, lib, oracle, nbytes):
    """Above 512 MiB per operand pgk_reduce is several back-to-back launches of
    at most 512 MiB (kSplitBytes in pgk_reduce.hip): exactly 512 MiB stays one
    launch, 512 MiB + 8 B is two, 1 GiB + 24 B three.  Every element against the
    oracle, the head element (one element past the 16-B phase) and the bytes
    around the range untouched, and the stamped form brackets all the pieces."""
    import ctypes
    torch = gpu
    for dt, op in ((1, 0), (0, 1)):
        es = 4 if dt == 0 else 8
        n = nbytes // es
        a, b = oracle.fill(n + 2, dt, op, 61), oracle.fill(n + 2, dt, op, 62)
        d, s = to_dev(torch, a), to_dev(torch, b)
        e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
        assert lib.pgk_event_create(ctypes.byref(e0)) == 0 and lib.pgk_event_create(ctypes.byref(e1)) == 0
        assert lib.pgk_reduce_timed(ptr(d) + es, ptr(s) + es, n, dt, op, stream(torch), e0, e1) == 0
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        assert lib.pgk_event_elapsed_ms(e0, e1, ctypes.byref(ms)) == 0
        assert 3 * nbytes / (ms.value * 1e-3) < 8.0e12 * 1.05, ms.value     # the stamps bracket every piece
        lib.pgk_event_destroy(e0)
        lib.pgk_event_destroy(e1)
        got = to_host(torch, d)
        want = a.copy()
        want[1:n + 1] = oracle.reduce(a[1:n + 1], b[1:n + 1], dt, op)
        assert got.tobytes() == want.tobytes(), (dt, op, nbytes)
        del d, s, got, want
        torch.cuda.empty_cache()


@pytest.mark.parametrize("nbytes", [(128 << 20) - 16, 128 << 20, (160 << 20) + 24, (256 << 20) - 8, 256 << 20])
def test_default_shape_boundaries(gpu, lib, oracle, nbytes):
    """Each size-chosen vector shape (shape_for in pgk_reduce.hip: 512x2 below
    128 MiB per operand, 256x4 up to 256 MiB, 1024x1 above) at and around its
    boundaries, with a ragged tail and a partial last tile, against the oracle;
    the double sums start one element past the 16-B phase (head element)."""
    torch = gpu
    for dt, op in ((1, 0), (0, 1)):
        es = 4 if dt == 0 else 8
        n = nbytes // es
        a, b = oracle.fill(n + 1, dt, op, 41), oracle.fill(n + 1, dt, op, 42)
        off = 1 if dt == 1 else 0
        d, s = to_dev(torch, a), to_dev(torch, b)
        assert lib.pgk_reduce(ptr(d) + off * es, ptr(s) + off * es, n, dt, op, stream(torch)) == 0
        got = to_host(torch, d)
        want = a.copy()
        want[off:off + n] = oracle.reduce(a[off:off + n], b[off:off + n], dt, op)
        assert got.tobytes() == want.tobytes(), (dt, op, nbytes)
        del d, s, got
        torch.cuda.empty_cache()


def test_maximum_counts(gpu, lib):
    """The API's largest count (INT_MAX elements, include/pg.h `int count`) on the
    vector path and on the element-wise path (dst one element off src's 16-B
    phase), then an element-wise launch over 2^32 + 3 int32 (16 GiB operands)
    whose grid is capped at 2^32 work-items and grid-strides over the rest:
    every element is reduced exactly once, nothing past n is touched."""
    torch = gpu
    n = (1 << 31) - 1
    d = torch.full((n + 2,), 1, dtype=torch.int32, device="cuda")
    s = torch.full((n + 2,), 2, dtype=torch.int32, device="cuda")
    assert lib.pgk_reduce(d.data_ptr(), s.data_ptr(), n, 0, 0, None) == 0, pgamd.last_error()
    torch.cuda.synchronize()
    assert bool(d[:n].eq(3).all()) and d[n:].tolist() == [1, 1]
    assert lib.pgk_reduce(d.data_ptr() + 4, s.data_ptr(), n, 0, 0, None) == 0, pgamd.last_error()
    torch.cuda.synchronize()
    assert int(d[0]) == 3 and bool(d[1:n].eq(5).all()) and d[n:].tolist() == [3, 1]
    del d, s
    torch.cuda.empty_cache()
    n = (1 << 32) + 3
    d = torch.full((n + 2,), 1, dtype=torch.int32, device="cuda")
    s = torch.full((n + 2,), 2, dtype=torch.int32, device="cuda")
    assert lib.pgk_reduce(d.data_ptr() + 4, s.data_ptr(), n, 0, 0, None) == 0, pgamd.last_error()
    torch.cuda.synchronize()
    assert int(d[0]) == 1 and bool(d[1:n + 1].eq(3).all()) and int(d[n + 1]) == 1
    del d, s
    torch.cuda.empty_cache()


def test_invalid_arguments(gpu, lib):
    torch = gpu
    t = torch.zeros(16, dtype=torch.int32, device="cuda")
    assert lib.pgk_reduce(ptr(t), ptr(t), 16, 2, 0, stream(torch)) == -1
    assert lib.pgk_reduce(ptr(t), ptr(t), 16, 0, 2, stream(torch)) == -1
    assert lib.pgk_reduce(ptr(t), None, 16, 0, 0, stream(torch)) == -1
    assert lib.pgk_reduce(ptr(t), ptr(t), 0, 0, 0, stream(torch)) == 0
    # operands that overlap at different addresses: the reference's loop (src/pg.c:151-159)
    # would feed results back in index order; refused, and nothing is written
    u = torch.arange(32, dtype=torch.int32, device="cuda")
    before = u.clone()
    for dst_off, src_off in ((0, 4), (4, 0), (0, 60)):
        assert lib.pgk_reduce(ptr(u) + dst_off, ptr(u) + src_off, 16, 0, 0, stream(torch)) == -1
        assert b"overlaps an operand" in lib.pgk_last_error()
    assert lib.pgk_reduce_out(ptr(u) + 8, ptr(u), ptr(u) + 64, 8, 0, 0, stream(torch)) == -1
    torch.cuda.synchronize()
    assert torch.equal(u, before)
    # adjacent, not overlapping: fine
    assert lib.pgk_reduce(ptr(u), ptr(u) + 64, 16, 0, 0, stream(torch)) == 0
    torch.cuda.synchronize()
    assert torch.equal(u[:16], before[:16] + before[16:])


def test_reduce_host_staged(gpu, lib, oracle):
    """pgx_reduce_host: both operands in host memory (pageable and pinned),
    piped through HBM slots (1 piece .. 25 pieces over 3 slots, ragged last
    piece, default 32 MiB pieces); identical to the oracle."""
    torch = gpu
    for dt, op, n, chunk in ((1, 0, (3 << 20) + 5, 1 << 20), (0, 1, 1000, 1 << 20), (1, 1, 1 << 22, 4 << 20),
                             (0, 0, (5 << 20) + 7, 1 << 20), (1, 0, (1 << 23) + 1, 0)):
        a, b = oracle.fill(n, dt, op, 51), oracle.fill(n, dt, op, 52)
        want = oracle.reduce(a, b, dt, op)
        d = a.copy()
        assert lib.pgx_reduce_host(d.ctypes.data, b.ctypes.data, n, dt, op, chunk) == 0
        assert d.tobytes() == want.tobytes()
        pd = torch.from_numpy(a.copy()).pin_memory()
        pb = torch.from_numpy(b).pin_memory()
        assert lib.pgx_reduce_host(pd.data_ptr(), pb.data_ptr(), n, dt, op, chunk) == 0
        assert pd.numpy().tobytes() == want.tobytes()
    assert lib.pgx_reduce_host(None, None, 0, 1, 0, 0) == 0
    assert lib.pgx_reduce_host(None, None, 5, 1, 0, 0) == -1
    assert lib.pgx_reduce_host(None, None, 5, 3, 0, 0) == -1


def test_reduce_host_pinned_direct(gpu, lib, oracle):
    """pgx_reduce_host with both operands pinned and mapped (hipHostMalloc):
    one kernel reduces them in place over PCIe.  Offsets inside the pinned
    allocations, odd lengths, and a pinned dst with a pageable src (which must
    take the staged path: a kernel may not touch pageable memory)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    cap = (3 << 20) * 8 + 4096
    ptrs = []
    for _ in range(2):
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), cap, 0x2) == 0      # hipHostMallocMapped
        ptrs.append(p.value)
    try:
        for dt, op, n, off in ((1, 0, 3 << 20, 0), (0, 1, (3 << 20) + 1, 4), (1, 1, 1001, 8), (0, 0, 7, 12)):
            es = 8 if dt else 4
            a, b = oracle.fill(n, dt, op, 61), oracle.fill(n, dt, op, 62)
            want = oracle.reduce(a, b, dt, op)
            ctypes.memmove(ptrs[0] + off, a.ctypes.data, n * es)
            ctypes.memmove(ptrs[1] + off, b.ctypes.data, n * es)
            assert lib.pgx_reduce_host(ptrs[0] + off, ptrs[1] + off, n, dt, op, 0) == 0, pgamd.last_error()
            assert ctypes.string_at(ptrs[0] + off, n * es) == want.tobytes(), (dt, op, n, off)
            assert ctypes.string_at(ptrs[1] + off, n * es) == b.tobytes()
            ctypes.memmove(ptrs[0] + off, a.ctypes.data, n * es)            # pinned dst, pageable src
            assert lib.pgx_reduce_host(ptrs[0] + off, b.ctypes.data, n, dt, op, 0) == 0, pgamd.last_error()
            assert ctypes.string_at(ptrs[0] + off, n * es) == want.tobytes()
    finally:
        for p in ptrs:
            hip.hipHostFree(p)


@pytest.mark.parametrize("dt,op", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_reduce_multi_fold_order(gpu, lib, oracle, dt, op):
    """pgk_reduce_multi folds left to right: equal to nsrc-1 successive
    reduce_inplace steps (the ring's per-element operation sequence)."""
    import ctypes
    torch = gpu
    for nsrc in (1, 2, 3, 5, 8, 9, 16):
        for n, shift in ((4099, 0), (1 << 18, 0), (1001, 1)):
            xs = [oracle.fill(n + 2, dt, op, 900 + 31 * nsrc + j) for j in range(nsrc)]
            want = xs[0][shift:shift + n].copy()
            for j in range(1, nsrc):
                want = oracle.reduce(want, xs[j][shift:shift + n], dt, op)
            D = [to_dev(torch, x) for x in xs]
            es = 4 if dt == 0 else 8
            out = torch.zeros(n + 2, dtype=D[0].dtype, device="cuda")
            srcs = (ctypes.c_void_p * nsrc)(*[ptr(d) + shift * es for d in D])
            assert lib.pgk_reduce_multi(ptr(out), srcs, nsrc, n, dt, op, stream(torch)) == 0
            assert to_host(torch, out)[:n].tobytes() == want.tobytes(), (nsrc, n, shift)
    srcs = (ctypes.c_void_p * 17)()
    assert lib.pgk_reduce_multi(ptr(out), srcs, 17, 4, dt, op, stream(torch)) == -1
    assert lib.pgk_reduce_multi(ptr(out), srcs, 0, 4, dt, op, stream(torch)) == -1


@pytest.mark.parametrize("nsrc,dt,op,nbytes,extra,shift,inplace", [
    (5, 1, 0, 32 << 20, 0, 0, None),        # one launch of 16 tiles per wave
    (8, 1, 0, 72 << 20, 5, 1, None),        # a full launch, a rest under 32 MiB (one tile per wave), ragged edges
    (6, 0, 1, 100 << 20, 3, 3, None),       # a full launch and a rest of 36 MiB (16 tiles per wave), int32 product
    (7, 0, 0, 130 << 20, 0, 0, None),       # two full launches and a 2 MiB rest
    (8, 1, 1, 64 << 20, 0, 0, 7),           # in place over the last source (the ring's own block)
    (5, 1, 0, 40 << 20, 2, 0, 0),           # in place over the first source
])
def test_reduce_multi_burst_form(gpu, lib, oracle, nsrc, dt, op, nbytes, extra, shift, inplace):
    """From 5 sources and 32 MiB per source pgk_reduce_multi gathers its stores
    into one burst per launch (launches of at most 64 MiB per source).  Same
    left-to-right fold as nsrc-1 successive reduce_inplace steps (src/pg.c:151-159),
    bit for bit; equal to the one-tile-per-wave form (pgk_tune_fold(0)), to
    the form for remote sources and to the form for a shared GPU (32 MiB
    launches), byte for byte; stamped by its events."""
    import ctypes
    torch = gpu
    es = 4 if dt == 0 else 8
    n = nbytes // es + extra
    xs = [oracle.fill(n + 4, dt, op, 4100 + 17 * nsrc + j) for j in range(nsrc)]
    want = xs[0][shift:shift + n].copy()
    for j in range(1, nsrc):
        want = oracle.reduce(want, xs[j][shift:shift + n], dt, op)
    D = [to_dev(torch, x) for x in xs]
    srcs = (ctypes.c_void_p * nsrc)(*[ptr(d) + shift * es for d in D])
    if inplace is None:
        out = torch.zeros(n + 4, dtype=D[0].dtype, device="cuda")
        ev = (ctypes.c_void_p(), ctypes.c_void_p())
        assert lib.pgk_event_create(ctypes.byref(ev[0])) == 0 and lib.pgk_event_create(ctypes.byref(ev[1])) == 0
        assert lib.pgk_reduce_multi_timed(ptr(out) + shift * es, srcs, nsrc, n, dt, op, stream(torch), ev[0], ev[1]) == 0
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        assert lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)) == 0
        # first launch's begin to last launch's end: no faster than the HBM peak allows
        assert ms.value * 1e-3 > (nsrc + 1) * n * es / 8e12
        got = to_host(torch, out)
        assert got[shift:shift + n].tobytes() == want.tobytes()
        assert not got[:shift].any() and not got[shift + n:].any()           # nothing outside the range
        for form in ("plain", pgamd.FOLD_REMOTE_SOURCES, pgamd.FOLD_SHARED_GPU,
                     pgamd.FOLD_REMOTE_SOURCES | pgamd.FOLD_SHARED_GPU):
            other = torch.zeros(n + 4, dtype=D[0].dtype, device="cuda")
            if form == "plain":
                assert lib.pgk_tune_fold(0) == 0
                try:
                    assert lib.pgk_reduce_multi(ptr(other) + shift * es, srcs, nsrc, n, dt, op, stream(torch)) == 0
                finally:
                    lib.pgk_tune_fold(1)
            else:
                assert lib.pgk_fold_timed(ptr(other) + shift * es, srcs, nsrc, n, dt, op, form, stream(torch),
                                          None, None) == 0
            assert torch.equal(other, out), form
            del other
        assert lib.pgk_fold_timed(ptr(out), srcs, nsrc, n, dt, op, 4, stream(torch), None, None) == -1
        assert b"unknown fold flags" in lib.pgk_last_error()
        lib.pgk_event_destroy(ev[0]), lib.pgk_event_destroy(ev[1])
    else:
        flags = pgamd.FOLD_SHARED_GPU if nsrc == 5 else 0
        assert lib.pgk_fold_timed(ptr(D[inplace]) + shift * es, srcs, nsrc, n, dt, op, flags, stream(torch),
                                  None, None) == 0
        got = to_host(torch, D[inplace])
        assert got[shift:shift + n].tobytes() == want.tobytes()
        assert got[:shift].tobytes() == xs[inplace][:shift].tobytes()
        assert got[shift + n:].tobytes() == xs[inplace][shift + n:].tobytes()
        for j in range(nsrc):
            if j != inplace:
                assert to_host(torch, D[j]).tobytes() == xs[j].tobytes()      # the other sources untouched
    del D
    torch.cuda.empty_cache()


def test_fold_blocks_and_gather(gpu, lib, oracle):
    """pgk_fold_blocks == the oracle's ring all-reduce (each block in its ring
    order); pgk_gather copies every range, 16-B and 4-B aligned forms."""
    import ctypes
    torch = gpu
    cases = ((2, 1001, 1, 0), (3, 10, 0, 1), (8, 65541, 1, 1), (5, 4, 1, 0), (4, 4099, 0, 0), (7, 7001, 1, 0))
    for (world, count, dt, op), rings in itertools.product(cases, (1, 2, 3, 4)):
        xs = [oracle.fill(count, dt, op, 77 + r) for r in range(world)]
        want = oracle.ring_all_reduce(xs, dt, op, rings)[0]
        D = [to_dev(torch, x) for x in xs]
        out = torch.zeros(count, dtype=D[0].dtype, device="cuda")
        srcs = (ctypes.c_void_p * world)(*[ptr(d) for d in D])
        blk = -(-count // world)
        assert lib.pgk_fold_blocks(ptr(out), srcs, world, count, blk, rings, dt, op, stream(torch)) == 0
        assert to_host(torch, out).tobytes() == want.tobytes(), (world, count, dt, op, rings)
    assert lib.pgk_fold_blocks(ptr(out), srcs, world, count, blk, 5, 1, 0, stream(torch)) == -1
    # gather: ranges of different sizes/alignments into one buffer
    src = torch.arange(1 << 16, dtype=torch.int32, device="cuda")
    dst = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    pieces = [(0, 0, 4096), (4096, 8192, 3), (5000, 20000, 1027), (30000, 40000, 8192)]   # (src elem, dst elem, n)
    ds = (ctypes.c_void_p * 4)(*[ptr(dst) + d * 4 for _, d, _ in pieces])
    ss = (ctypes.c_void_p * 4)(*[ptr(src) + s_ * 4 for s_, _, _ in pieces])
    nb = (ctypes.c_size_t * 4)(*[n * 4 for _, _, n in pieces])
    assert lib.pgk_gather(ds, ss, nb, 4, stream(torch)) == 0
    got = to_host(torch, dst)
    want = np.zeros(1 << 16, np.int32)
    for s_, d, n in pieces:
        want[d:d + n] = np.arange(s_, s_ + n)
    assert np.array_equal(got, want)
    bad = (ctypes.c_size_t * 1)(3)
    assert lib.pgk_gather(ds, ss, bad, 1, stream(torch)) == -1


def test_reduce_captured_in_hip_graph(gpu, lib, oracle):
    """include/pgk.h promises pgk_reduce allocates nothing and is safe to
    capture: a chain of reduces captured into a hipGraph (torch.cuda.CUDAGraph
    is hipGraph on ROCm) and replayed three times gives the oracle's result of
    the same chain applied three times, bit for bit."""
    torch = gpu
    n = (1 << 20) + 5
    for dt, op in ((1, 0), (0, 1)):
        a, b, c = (oracle.fill(n, dt, op, 60 + k) for k in range(3))
        A, B, C = to_dev(torch, a), to_dev(torch, b), to_dev(torch, c)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                sh = torch.cuda.current_stream().cuda_stream
                assert lib.pgk_reduce(ptr(A), ptr(B), n, dt, op, sh) == 0      # A op= B
                assert lib.pgk_reduce(ptr(A), ptr(C), n, dt, op, sh) == 0      # A op= C
        want = a.copy()
        for _ in range(3):
            g.replay()
            want = oracle.reduce(oracle.reduce(want, b, dt, op), c, dt, op)
        torch.cuda.synchronize()
        assert to_host(torch, A).tobytes() == want.tobytes(), (dt, op)


def test_burst_fold_captured_in_hip_graph(gpu, lib, oracle):
    """The fold's burst form is several plain kernel launches on the caller's
    stream and allocates nothing: a 6-source fold of 72 MiB + 3 doubles per source
    (one full launch, a rest one tile per wave, ragged edges), in place over its
    last source, captured into a hipGraph.  Every replay, with eager work and a
    synchronization between replays, equals the eager call on the same inputs."""
    import ctypes
    torch = gpu
    nsrc, n = 6, (72 << 20) // 8 + 3
    xs = [oracle.fill(n + 2, 1, 0, 7300 + j) for j in range(nsrc)]
    D = [to_dev(torch, x) for x in xs]
    srcs = (ctypes.c_void_p * nsrc)(*[ptr(d) + 8 for d in D])          # one element in: a ragged head
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            sh = torch.cuda.current_stream().cuda_stream
            assert lib.pgk_reduce_multi(ptr(D[nsrc - 1]) + 8, srcs, nsrc, n, 1, 0, sh) == 0
    for rep in range(3):
        # fresh inputs for this replay (eager copies), the expected result by the eager call on copies of them
        fresh = [oracle.fill(n + 2, 1, 0, 7400 + 10 * rep + j) for j in range(nsrc)]
        for d, x in zip(D, fresh):
            d.copy_(torch.from_numpy(x))
        E = [d.clone() for d in D]
        esrcs = (ctypes.c_void_p * nsrc)(*[ptr(e) + 8 for e in E])
        assert lib.pgk_reduce_multi(ptr(E[nsrc - 1]) + 8, esrcs, nsrc, n, 1, 0, stream(torch)) == 0
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(D[nsrc - 1], E[nsrc - 1]), rep
        want = fresh[0][1:1 + n].copy()
        for j in range(1, nsrc):
            want = oracle.reduce(want, fresh[j][1:1 + n], 1, 0)
        got = to_host(torch, D[nsrc - 1])
        assert got[1:1 + n].tobytes() == want.tobytes(), rep
        assert got[0] == fresh[nsrc - 1][0] and got[1 + n] == fresh[nsrc - 1][1 + n]
        del E
    del D
    torch.cuda.empty_cache()


def test_reduce_ranges(gpu, lib, oracle):
    """pgk_reduce_ranges (one launch for every ring's arrived segments of an
    executor batch): 1..8 ranges of ragged lengths at aligned and misaligned
    offsets of one pool, in both operand orders (out = a op b with out = a, or
    out = b -- the in-place last round's arrival-first order), each range
    bit-exact against the oracle's reduce of the same operands."""
    import ctypes
    torch = gpu
    rng = np.random.default_rng(7)
    VP, SZ = ctypes.c_void_p, ctypes.c_size_t
    for trial in range(40):
        dt, op = int(rng.integers(2)), int(rng.integers(2))
        es = 4 if dt == 0 else 8
        k = int(rng.integers(1, 9))
        lens = [int(rng.choice([0, 1, 3, 5, 64, 1000, 4099, 65536 + 7, 1 << 20])) for _ in range(k)]
        shift = int(rng.integers(0, 4)) if trial % 3 == 0 else 0      # misaligned: one range off by elements
        size = sum(2 * (n + 8) for n in lens) + 16
        a_np = oracle.fill(size, dt, op, 100 + trial)
        b_np = oracle.fill(size, dt, op, 200 + trial)
        A, B = to_dev(torch, a_np), to_dev(torch, b_np)
        outs, as_, bs_, ns = (VP * k)(), (VP * k)(), (VP * k)(), (SZ * k)()
        want_a, want_b = a_np.copy(), b_np.copy()
        off = 0
        for j, n in enumerate(lens):
            o = off + (shift if j == k - 1 else 0)
            rev = (j + trial) % 2 == 1
            pa, pb = ptr(A) + o * es, ptr(B) + o * es
            if rev:       # out = b = a op b
                outs[j], as_[j], bs_[j] = pb, pa, pb
                want_b[o:o + n] = oracle.reduce(a_np[o:o + n], b_np[o:o + n], dt, op)
            else:         # out = a = a op b
                outs[j], as_[j], bs_[j] = pa, pa, pb
                want_a[o:o + n] = oracle.reduce(a_np[o:o + n], b_np[o:o + n], dt, op)
            ns[j] = n
            off += n + 8
        assert lib.pgk_reduce_ranges(outs, as_, bs_, ns, k, dt, op, stream(torch), None, None) == 0, \
            pgamd.last_error()
        assert to_host(torch, A).tobytes() == want_a.tobytes(), (trial, lens, shift)
        assert to_host(torch, B).tobytes() == want_b.tobytes(), (trial, lens, shift)
    # argument checks and stamps
    assert lib.pgk_reduce_ranges(None, None, None, None, 0, 1, 0, stream(torch), None, None) == 0
    nine = (VP * 9)()
    assert lib.pgk_reduce_ranges(nine, nine, nine, (SZ * 9)(), 9, 1, 0, stream(torch), None, None) == -1
    x = torch.ones(1 << 20, dtype=torch.float64, device="cuda")
    ev0, ev1 = VP(), VP()
    pgamd.check(lib.pgk_event_create(ctypes.byref(ev0)), "event")
    pgamd.check(lib.pgk_event_create(ctypes.byref(ev1)), "event")
    p2 = (VP * 2)(ptr(x), ptr(x) + (1 << 22))
    assert lib.pgk_reduce_ranges(p2, p2, p2, (SZ * 2)(1 << 18, 1 << 18), 2, 1, 0, stream(torch), ev0, ev1) == 0
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    pgamd.check(lib.pgk_event_elapsed_ms(ev0, ev1, ctypes.byref(ms)), "elapsed")
    assert ms.value > 0
    assert float(x[:1 << 18].sum()) == 2.0 * (1 << 18) and float(x[1 << 18:1 << 19].sum()) == 1 << 18
    lib.pgk_event_destroy(ev0)
    lib.pgk_event_destroy(ev1)
