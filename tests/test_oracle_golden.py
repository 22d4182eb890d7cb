"""The CPU oracle against the reference's own outputs (tests/golden/, generated
by tests/golden/gen_golden.py from the compiled reference src/pg.c), and --
when oracle/_ref/libpgref.so is present -- against the reference directly."""
import hashlib

import numpy as np
import pytest

from oracle.pyoracle import REF_LIB, NP_DTYPE, splitmix64_numpy


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_kernel_kats(golden, oracle):
    man, arr = golden
    for c in man["kernel"]:
        d0 = oracle.fill(c["n"], c["dt"], c["op"], c["seed_dst"])
        s = oracle.fill(c["n"], c["dt"], c["op"], c["seed_src"])
        assert sha(d0) == c["sha_dst0"] and sha(s) == c["sha_src"], c["key"]
        out = oracle.reduce(d0, s, c["dt"], c["op"])
        assert sha(out) == c["sha_out"], c["key"]
        if c["stored"]:
            assert out.tobytes() == arr[c["key"] + "_out"].tobytes()


def test_special_values(golden, oracle):
    man, arr = golden
    for c in man["specials"]:
        out = oracle.reduce(arr[c["key"] + "_dst0"], arr[c["key"] + "_src"], c["dt"], c["op"])
        assert out.tobytes() == arr[c["key"] + "_out"].tobytes(), c["key"]


def test_survey_known_answers(oracle):
    i = lambda *v: np.array(v, np.int32)  # noqa: E731
    assert oracle.reduce(i(2**31 - 1), i(2**31 - 1), 0, 0)[0] == -2
    assert oracle.reduce(i(65536), i(65536), 0, 1)[0] == 0
    assert oracle.reduce(i(-123456789), i(987654), 0, 1)[0] == 1530050434
    # W=2, R=0, chunk 4 i32, n=8
    send = np.arange(1, 9, dtype=np.int32)
    recv = (1000 * np.arange(1, 9)).astype(np.int32)
    rc, out = oracle.mock_reduce_scatter(0, 2, 16, send, recv, 0, 0)
    assert rc == 0 and out.tolist() == [1000, 2000, 3000, 4000, 5001, 6002, 7003, 8004]
    rc, out = oracle.mock_reduce_scatter(2, 4, 8, send, recv, 0, 0)
    assert out.tolist() == [1003, 2004, 3005, 4006, 5000, 6000, 7001, 8002]


def test_mock_reduce_scatter(golden, oracle):
    man, arr = golden
    for c in man["mock_rs"]:
        k = c["key"]
        if c.get("in_place"):
            buf = np.array(arr[k + "_buf0"], copy=True)
            rc = oracle.lib.orc_mock_reduce_scatter(c["rank"], c["world"], c["chunk_bytes"], buf.ctypes.data,
                                                    buf.ctypes.data, c["count"], c["dt"], c["op"])
            assert rc == 0 and buf.tobytes() == arr[k + "_buf1"].tobytes(), k
            continue
        rc, out = oracle.mock_reduce_scatter(c["rank"], c["world"], c["chunk_bytes"], arr[k + "_send"],
                                             arr[k + "_recv0"], c["dt"], c["op"])
        assert rc == 0 and out.tobytes() == arr[k + "_recv1"].tobytes(), k


def test_mock_all_gather(golden, oracle):
    man, arr = golden
    for c in man["mock_ag"]:
        k = c["key"]
        send = arr[k + "_send"] if c["with_send"] else None
        rc, out = oracle.mock_all_gather(c["rank"], c["world"], send, arr[k + "_recv0"], c["count"], c["dt"])
        assert rc == 0 and out.tobytes() == arr[k + "_recv1"].tobytes(), k


def test_world1_api(golden, oracle):
    man, arr = golden
    for c in man["w1"]:
        k = c["key"]
        send, recv0 = arr[k + "_send"], arr[k + "_recv0"]
        rc, rs = oracle.mock_reduce_scatter(0, 1, 4096, send, recv0, c["dt"], c["op"])
        assert rc == 0 and rs.tobytes() == arr[k + "_rs"].tobytes()
        rc, ag = oracle.mock_all_gather(0, 1, send, recv0, c["count"], c["dt"])
        assert rc == 0 and ag.tobytes() == arr[k + "_ag"].tobytes()


def test_error_codes(golden, oracle):
    man, _ = golden
    buf = np.zeros(16, np.int32)
    p = buf.ctypes.data
    L = oracle.lib
    got = {
        ("reduce_scatter", "null_send"): L.orc_mock_reduce_scatter(0, 2, 16, None, p, 8, 0, 0),
        ("reduce_scatter", "null_recv"): L.orc_mock_reduce_scatter(0, 2, 16, p, None, 8, 0, 0),
        ("reduce_scatter", "negative_count"): L.orc_mock_reduce_scatter(0, 2, 16, p, p, -1, 0, 0),
        ("reduce_scatter", "bad_datatype"): L.orc_mock_reduce_scatter(0, 2, 16, p, p, 8, 7, 0),
        ("reduce_scatter", "zero_count"): L.orc_mock_reduce_scatter(0, 2, 16, p, p, 0, 0, 0),
        ("all_gather", "null_recv"): L.orc_mock_all_gather(0, 2, p, None, 8, 0),
        ("all_gather", "negative_count"): L.orc_mock_all_gather(0, 2, p, p, -1, 0),
        ("all_gather", "bad_datatype"): L.orc_mock_all_gather(0, 2, p, p, 8, 7),
        ("all_gather", "null_send_world1"): L.orc_mock_all_gather(0, 1, None, p, 8, 0),
        ("all_reduce", "null_send"): L.orc_mock_all_reduce(0, 1, 16, None, p, 8, 0, 0),
        ("all_reduce", "null_recv"): L.orc_mock_all_reduce(0, 1, 16, p, None, 8, 0, 0),
        ("all_reduce", "negative_count"): L.orc_mock_all_reduce(0, 1, 16, p, p, -1, 0, 0),
        ("all_reduce", "bad_datatype"): L.orc_mock_all_reduce(0, 1, 16, p, p, 8, 7, 0),
    }
    for e in man["errors"]:
        assert got[(e["fn"], e["case"])] == e["rc"], e


def test_splitmix_stream(oracle):
    n = 1000
    a = oracle.fill(n, 0, 0, 12345)
    z = splitmix64_numpy(12345, n)
    assert np.array_equal(a.view(np.uint32), (z >> np.uint64(32)).astype(np.uint32))


@pytest.mark.parametrize("rings", [1, 2, 3, 4])
def test_ring_simulator_semantics(oracle, rings):
    """orc_ring_*: integer sums equal the wrapped total; doubles follow the
    documented fold order x[b+1] op x[b+2] op ... op x[b] (with R rings, part
    g = [ceil(g*len/R), ceil((g+1)*len/R)) of each block x[b+d] op x[b+2d] op
    ... op x[b], d = +1, -1, +3, -3 where coprime with W and new mod W)."""
    rng = np.random.default_rng(7)
    for world in (1, 2, 3, 5, 8):
        for count in (0, 1, 7, 64, 1001):
            xs = [rng.integers(-2**31, 2**31, count, dtype=np.int64).astype(np.int32) for _ in range(world)]
            outs = oracle.ring_reduce_scatter(xs, 0, 0, rings)
            total = np.zeros(count, np.uint32)
            for x in xs:
                total += x.view(np.uint32)
            for b in range(world):
                off, ln = oracle.ring_block(count, world, b)
                assert np.array_equal(outs[b].view(np.uint32), total[off:off + ln])
            fs = [rng.standard_normal(count) * np.exp2(rng.integers(-30, 31, count)) for _ in range(world)]
            outs = oracle.ring_reduce_scatter(fs, 1, 0, rings)
            steps, c = [1, -1], 3
            while len(steps) < 4 and c < 2 * world:
                for d in (c, -c):
                    if len(steps) < 4 and d % world and np.gcd(d % world, world) == 1 and \
                            all(d % world != e % world for e in steps):
                        steps.append(d)
                c += 2
            for b in range(world):
                off, ln = oracle.ring_block(count, world, b)
                for g in range(rings):
                    lo, hi, step = -(-g * ln // rings), -(-(g + 1) * ln // rings), steps[g % len(steps)] % world
                    acc = fs[(b + step) % world][off + lo:off + hi].copy()
                    for j in range(2, world + 1):
                        acc = acc + fs[(b + j * step) % world][off + lo:off + hi]
                    assert acc.tobytes() == outs[b][lo:hi].tobytes()
            ar = oracle.ring_all_reduce(fs, 1, 0, rings)
            full = np.concatenate(outs) if outs else np.zeros(0)
            assert all(r.tobytes() == full.tobytes() for r in ar)
            ag = oracle.ring_all_gather(fs, 1)
            assert all(r.tobytes() == np.concatenate(fs).tobytes() for r in ag)


@pytest.mark.skipif(not REF_LIB.exists(), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_matches_reference_live(oracle):
    from oracle.pyoracle import Reference
    ref = Reference()
    for dt in (0, 1):
        for cb in (1, 3, 4, 7, 8, 12, 4096):
            assert oracle.lib.orc_chunk_elems_from_bytes(cb, dt) == ref.lib.ref_chunk_elems_from_bytes(cb, dt)
    for w in range(1, 9):
        for r in range(w):
            for k in range(w):
                assert oracle.lib.orc_rs_send_chunk_index(k, r, w) == ref.lib.ref_rs_send_chunk_index(k, r, w)
                assert oracle.lib.orc_rs_recv_chunk_index(k, r, w) == ref.lib.ref_rs_recv_chunk_index(k, r, w)
    rng = np.random.default_rng(3)
    for dt in (0, 1):
        for op in (0, 1, 5):
            for n in (1, 17, 4096, 100003):
                if dt == 0:
                    d = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
                    s = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
                else:
                    d = rng.standard_normal(n) * 1e300
                    s = rng.standard_normal(n) * 1e10
                assert oracle.reduce(d, s, dt, op).tobytes() == ref.reduce(d, s, dt, op).tobytes()
