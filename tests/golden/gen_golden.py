"""Generate tests/golden/ from the reference's OWN compiled code.

Run in the development container (needs /root/reference and oracle/_ref/libpgref.so,
built by `make -C oracle`):

    python tests/golden/gen_golden.py

Every expected output below comes from the reference's src/pg.c (lines 104-179
and 264-339 compiled unchanged by oracle/Makefile) -- reduce_inplace exposed
through ref_reduce_inplace, and pg_reduce_scatter / pg_all_gather /
pg_all_reduce driven with a hand-filled struct pg.
Inputs come from the splitmix64 generator (orc_fill); the
stored digests let a test regenerate the large inputs and check them.
Only in-bounds shapes are generated (the reference reads/writes past its
buffers for some shapes).
"""
from __future__ import annotations

import hashlib
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle.pyoracle import Oracle, Reference, NP_DTYPE  # noqa: E402

OUT = pathlib.Path(__file__).resolve().parent
ES = {0: 4, 1: 8}
BASE_SEED = 0x5EEDC0DE


def seed(cfg: int, rank: int, role: int) -> int:
    return (BASE_SEED ^ (cfg << 32) ^ rank ^ (role << 48)) & 0xFFFFFFFFFFFFFFFF


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def mock_in_bounds(rank, world, count, ce):
    for k in range(world - 1):
        so = ((rank - k) % world) * ce
        ro = ((rank - k - 1) % world) * ce
        rl = max(0, min(ro + ce, count) - ro) if ro < count else 0
        if rl and so + rl > count:
            return False
    return True


def main() -> None:
    orc, ref = Oracle(), Reference()
    arrays: dict[str, np.ndarray] = {}
    manifest: dict = {"generator": "tests/golden/gen_golden.py",
                      "reference": "gevahaviv1/RDMA-Ring-Collectives src/pg.c:104-179,264-339 (compiled by oracle/Makefile)",
                      "seed_rule": "0x5EEDC0DE ^ (cfg<<32) ^ rank ^ (role<<48); orc_fill(dt, op)",
                      "kernel": [], "specials": [], "mock_rs": [], "mock_ag": [], "w1": [], "errors": []}

    # (1) kernel KATs: reduce_inplace over n elements
    cfg = 100
    for dt in (0, 1):
        for op in (0, 1):
            for n in (1, 3, 64, 1000, 4099, 65536):
                cfg += 1
                d0 = orc.fill(n, dt, op, seed(cfg, 0, 1))
                s = orc.fill(n, dt, op, seed(cfg, 0, 2))
                out = ref.reduce(d0, s, dt, op)
                # cross-check through the public RS (W=2, R=0, chunk=n*es, count=2n)
                send = np.concatenate([s, np.zeros(n, NP_DTYPE[dt])])
                recv = np.concatenate([np.zeros(n, NP_DTYPE[dt]), d0])
                rc, r2 = ref.reduce_scatter(0, 2, n * ES[dt], send, recv, dt, op)
                assert rc == 0 and r2[n:].tobytes() == out.tobytes()
                key = f"k{cfg}"
                case = {"key": key, "dt": dt, "op": op, "n": n, "seed_dst": seed(cfg, 0, 1),
                        "seed_src": seed(cfg, 0, 2), "sha_dst0": sha(d0), "sha_src": sha(s), "sha_out": sha(out)}
                if n <= 4099:
                    arrays[key + "_dst0"], arrays[key + "_src"], arrays[key + "_out"] = d0, s, out
                    case["stored"] = True
                else:
                    case["stored"] = False
                manifest["kernel"].append(case)

    # special values: every (dst, src) pair
    i32 = np.array([0, 1, -1, 2, -2, 2**31 - 1, -2**31, -2**31 + 1, 65536, -65536, 0x55555555,
                    -123456789, 987654, 46341, 46340, 3, 7], dtype=np.int32)
    f64 = np.array([0.0, -0.0, 1.0, -1.0, 0.5, 3.0, 1.0 / 3.0, 1.0 + 2.0**-52, np.finfo(np.float64).max,
                    -np.finfo(np.float64).max, np.finfo(np.float64).tiny, 5e-324, -5e-324,
                    2.2250738585072009e-308, 1e308, 1e-308, 1e-160, np.inf, -np.inf, np.nan,
                    0.1, 0.2], dtype=np.float64)
    for dt, vals in ((0, i32), (1, f64)):
        for op in (0, 1):
            d0 = np.repeat(vals, vals.size)
            s = np.tile(vals, vals.size)
            out = ref.reduce(d0, s, dt, op)
            key = f"sp{dt}{op}"
            arrays[key + "_dst0"], arrays[key + "_src"], arrays[key + "_out"] = d0, s, out
            manifest["specials"].append({"key": key, "dt": dt, "op": op, "n": int(d0.size)})
    # known answers (worked by hand from reference src/pg.c:151-159, :264-291) must hold
    assert ref.reduce(np.array([2**31 - 1], np.int32), np.array([2**31 - 1], np.int32), 0, 0)[0] == -2
    assert ref.reduce(np.array([65536], np.int32), np.array([65536], np.int32), 0, 1)[0] == 0
    assert ref.reduce(np.array([-123456789], np.int32), np.array([987654], np.int32), 0, 1)[0] == 1530050434

    # (2) schedule KATs: the mock reduce-scatter, every rank
    cfg = 1000
    for world in (2, 3, 4, 8):
        for dt in (0, 1):
            for op in (0, 1, 2):           # 2: any non-OP_SUM value multiplies
                if op == 2 and world not in (2, 4):
                    continue
                for chunk_bytes in (12, 16, 100):
                    ce = max(1, chunk_bytes // ES[dt])
                    for count in sorted({0, world * ce, world * ce + 5, world * ce - ce // 2, ce + 1}):
                        if count < 0:
                            continue
                        for rank in range(world):
                            if not mock_in_bounds(rank, world, count, ce):
                                continue
                            cfg += 1
                            kop = 0 if op == 0 else 1
                            send = orc.fill(count, dt, kop, seed(cfg, rank, 1))
                            recv0 = orc.fill(count, dt, kop, seed(cfg, rank, 2))
                            rc, recv1 = ref.reduce_scatter(rank, world, chunk_bytes, send, recv0, dt, op)
                            assert rc == 0
                            key = f"rs{cfg}"
                            arrays[key + "_send"], arrays[key + "_recv0"], arrays[key + "_recv1"] = send, recv0, recv1
                            manifest["mock_rs"].append({"key": key, "world": world, "rank": rank, "dt": dt, "op": op,
                                                        "chunk_bytes": chunk_bytes, "count": count})
    # the in-place form used by pg_all_reduce (sendbuf == recvbuf)
    for world, rank, dt, op, cb, count in ((2, 1, 1, 0, 16, 8), (4, 2, 0, 0, 8, 8), (3, 0, 1, 1, 24, 9)):
        cfg += 1
        buf = orc.fill(count, dt, op, seed(cfg, rank, 1))
        rc, out = ref.reduce_scatter(rank, world, cb, buf, buf, dt, op)   # recv copy; send separate copy
        # in place: drive the reference with one buffer
        one = np.array(buf, copy=True)
        rc2 = ref.lib.ref_reduce_scatter(rank, world, cb, one.ctypes.data, one.ctypes.data, count, dt, op)
        assert rc == 0 and rc2 == 0
        key = f"rsip{cfg}"
        arrays[key + "_buf0"], arrays[key + "_buf1"] = buf, one
        manifest["mock_rs"].append({"key": key, "world": world, "rank": rank, "dt": dt, "op": op,
                                    "chunk_bytes": cb, "count": count, "in_place": True})

    # (2b) mock all-gather (sums instead of copying, src/pg.c:317)
    for world in (2, 3, 4):
        for dt in (0, 1):
            for count in (1, 7, 64):
                for with_send in (True, False):
                    for rank in range(world):
                        cfg += 1
                        send = orc.fill(count, dt, 0, seed(cfg, rank, 1)) if with_send else None
                        recv0 = orc.fill(count * world, dt, 0, seed(cfg, rank, 2))
                        rc, recv1 = ref.all_gather(rank, world, send, recv0, count, dt)
                        assert rc == 0
                        key = f"ag{cfg}"
                        if with_send:
                            arrays[key + "_send"] = send
                        arrays[key + "_recv0"], arrays[key + "_recv1"] = recv0, recv1
                        manifest["mock_ag"].append({"key": key, "world": world, "rank": rank, "dt": dt,
                                                    "count": count, "with_send": with_send})

    # (3) world_size == 1 API
    for dt in (0, 1):
        for op in (0, 1):
            for count in (0, 1, 5, 1000):
                cfg += 1
                send = orc.fill(count, dt, op, seed(cfg, 0, 1))
                recv0 = orc.fill(count, dt, op, seed(cfg, 0, 2))
                rc_rs, rs = ref.reduce_scatter(0, 1, 4096, send, recv0, dt, op)
                rc_ag, ag = ref.all_gather(0, 1, send, recv0, count, dt)
                rc_ar, ar = ref.all_reduce(0, 1, 4096, send, recv0, dt, op)
                rc_ip, ip = ref.all_reduce(0, 1, 4096, None, send, dt, op)
                assert rc_rs == rc_ag == rc_ar == rc_ip == 0
                key = f"w1{cfg}"
                arrays.update({key + "_send": send, key + "_recv0": recv0, key + "_rs": rs, key + "_ag": ag,
                               key + "_ar": ar, key + "_arip": ip})
                manifest["w1"].append({"key": key, "dt": dt, "op": op, "count": count})

    # (4) validation return codes (src/pg.c:267, :295, :325)
    buf = np.zeros(16, np.int32)
    p = buf.ctypes.data
    L = ref.lib
    errs = [
        ("reduce_scatter", "null_send", L.ref_reduce_scatter(0, 2, 16, None, p, 8, 0, 0)),
        ("reduce_scatter", "null_recv", L.ref_reduce_scatter(0, 2, 16, p, None, 8, 0, 0)),
        ("reduce_scatter", "negative_count", L.ref_reduce_scatter(0, 2, 16, p, p, -1, 0, 0)),
        ("reduce_scatter", "bad_datatype", L.ref_reduce_scatter(0, 2, 16, p, p, 8, 7, 0)),
        ("reduce_scatter", "zero_count", L.ref_reduce_scatter(0, 2, 16, p, p, 0, 0, 0)),
        ("all_gather", "null_recv", L.ref_all_gather(0, 2, p, None, 8, 0)),
        ("all_gather", "negative_count", L.ref_all_gather(0, 2, p, p, -1, 0)),
        ("all_gather", "bad_datatype", L.ref_all_gather(0, 2, p, p, 8, 7)),
        ("all_gather", "null_send_world1", L.ref_all_gather(0, 1, None, p, 8, 0)),
        ("all_reduce", "null_send", L.ref_all_reduce(0, 1, 16, None, p, 8, 0, 0)),
        ("all_reduce", "null_recv", L.ref_all_reduce(0, 1, 16, p, None, 8, 0, 0)),
        ("all_reduce", "negative_count", L.ref_all_reduce(0, 1, 16, p, p, -1, 0, 0)),
        ("all_reduce", "bad_datatype", L.ref_all_reduce(0, 1, 16, p, p, 8, 7, 0)),
    ]
    manifest["errors"] = [{"fn": f, "case": c, "rc": int(rc)} for f, c, rc in errs]

    np.savez_compressed(OUT / "golden.npz", **arrays)
    (OUT / "golden.json").write_text(json.dumps(manifest, indent=1) + "\n")
    total = sum(a.nbytes for a in arrays.values())
    print(f"wrote {len(arrays)} arrays ({total / 1e6:.2f} MB raw), "
          f"{len(manifest['kernel'])} kernel / {len(manifest['mock_rs'])} rs / {len(manifest['mock_ag'])} ag cases")


if __name__ == "__main__":
    main()
