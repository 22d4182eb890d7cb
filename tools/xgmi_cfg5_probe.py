#!/usr/bin/env python3
"""EXPERIMENTS ONLY: replay bench.py's config-5 sequence on the xgmi transport
(W processes on one GPU): int32 / double product, eager size interleaved with
2 GiB, every call's result checked on the device; a mismatch prints the rank,
call, and the first differing elements.
    python tools/xgmi_cfg5_probe.py --world 8 [--rounds 3]"""
import argparse
import ctypes
import multiprocessing as mp
import os
import pathlib
import socket
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, rounds, q):
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port),
                      PG_BARRIER_TIMEOUT_MS="60000", PG_TRACE=os.environ.get("PG_TRACE", "0"),
                      PG_TRACE_FILE=os.environ.get("PG_TRACE_FILE", ""))
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    import torch
    import bench
    import pgamd
    torch.cuda.set_device(0)
    lib = pgamd.load()
    h = ctypes.c_void_p()
    assert lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) == 0
    bad = []
    ncalls = 0
    for rnd in range(rounds):
        for dt, big in ((pgamd.DT_DOUBLE, 1 << 28), (pgamd.DT_INT32, 1 << 29)):
            small = 4096 // pgamd.ELEM_SIZE[dt]
            for cnt in (small, big, small):
                xv = bench._pattern(cnt, rank, world, dt, pgamd.OP_PROD)
                off, ln = pgamd.block_range(cnt, world, rank)
                want = bench._expected_block(cnt, off, ln, world, dt, pgamd.OP_PROD)
                reps = 20 if cnt == small else 2
                for it in range(reps + 1):
                    ov = torch.full((max(ln, 1),), 7, dtype=xv.dtype, device="cuda")
                    rc = lib.pg_reduce_scatter(xv.data_ptr(), ov.data_ptr(), cnt, dt, pgamd.OP_PROD, h)
                    ncalls += 1
                    if rc != 0:
                        bad.append((rnd, dt, cnt, it, "rc", pgamd.last_error()))
                        break
                    if not torch.equal(ov[:ln], want):
                        d = (ov[:ln] != want).nonzero().flatten()
                        bad.append((rnd, dt, cnt, it, "call", ncalls - 1, int(d.numel()), d[:8].tolist(),
                                    ov[:ln][d[:4]].tolist(), want[d[:4]].tolist()))
                del xv, ov, want
                torch.cuda.empty_cache()
    lib.pg_close(h)
    q.put((rank, ncalls, bad))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, a.rounds, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = []
    t0 = time.time()
    for _ in ps:
        res.append(q.get(timeout=600))
    for p in ps:
        p.join(30)
    nbad = 0
    for rank, ncalls, bad in sorted(res):
        print(f"rank {rank}: {ncalls} calls, {len(bad)} bad", flush=True)
        for b in bad[:6]:
            print("   ", b, flush=True)
        nbad += len(bad)
    print(f"{'FAIL' if nbad else 'ok'} in {time.time() - t0:.1f} s", flush=True)
    sys.exit(1 if nbad else 0)


if __name__ == "__main__":
    main()
