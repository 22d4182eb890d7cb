#!/usr/bin/env python3
"""Per-call latency/throughput of pg_all_reduce / pg_reduce_scatter over the
xgmi transport or the RCCL ring with W real processes sharing this box's GPU(s)
(device and host buffers), across message sizes from eager (4 KiB) to 256 MiB.

    python tools/latency.py [--world 2] [--transport xgmi|rccl] [--out gpurun_out/latency.csv]

With --transport rccl on one GPU every rank gets its own NCCL_HOSTID, so RCCL
carries the hops over its socket transport (tests/test_rccl_gpu.py): the
small-call figures show our fixed cost plus a loopback socket round trip.

Rows: size, rounds, inflight, time_us, GB/s (reference README.md:85 schema)
plus collective / memory kind.  On a 1-GPU box all ranks share one device, so
large-size rates are a lower bound for a real node."""
import argparse
import os
import pathlib
import socket
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]


def worker(rank, world, port, q, sizes, transport):
    try:
        _worker(rank, world, port, q, sizes, transport)
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, [("error", repr(e))]))


def _worker(rank, world, port, q, sizes, transport):
    os.environ.update(PG_TRANSPORT=transport, PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port))
    if transport == "rccl":
        os.environ.update(NCCL_HOSTID=f"pg-latency-{port}-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    import ctypes

    import numpy as np
    import torch

    import pgamd
    torch.cuda.set_device(0)
    lib = pgamd.load()
    h = ctypes.c_void_p()
    pgamd.check(lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)), "connect")
    rows = []
    for nbytes in sizes:
        n = nbytes // 8
        for kind in ("device", "host"):
            if kind == "device":
                x = torch.rand(n, dtype=torch.float64, device="cuda")
                y = torch.empty(n, dtype=torch.float64, device="cuda")
                xp, yp = x.data_ptr(), y.data_ptr()
            else:
                x = np.random.rand(n)
                y = np.empty(n)
                xp, yp = x.ctypes.data, y.ctypes.data
            for coll in ("all_reduce", "reduce_scatter"):
                fn = lib.pg_all_reduce if coll == "all_reduce" else lib.pg_reduce_scatter
                reps = 200 if nbytes <= (1 << 20) else 10
                ts = []
                for i in range(reps + 3):
                    t0 = time.perf_counter()
                    pgamd.check(fn(xp, yp, n, 1, 0, h), coll)
                    if i >= 3:
                        ts.append(time.perf_counter() - t0)
                med = statistics.median(ts)
                st = pgamd.stats(h)
                phases = "sync %.0f copy %.0f barrier %.0f kernel %.0f device %.0f wall %.0f" % (
                    st["sync_us"], st["copy_us"], st["barrier_us"], st["kernel_us"], st["ring_us"], st["wall_us"])
                rows.append((nbytes, world - 1, 0, round(med * 1e6, 2), round(nbytes / med / 1e9, 3), coll, kind,
                             phases))
            del x, y
    lib.pg_close(h)
    q.put((rank, rows))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--transport", default="xgmi", choices=("xgmi", "rccl"))
    ap.add_argument("--out", default="gpurun_out/latency.csv")
    a = ap.parse_args()
    import multiprocessing as mp
    sizes = [4096, 65536, 1 << 20, 16 << 20, 256 << 20]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, q, sizes, a.transport)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(a.world))
    for p in ps:
        p.join(timeout=60)
    out = pathlib.Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    with out.open("w") as f:
        f.write(f"# transport {a.transport}, {a.world} processes on one GPU\n")
        f.write("size,rounds,inflight,time_us,GB/s,collective,memory,last_call_phases_us\n")
        for row in res[0]:
            f.write(",".join(map(str, row)) + "\n")
            print(*row)


if __name__ == "__main__":
    main()
