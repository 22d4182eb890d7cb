#!/usr/bin/env python3
"""EXPERIMENTS ONLY: W real processes on one GPU run PG_TRANSPORT=xgmi
reduce-scatters of growing size, each phase stamped to gpurun_out/xprobe_r<rank>.log,
to find where a large multi-rank call stalls.

    python tools/xgmi_probe.py --world 4 --log2 20 24 26 28 [--dt 0] [--zero-copy 1]
"""
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


def worker(rank, world, port, sizes, dt, zc, tag):
    os.environ.update(PG_TRANSPORT="xgmi", PG_RANK=str(rank), PG_DEVICE="0", PG_PORT=str(port), PG_DEBUG="1",
                      PG_BARRIER_TIMEOUT_MS="40000", PG_XGMI_ZERO_COPY=zc, PG_TRACE="1")
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    log = open(ROOT / "gpurun_out" / f"xprobe{tag}_r{rank}.log", "w", buffering=1)
    t0 = time.perf_counter()

    def say(msg):
        log.write(f"+{time.perf_counter() - t0:8.3f}s {msg}\n")

    import torch
    import pgamd
    torch.cuda.set_device(0)
    lib = pgamd.load()
    h = ctypes.c_void_p()
    say("connect")
    if lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h)) != 0:
        say("connect failed: " + pgamd.last_error())
        return
    tdt = torch.int32 if dt == 0 else torch.float64
    for lg in sizes:
        count = 1 << lg
        say(f"alloc count=2^{lg}")
        x = (torch.arange(count, device="cuda", dtype=torch.int64) % 1000 + rank).to(tdt)
        off, ln = pgamd.block_range(count, world, rank)
        out = torch.empty(max(ln, 1), dtype=tdt, device="cuda")
        torch.cuda.synchronize()
        for rep in range(2):
            say(f"  RS rep {rep} start")
            rc = lib.pg_reduce_scatter(x.data_ptr(), out.data_ptr(), count, dt, 0, h)
            say(f"  RS rep {rep} rc={rc} {pgamd.last_error() if rc else ''}")
            if rc:
                return
        i = torch.arange(off, off + ln, device="cuda", dtype=torch.int64)
        want = (world * (i % 1000) + world * (world - 1) // 2).to(tdt)
        say(f"  ok={bool(torch.equal(out[:ln], want))}")
        del x, out, i, want
        torch.cuda.empty_cache()
    lib.pg_close(h)
    say("closed")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--log2", type=int, nargs="+", default=[20, 24, 26, 28])
    ap.add_argument("--dt", type=int, default=0)
    ap.add_argument("--zero-copy", default="1")
    ap.add_argument("--timeout", type=float, default=150)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, a.log2, a.dt, a.zero_copy, a.tag)) for r in range(a.world)]
    for p in ps:
        p.start()
    deadline = time.time() + a.timeout
    for p in ps:
        p.join(max(1.0, deadline - time.time()))
    alive = [p for p in ps if p.is_alive()]
    for p in alive:
        p.kill()
    for p in ps:
        p.join()
    for r in range(a.world):
        f = ROOT / "gpurun_out" / f"xprobe{a.tag}_r{r}.log"
        print(f"== rank {r}\n" + (f.read_text() if f.exists() else "(no log)"))
    print("timed out" if alive else "done", flush=True)
    sys.exit(1 if alive else 0)


if __name__ == "__main__":
    main()
