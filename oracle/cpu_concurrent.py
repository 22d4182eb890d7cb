"""TEST INFRASTRUCTURE ONLY -- the CPU baseline with W concurrent ranks.

Besides the 1-core figure, time W processes at once, each
pinned to its own host core and each running the reference's reduce loop
(oracle/_ref, src/pg.c:151-159) over its own 256 MiB double chunk -- what W
CPU ranks of the reference would sustain on this host.  Started by bench.py's
cpu_baseline leg as a child process (`python -m oracle.cpu_concurrent`), so
no worker inherits the parent's GPU state.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import time

from oracle.pyoracle import DT_DOUBLE, OP_SUM, Oracle, Reference

N = 1 << 25          # 256 MiB of doubles, BASELINE config 2's chunk


def _worker(core, seconds, start, q):
    try:
        os.sched_setaffinity(0, {core})
    except (AttributeError, OSError):
        pass
    try:
        impl, kind = Reference(), "reference"
    except RuntimeError:
        impl, kind = Oracle(), "port"
    orc = Oracle()
    d = orc.fill(N, DT_DOUBLE, OP_SUM, 0x5EEDC0DE ^ (2 << 32) ^ (core << 1))
    s = orc.fill(N, DT_DOUBLE, OP_SUM, 0x5EEDC0DE ^ (2 << 32) ^ (core << 1) ^ 1)
    impl.time_reduce(d, s, DT_DOUBLE, OP_SUM, 1)          # touch pages
    start.wait()
    reps, secs = 0, 0.0
    while secs < seconds:
        secs += impl.time_reduce(d, s, DT_DOUBLE, OP_SUM, 1)
        reps += 1
    q.put((core, reps, secs, kind))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=5.0)
    a = ap.parse_args()
    # spread over the allowed cores: adjacent cores share a CCD (and its link to
    # the memory controllers) on EPYC, which would measure one CCD, not W ranks
    allowed = sorted(os.sched_getaffinity(0))
    k = min(a.procs, len(allowed))
    cores = [allowed[(i * len(allowed)) // k] for i in range(k)]
    ctx = mp.get_context("fork")            # this process never touched a GPU
    start, q = ctx.Event(), ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(c, a.seconds, start, q)) for c in cores]
    for p in ps:
        p.start()
    time.sleep(0.5)
    start.set()
    res = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join()
    per = [3 * N * 8 * reps / secs / 2**30 for _, reps, secs, _ in res]
    print(json.dumps({"procs": len(cores), "cores": cores, "kind": res[0][3],
                      "aggregate_gibs": round(sum(per), 2), "per_proc_min_gibs": round(min(per), 2),
                      "per_proc_max_gibs": round(max(per), 2), "unit": "GiB/s (3*n*8 B traffic)",
                      "sample": f"{len(cores)} processes x reduce_inplace(double, sum) over their own 256 MiB "
                                f"chunks, {a.seconds:.0f} s each, one pinned core per process"}))


if __name__ == "__main__":
    main()
