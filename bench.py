#!/usr/bin/env python3
"""Benchmark: device-resident chunk reduce on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Step = one pass of the hot path over one batch of synthetic input: one
pgk_reduce (include/pgk.h -- the kernel that replaces the reference's
reduce_inplace, src/pg.c:151-159) of a device-resident chunk, BASELINE config 2:
DT_DOUBLE OP_SUM over 256 MiB (dst op= src).  Inputs are resident in HBM
before the timed region; 4 dst/src pairs (2 GiB) rotate so the 256 MiB
Infinity Cache cannot serve them.

At N > 1 every rank (one process per GPU) runs the same per-GPU workload
concurrently: weak scaling, no collective in the data path of the measured
step.  The ring itself (RCCL over xGMI + the same kernel, through the public
pg_reduce_scatter) is timed after the main measurement and reported in the
same JSON line under "ring" (BASELINE configs 3/4 shapes).

value      = whole-job GiB/s of algorithmic HBM traffic, 3 * n * 8 bytes per
             step (read dst, read src, write dst), summed over ranks, divided by
             the max-over-ranks wall time of the K timed steps.
roofline   = the kernel's achieved GB/s: the same bytes / the mean launch duration
             (HIP events bracketing the K timed launches on the launch stream,
             divided by K) against 8000 GB/s HBM3E peak; kernel-stamped
             per-launch times from an untimed pass are reported beside it.
cpu_baseline = the reference's own reduce loop (oracle/_ref, compiled from the
             reference src/pg.c) or its C restatement, 1 pinned host core,
             rank 0 at N = 1 only, on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pgamd  # noqa: E402

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
N_ELEMS = 1 << 25                # 256 MiB of float64 (BASELINE config 2)
N_PAIRS = 4                      # 4 x (dst, src) = 2 GiB > 256 MiB MALL
DT, OP = pgamd.DT_DOUBLE, pgamd.OP_SUM


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length")
    ap.add_argument("--cpu-procs", type=int, default=8,
                    help="CPU baseline: also time this many concurrent reference processes (0/1: skip)")
    ap.add_argument("--no-ring", action="store_true", help="skip the RCCL ring leg at N > 1")
    ap.add_argument("--ring-steps", type=int, default=3)
    ap.add_argument("--ring-timeout", type=float, default=300.0, help="watchdog for the ring leg (s)")
    ap.add_argument("--transports", default="xgmi,xgmi_push,xgmi_read,rccl",
                    help="ring-leg transports, comma separated (rccl last, so a stalled RCCL leg cannot take "
                         "the tested xgmi rows with it; xgmi = the library default, PG_XGMI_MODE=auto; "
                         "xgmi_push / xgmi_read = the mode forced, correctness probe and timed call only)")
    ap.add_argument("--ring-div", type=int, default=1,
                    help="divide the ring-leg element counts (one-GPU rehearsals over RCCL's socket transport "
                         "only; the driver's runs keep the BASELINE shapes)")
    ap.add_argument("--time-budget", type=float, default=480.0,
                    help="seconds since start after which no further optional leg is started (it is recorded as "
                         "skipped instead); the primary line always prints.  The driver gives one run 600 s")
    ap.add_argument("--preflight", default=None, metavar="TRANSPORTS",
                    help="(internal) child mode: two small checked calls per listed transport, nothing else; "
                         "at N > 1 every rank starts one such child before it touches the GPU itself")
    ap.add_argument("--no-preflight", action="store_true",
                    help="skip the ring legs' preflight children (N > 1)")
    ap.add_argument("--no-host", action="store_true", help="skip the host-memory (PCIe-inclusive) leg")
    ap.add_argument("--no-sizes", action="store_true", help="skip the 64 MiB .. 1 GiB kernel size table")
    return ap.parse_args()


def rank_setup(args):
    """Rank, world size and this rank's device number from the launcher's
    environment.  Touches no GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    on_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > 1 and os.environ.get("PG_BENCH_ONE_GPU") != "1" and torch.cuda.device_count() < on_node:
        # (device_count() initialises nothing, and every rank of the node gets the same
        # answer.)  More ranks than GPUs: the run can only be the one-GPU rehearsal, at its
        # sizes; the line says so instead of the launch failing
        os.environ["PG_BENCH_ONE_GPU"] = "1"
        os.environ["PG_BENCH_ONE_GPU_AUTO"] = "1"
        if args.ring_div == 1:
            args.ring_div = 4 if world <= 4 else 8
    if os.environ.get("PG_BENCH_ONE_GPU") == "1":   # rehearsal of the N>1 path on a 1-GPU box
        local = 0
        os.environ["PG_DEVICE"] = "0"
        # RCCL refuses two ranks on one device (its check compares host hash and
        # bus id): a host id per rank makes it treat the ranks as separate nodes,
        # so the rccl leg and the RCCL-native cross-check run over its socket
        # transport on loopback (tests/test_rccl_gpu.py)
        os.environ["NCCL_HOSTID"] = f"pg-bench-rehearsal-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    return rank, world, local


def dist_setup(rank, world):
    """The control plane: gloo over CPU tensors only.  Touches no GPU."""
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)


_T0 = time.perf_counter()
_LEG_INPUT = {}                # (count, dt) -> the ring legs' shared input tensor (ring_leg)


def progress(rank, msg):
    """One line per leg on stderr (rank-tagged, seconds since start): the
    driver and gpurun read a silent run as hung, and a stalled leg is named."""
    print(f"[bench r{rank} +{time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


_BUDGET_S = None               # --time-budget
_ELAPSED = {}                  # leg name -> seconds (rank 0's clock; reported under "elapsed_s")


def past_budget(world) -> bool:
    """True once the slowest rank's clock has passed --time-budget: every rank
    gets the same answer (one max-reduce), so a skipped leg is skipped by all."""
    if _BUDGET_S is None:
        return False
    return max_over_ranks(time.perf_counter() - _T0, world) > _BUDGET_S


class leg_clock:
    """with leg_clock("name"): ... -> _ELAPSED["name"] = seconds spent inside."""
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.t = time.perf_counter()

    def __exit__(self, *exc):
        _ELAPSED[self.name] = round(_ELAPSED.get(self.name, 0.0) + time.perf_counter() - self.t, 2)
        return False


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(x: float, rank: int, world: int) -> list:
    if world == 1:
        return [x]
    import torch.distributed as dist
    t = torch.zeros(world, dtype=torch.float64)
    t[rank] = x
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t]


def sum_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def kernel_leg(lib, args, rank, world):
    """The timed steps.  Returns wall seconds of the K timed steps, the mean
    launch duration over them (HIP events bracketing the timed region on the
    launch stream, / K), and kernel-stamped per-launch durations from an
    untimed cross-check pass."""
    # one allocation carved into N_PAIRS adjacent (dst, src) pairs, as the size
    # table does: operand placement moves this kernel by 1-5 % (measured:
    # "placement"), and separate torch allocations land wherever the caching
    # allocator puts them, so the primary figure would depend on what ran before
    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    pool = torch.empty(2 * N_PAIRS * N_ELEMS, dtype=torch.float64, device="cuda")
    pool.uniform_(-1.0, 1.0, generator=g)
    dst = [pool[(2 * i) * N_ELEMS:(2 * i + 1) * N_ELEMS] for i in range(N_PAIRS)]
    src = [pool[(2 * i + 1) * N_ELEMS:(2 * i + 2) * N_ELEMS] for i in range(N_PAIRS)]
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    def step(i, ev=None):
        d, s = dst[i % N_PAIRS].data_ptr(), src[i % N_PAIRS].data_ptr()
        rc = (lib.pgk_reduce_timed(d, s, N_ELEMS, DT, OP, sh, ev[0], ev[1]) if ev
              else lib.pgk_reduce(d, s, N_ELEMS, DT, OP, sh))
        if rc != 0:
            raise RuntimeError(pgamd.last_error())

    for i in range(args.warmup):
        step(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for i in range(args.steps):
        step(i)
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    region_mean_ms = e0.elapsed_time(e1) / args.steps

    # untimed cross-check: each launch stamped by its own dispatch
    # (hipExtLaunchKernelGGL start/stop events), the figure rocprofv3 reports
    stamped = []
    for i in range(min(args.steps, 20)):
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        pgamd.check(lib.pgk_event_create(ctypes.byref(a)), "event")
        pgamd.check(lib.pgk_event_create(ctypes.byref(b)), "event")
        step(i, (a, b))
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        pgamd.check(lib.pgk_event_elapsed_ms(a, b, ctypes.byref(ms)), "elapsed")
        stamped.append(ms.value)
        lib.pgk_event_destroy(a)
        lib.pgk_event_destroy(b)
    del dst, src, pool
    torch.cuda.empty_cache()
    return t1 - t0, region_mean_ms, stamped


def sustained_leg(lib, rank, world, seconds=2.0, batch=200):
    """The config-2 launch held for `seconds` on every GPU at once (the timed
    steps above last a few milliseconds): back-to-back pgk_reduce launches of
    256 MiB doubles over 4 rotating pairs, one HIP event per `batch` launches.
    Reports the rate of every batch window (min / median / max over windows,
    slowest rank per window) so that a clock or thermal droop over time shows."""
    pool = torch.empty(2 * N_PAIRS * N_ELEMS, dtype=torch.float64, device="cuda")
    pool.uniform_(-1e-3, 1e-3, generator=torch.Generator(device="cuda").manual_seed(4321 + rank))
    base, size = pool.data_ptr(), N_ELEMS * 8
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    nbatches = max(2, int(seconds / (batch * 125e-6)))
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(nbatches + 1)]
    for i in range(8):
        lib.pgk_reduce(base + 2 * size * (i % N_PAIRS), base + 2 * size * (i % N_PAIRS) + size, N_ELEMS, DT, OP, sh)
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    evs[0].record(stream)
    k = 0
    for b in range(nbatches):
        for _ in range(batch):
            d = base + 2 * size * (k % N_PAIRS)
            k += 1
            if lib.pgk_reduce(d, d + size, N_ELEMS, DT, OP, sh) != 0:
                raise RuntimeError(pgamd.last_error())
        evs[b + 1].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    per = [evs[b].elapsed_time(evs[b + 1]) / batch for b in range(nbatches)]          # ms per launch, per window
    worst = [max_over_ranks(v, world) for v in per]                                    # slowest rank per window
    gbs = [3 * size / (v * 1e-3) / 1e9 for v in worst]
    del pool
    torch.cuda.empty_cache()
    return {"seconds": round(max_over_ranks(wall, world), 2), "launches": nbatches * batch, "window_launches": batch,
            "frac_min": round(min(gbs) / HBM_PEAK_GBS, 4), "frac_median": round(float(np.median(gbs)) / HBM_PEAK_GBS, 4),
            "frac_max": round(max(gbs) / HBM_PEAK_GBS, 4), "frac_first_window": round(gbs[0] / HBM_PEAK_GBS, 4),
            "frac_last_window": round(gbs[-1] / HBM_PEAK_GBS, 4),
            "note": "256 MiB double sum, back-to-back launches (kernel boundaries included), every rank at once; "
                    "each window = window_launches launches between two HIP events, slowest rank per window"}


# per operand: the in-ring launch sizes (4-32 MiB: PG_CHUNK_BYTES x PG_INFLIGHT) and north_star's >= 64 MiB
SWEEP_BYTES = (4 << 20, 16 << 20, 32 << 20, 64 << 20, 128 << 20, 256 << 20, 512 << 20, 1 << 30)
SWEEP_POOL = 4 << 30


def size_leg(lib, rank, world, reps=20):
    """The kernel on power-of-two chunks of 64 MiB .. 1 GiB per operand, int32
    and double sum (the metric's two cases), plus int32/double prod at 256 MiB.

    One 4 GiB pool is carved into dst/src pairs of the size under test and the
    launches rotate over all of them, so every launch streams from HBM (the
    pool is 16x the 256 MiB Infinity Cache).  Each row is timed like the
    primary measurement (HIP events bracketing `reps` launches on the launch
    stream) with every rank launching at once after a barrier; the row keeps
    the slowest rank's time."""
    pool = torch.empty(SWEEP_POOL // 8, dtype=torch.float64, device="cuda")
    pool.uniform_(-1.0, 1.0, generator=torch.Generator(device="cuda").manual_seed(99 + rank))
    base = pool.data_ptr()
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stamp = (ctypes.c_void_p(), ctypes.c_void_p())
    pgamd.check(lib.pgk_event_create(ctypes.byref(stamp[0])), "event")
    pgamd.check(lib.pgk_event_create(ctypes.byref(stamp[1])), "event")
    cases = [(pgamd.DT_DOUBLE, pgamd.OP_SUM, SWEEP_BYTES), (pgamd.DT_INT32, pgamd.OP_SUM, SWEEP_BYTES),
             (pgamd.DT_DOUBLE, pgamd.OP_PROD, (256 << 20,)), (pgamd.DT_INT32, pgamd.OP_PROD, (256 << 20,))]
    rows = []
    for dt, op, sizes in cases:
        for size in sizes:
            n = size // pgamd.ELEM_SIZE[dt]
            pairs = SWEEP_POOL // (2 * size)

            def launch(i, ev=None):
                d = base + 2 * size * (i % pairs)
                rc = (lib.pgk_reduce_timed(d, d + size, n, dt, op, sh, ev[0], ev[1]) if ev
                      else lib.pgk_reduce(d, d + size, n, dt, op, sh))
                if rc != 0:
                    raise RuntimeError(pgamd.last_error())

            for i in range(4):
                launch(i)
            torch.cuda.synchronize()
            barrier(world)
            e0.record(stream)
            for i in range(reps):
                launch(i)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = max_over_ranks(e0.elapsed_time(e1) / reps, world)
            gbs = 3 * size / (ms * 1e-3) / 1e9
            # kernel-stamped launches (the kernel alone, as rocprofv3 reports it)
            st = []
            for i in range(8):
                launch(i, stamp)
                torch.cuda.synchronize()
                v = ctypes.c_float()
                pgamd.check(lib.pgk_event_elapsed_ms(stamp[0], stamp[1], ctypes.byref(v)), "elapsed")
                st.append(v.value)
            sms = max_over_ranks(float(np.median(st)), world)
            sgbs = 3 * size / (sms * 1e-3) / 1e9
            rows.append(["f64" if dt == pgamd.DT_DOUBLE else "i32", "sum" if op == pgamd.OP_SUM else "prod",
                         size, round(ms * 1e3, 2), round(gbs, 1), round(gbs / HBM_PEAK_GBS, 4),
                         round(sms * 1e3, 2), round(sgbs / HBM_PEAK_GBS, 4)])
    # the per-launch edge: least-squares t = t0 + traffic / bw over the f64-sum rows >= 16 MiB
    # (a fixed ramp + drain per launch against a streaming rate)
    fit = {}
    for col, key in ((3, "events"), (6, "stamped")):
        pts = [(3 * r_[2], r_[col]) for r_ in rows if r_[0] == "f64" and r_[1] == "sum" and r_[2] >= (16 << 20)]
        if len(pts) >= 3:
            xs_, ys_ = np.array([p_[0] for p_ in pts], dtype=np.float64), np.array([p_[1] for p_ in pts])
            slope, t0 = np.polyfit(xs_, ys_, 1)
            fit[key] = {"t0_us": round(float(t0), 2), "stream_GBps": round(float(1.0 / slope / 1e3), 1)}
    batches = ring_batch_rows(lib, base, sh, e0, e1, stamp, rank, world, reps)
    direct = direct_batch_rows(lib, base, sh, e0, e1, stamp, rank, world, reps)
    lib.pgk_event_destroy(stamp[0])
    lib.pgk_event_destroy(stamp[1])
    del pool
    torch.cuda.empty_cache()
    return {"columns": ["dtype", "op", "bytes_per_operand", "kernel_us", "GB/s", "frac", "stamped_us",
                        "stamped_frac"], "rows": rows, "edge_fit": fit, "ring_batches": batches,
            "direct_batches": direct,
            "timing": f"kernel_us: HIP events bracketing {reps} back-to-back launches rotating over a 4 GiB pool "
                      "(includes the ~1-2 us kernel boundaries), all ranks at once, slowest rank; stamped_us: median "
                      "of 8 kernel-stamped launches (hipExtLaunchKernelGGL events, the kernel alone as rocprofv3 "
                      "times it), slowest rank; GB/s and frac count 3 x bytes_per_operand (read dst, read src, "
                      "write dst) against 8000 GB/s"}


def _time_launches(launch, e0, e1, stamp, lib, world, reps):
    """(ms per launch from events bracketing `reps` back-to-back launches, ms of
    the median kernel-stamped launch), slowest rank."""
    for i in range(4):
        launch(i)
    torch.cuda.synchronize()
    barrier(world)
    e0.record(torch.cuda.current_stream())
    for i in range(reps):
        launch(i)
    e1.record(torch.cuda.current_stream())
    torch.cuda.synchronize()
    ms = max_over_ranks(e0.elapsed_time(e1) / reps, world)
    st = []
    for i in range(8):
        launch(i, stamp)
        torch.cuda.synchronize()
        v = ctypes.c_float()
        pgamd.check(lib.pgk_event_elapsed_ms(stamp[0], stamp[1], ctypes.byref(v)), "elapsed")
        st.append(v.value)
    return ms, max_over_ranks(float(np.median(st)), world)


def ring_batch_rows(lib, base, sh, e0, e1, stamp, rank, world, reps):
    """What one reduce launch of the ring executor costs.  pg_exec.c reduces the
    arrived segments of a round once PG_REDUCE_BYTES per operand are pending
    (default 128 MiB, or at the round's end), every ring's contiguous run as one
    range of ONE pgk_reduce_ranges launch.  Timed here alone, each ring's range
    in its own region of the 4 GiB pool, rotating, so every launch streams from
    HBM.  double sum.  First row = the library defaults; the second is a single
    transport group (4 MiB x 4 inflight x 2 rings), what PG_REDUCE_BYTES=0 or a
    round that short launches."""
    rows = []
    dt, op = pgamd.DT_DOUBLE, pgamd.OP_SUM
    VP, SZ = ctypes.c_void_p, ctypes.c_size_t
    for label, rings, rng in (("defaults: PG_REDUCE_BYTES 128 MiB, 2 rings", 2, 64 << 20),
                              ("one transport group: 4 MiB x 4 inflight x 2 rings", 2, 16 << 20),
                              ("64 MiB pending, 2 rings", 2, 32 << 20), ("256 MiB pending, 2 rings", 2, 128 << 20),
                              ("128 MiB, 1 ring", 1, 128 << 20), ("128 MiB, 4 rings", 4, 32 << 20),
                              ("one group of 1 MiB x 4 x 2 rings", 2, 4 << 20),
                              ("one group of 64 KiB x 4 x 2 rings", 2, 256 << 10)):
        stride = max(64 << 20, rng)               # one ring's range per region
        slots = (SWEEP_POOL // (2 * stride)) // rings

        def launch(i, ev=(None, None)):
            outs, bs, ns = (VP * rings)(), (VP * rings)(), (SZ * rings)()
            for g in range(rings):
                d = base + 2 * stride * ((i % slots) * rings + g)
                outs[g], bs[g], ns[g] = d, d + stride, rng // 8
            if lib.pgk_reduce_ranges(outs, outs, bs, ns, rings, dt, op, sh, ev[0], ev[1]) != 0:
                raise RuntimeError(pgamd.last_error())

        ms, sms = _time_launches(launch, e0, e1, stamp, lib, world, reps)
        traffic = 3 * rng * rings
        rows.append([label, rings, rng * rings, round(ms * 1e3, 2),
                     round(traffic / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), round(sms * 1e3, 2),
                     round(traffic / (sms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)])
    return {"columns": ["launch", "rings", "bytes_per_operand", "kernel_us", "frac", "stamped_us", "stamped_frac"],
            "rows": rows,
            "note": "one pgk_reduce_ranges launch of the ring executor (one range per ring), double sum; first row = "
                    "the library defaults"}


def direct_batch_rows(lib, base, sh, e0, e1, stamp, rank, world, reps, nsrc=8):
    """What one fold of the direct exchange costs (PG_ALGO=direct, the rccl
    transport's default on one node): the landed segments of one ring part,
    folded from the W = 8 copies of the block (7 received + this rank's own) by
    ONE pgk_reduce_multi launch once PG_REDUCE_BYTES per source are pending over
    the rings (default 128 MiB: 64 MiB per ring at 2 rings); traffic (W+1) x
    bytes per source.  Sources rotate over the 4 GiB pool.  double sum."""
    rows = []
    dt, op = pgamd.DT_DOUBLE, pgamd.OP_SUM
    VP = ctypes.c_void_p
    for label, rng, burst, flags in (
            ("defaults: PG_REDUCE_BYTES 128 MiB, 2 rings; the GPU to itself (the last flush of a call)", 64 << 20, 1, 0),
            ("the same, one tile per wave (burst form off)", 64 << 20, 0, 0),
            ("the same, PGK_FOLD_SHARED_GPU (the flushes that run beside transfers): two 32 MiB launches", 64 << 20, 1,
             pgamd.FOLD_SHARED_GPU),
            ("one transport group: 4 MiB x 4 inflight", 16 << 20, 1, 0),
            ("32 MiB per source", 32 << 20, 1, 0), ("128 MiB per source", 128 << 20, 1, 0),
            ("one group of 1 MiB x 4", 4 << 20, 1, 0)):
        slot = max(64 << 20, rng)
        sets = SWEEP_POOL // (slot * (nsrc + 1))

        def launch(i, ev=(None, None)):
            b0 = base + slot * (nsrc + 1) * (i % sets)
            srcs = (VP * nsrc)(*[b0 + slot * j for j in range(nsrc)])
            if lib.pgk_fold_timed(b0 + slot * nsrc, srcs, nsrc, rng // 8, dt, op, flags, sh, ev[0], ev[1]) != 0:
                raise RuntimeError(pgamd.last_error())

        lib.pgk_tune_fold(burst)
        try:
            ms, sms = _time_launches(launch, e0, e1, stamp, lib, world, reps)
        finally:
            lib.pgk_tune_fold(1)
        traffic = (nsrc + 1) * rng
        rows.append([label, nsrc, rng, round(ms * 1e3, 2),
                     round(traffic / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), round(sms * 1e3, 2),
                     round(traffic / (sms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)])
    return {"columns": ["launch", "sources", "bytes_per_source", "kernel_us", "frac", "stamped_us", "stamped_frac"],
            "rows": rows,
            "note": "one pgk_reduce_multi call = one direct-exchange fold of one ring part (W = 8 sources), "
                    "(W+1) x bytes_per_source of traffic, double sum, local HBM sources; first row = the defaults. "
                    "From 32 MiB per source the call takes the burst form (launches of at most 64 MiB per source "
                    "in which every wave folds all its tiles before it stores any); row 2 is row 1 without it, "
                    "row 3 the form the direct exchange uses while transfers are still running (32 MiB launches "
                    "that leave half of every CU's registers to the transport's kernels)"}


def cpu_baseline(args):
    """Reference reduce loop on 1 pinned host core, bounded sample of the workload."""
    from oracle.pyoracle import REF_LIB, Oracle, Reference
    try:
        impl, kind = Reference(), "reference"
    except RuntimeError:
        impl, kind = Oracle(), "port"
    orc = Oracle()
    orig_aff = None
    try:
        orig_aff = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {sorted(orig_aff)[0]})
    except (AttributeError, OSError):
        pass
    n = N_ELEMS                                   # the same 256 MiB chunk
    d = orc.fill(n, DT, OP, 0x5EEDC0DE ^ (2 << 32))
    s = orc.fill(n, DT, OP, 0x5EEDC0DE ^ (2 << 32) ^ 1)
    impl.time_reduce(d, s, DT, OP, 1)             # touch pages
    reps, secs = 0, 0.0
    while secs < args.cpu_seconds:
        secs += impl.time_reduce(d, s, DT, OP, 1)
        reps += 1
    gibs = 3 * n * 8 * reps / secs / GIB
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    if orig_aff:
        try:
            os.sched_setaffinity(0, orig_aff)     # the rest of the bench (and the child below) unpinned
        except OSError:
            pass
    del d, s
    concurrent = None
    if args.cpu_procs > 1:       # W ranks of the reference at once, in a fresh child process
        import subprocess
        try:
            r = subprocess.run([sys.executable, "-m", "oracle.cpu_concurrent", "--procs", str(args.cpu_procs),
                                "--seconds", "5"], cwd=str(ROOT), capture_output=True, text=True, timeout=300)
            concurrent = (json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0
                          else {"error": r.stderr.strip()[-300:]})
        except Exception as e:  # noqa: BLE001 -- reported, never fatal for the primary line
            concurrent = {"error": f"{type(e).__name__}: {e}"}
    return {"value": round(gibs, 3), "unit": "GiB/s (3*n*8 B traffic)", "cores": 1, "kind": kind,
            "concurrent": concurrent,
            "payload_gibs": round(n * 8 * reps / secs / GIB, 3),
            "sample": f"{reps} x reduce_inplace(double, sum) over 256 MiB chunks, {secs:.1f} s, "
                      f"1 pinned core of {os.cpu_count()} ({cpu}); "
                      f"{'oracle/_ref = reference src/pg.c:151-159 compiled -O2' if kind == 'reference' else 'oracle/pg_oracle.c restatement -O2'}"}


def host_leg(lib, reps=3):
    """PCIe-inclusive rate of the same chunk reduce with dst/src in host memory
    (pgx_reduce_host: 16 MiB pieces, uploads + reduce on the calling thread,
    downloads on a helper thread, so both PCIe directions work at once).
    Reported, never `value`."""
    out = {}
    n = N_ELEMS
    for kind in ("pageable", "pinned"):
        d = torch.rand(n, dtype=torch.float64)
        s_ = torch.rand(n, dtype=torch.float64)
        if kind == "pinned":
            d, s_ = d.pin_memory(), s_.pin_memory()
        pgamd.check(lib.pgx_reduce_host(d.data_ptr(), s_.data_ptr(), n, DT, OP, 0), "host reduce")
        t0 = time.perf_counter()
        for _ in range(reps):
            pgamd.check(lib.pgx_reduce_host(d.data_ptr(), s_.data_ptr(), n, DT, OP, 0), "host reduce")
        dt_ = (time.perf_counter() - t0) / reps
        out[kind] = {"ms": round(dt_ * 1e3, 3), "traffic_gibs": round(3 * n * 8 / dt_ / GIB, 2),
                     "payload_gibs": round(n * 8 / dt_ / GIB, 2),
                     "pcie_gbs": round(3 * n * 8 / dt_ / 1e9, 2)}
        del d, s_
    out["note"] = ("256 MiB double sum, dst/src in host memory (pgx_reduce_host). pageable: 16 MiB pieces through "
                   "3 HBM slots, H2D dst+src and the reduce on one thread, D2H dst on another; pinned: one reduce "
                   "kernel on the mapped host pointers, reading and writing across PCIe at once. pcie_gbs counts "
                   "the 3*n*8 bytes that cross PCIe")
    return out


def config1_leg(lib):
    """BASELINE config 1 (2-rank ring, int32 sum, count 1,048,576): each rank
    reduces one 2 MiB block (524,288 elements).  CPU: the reference's own
    pg_reduce_scatter(W=2, R=0, chunk 2 MiB), which is exactly that one
    reduce_inplace.  GPU: pgk_reduce on the same block, kernel
    time and host-call wall time."""
    import statistics
    from oracle.pyoracle import Oracle, Reference
    n = 1 << 19
    out = {"block_bytes": n * 4}
    orc = Oracle()
    send = orc.fill(2 * n, pgamd.DT_INT32, 0, 11)
    recv = orc.fill(2 * n, pgamd.DT_INT32, 0, 12)
    try:
        ref = Reference()
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            ref.lib.ref_reduce_scatter(0, 2, n * 4, send.ctypes.data, recv.ctypes.data, 2 * n, 0, 0)
            ts.append(time.perf_counter() - t0)
        out["cpu_reference_us"] = round(statistics.median(ts) * 1e6, 2)
    except RuntimeError:
        out["cpu_reference_us"] = None
    d = torch.from_numpy(recv[n:]).cuda()
    s_ = torch.from_numpy(send[:n]).cuda()
    sh = torch.cuda.current_stream().cuda_stream
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    lib.pgk_event_create(ctypes.byref(a))
    lib.pgk_event_create(ctypes.byref(b))
    kt, wt = [], []
    for _ in range(200):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pgamd.check(lib.pgk_reduce_timed(d.data_ptr(), s_.data_ptr(), n, pgamd.DT_INT32, 0, sh, a, b), "cfg1")
        torch.cuda.synchronize()
        wt.append(time.perf_counter() - t0)
        ms = ctypes.c_float()
        lib.pgk_event_elapsed_ms(a, b, ctypes.byref(ms))
        kt.append(ms.value * 1e3)
    lib.pgk_event_destroy(a)
    lib.pgk_event_destroy(b)
    out["gpu_kernel_us"] = round(statistics.median(kt), 2)
    out["gpu_call_wall_us"] = round(statistics.median(wt) * 1e6, 2)
    out["note"] = "2 MiB is launch/latency-bound on the GPU (6 MiB of traffic = 1 us at HBM rate)"
    return out


def load_traffic():
    """HBM bytes per launch from the committed rocprofv3 PMC pass (see
    profiles/README.md): (FETCH_SIZE*2 + WRITE_SIZE) KiB per dispatch, gfx950
    FETCH_SIZE correction applied by tools/pmc_traffic.py."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    try:
        d = json.loads(p.read_text())
        return d.get("reduce_f64_sum_256MiB", {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def _timed_rs(lib, h, x, out, count, dt, op, reps, world):
    pgamd.check(lib.pg_reduce_scatter(x.data_ptr(), out.data_ptr(), count, dt, op, h), "ring RS")   # warm
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(reps):
        pgamd.check(lib.pg_reduce_scatter(x.data_ptr(), out.data_ptr(), count, dt, op, h), "ring RS")
    barrier(world)
    return max_over_ranks(time.perf_counter() - t0, world) / reps


def _pattern(count, rank, world, dt, op, off=0, ln=None, device="cuda"):
    """Inputs whose W-rank reduction is exact in both dtypes, so every rank can
    check its block on the device: sum -> (i % 1000) + rank; prod -> powers of
    two (double) / {1, 2, -1} (int32).  Elements [off, off + ln) of rank
    `rank`'s input (default: all `count`), built in the target dtype without
    full-size int64 temporaries.  (device="cpu": tests/test_bench_gloo.py pins
    these against the oracle's ring.)"""
    tdt = torch.int32 if dt == pgamd.DT_INT32 else torch.float64
    ln = count - off if ln is None else ln
    i = torch.arange(off, off + ln, device=device, dtype=torch.int64)
    if op == pgamd.OP_SUM:
        i.remainder_(1000).add_(rank)
        return i.to(tdt)
    i.add_(rank).remainder_(3)
    if dt == pgamd.DT_DOUBLE:
        return torch.pow(2.0, (i - 1).to(torch.float64))
    return torch.where(i == 2, -1, i + 1).to(torch.int32)


def _expected_block(count, off, ln, world, dt, op, device="cuda"):
    tdt = torch.int32 if dt == pgamd.DT_INT32 else torch.float64
    acc = None
    for q in range(world):
        v = _pattern(count, q, world, dt, op, off, ln, device).to(torch.float64 if dt == pgamd.DT_DOUBLE else torch.int64)
        acc = v if acc is None else (acc + v if op == pgamd.OP_SUM else acc * v)
    if dt == pgamd.DT_INT32:
        acc = ((acc + 2**31) % 2**32 - 2**31)
    return acc.to(tdt)


_NCCL_GROUP = None


def _nccl_group():
    """An RCCL process group beside the gloo control plane (backend "nccl" is
    RCCL on ROCm), created collectively on first use."""
    global _NCCL_GROUP
    if _NCCL_GROUP is None:
        import torch.distributed as dist
        _NCCL_GROUP = dist.new_group(backend="nccl")
    return _NCCL_GROUP


def native_crosscheck(lib, h, rank, world, x_full, dt_full):
    """pg_reduce_scatter against RCCL's own reduce-scatter.

    Random inputs, 16 Mi elements per rank (a multiple of W, so both libraries
    use the same uniform blocks): full-range int32 for sum and product, U[-1,1)
    doubles for sum, 1 + U[-2^-10, 2^-10) doubles for product (normal over 8
    ranks).  int32: bit-exact (wrapping + and * do not depend on the order).
    double: the two libraries fold the W values in different orders, and each
    order is within g of the exact result (g = (W-1)u/(1-(W-1)u), u = 2^-53):
    g*sum|x| for the sum, g*|prod x| for the product.  So |ours - rccl| <=
    2*g*sum|x| (sum|x| from an RCCL reduce-scatter of |x|) and <= 2*g/(1-g)*|rccl|
    (product) element-wise.  Also times RCCL's reduce-scatter on the leg's
    full-size input beside ours."""
    import torch.distributed as dist
    grp = _nccl_group()
    n = ((1 << 24) // world) * world
    gen = torch.Generator(device="cuda").manual_seed(777 + rank)
    res = {}
    k = (world - 1) * 2.0**-53
    g = k / (1 - k)
    for dt, op in ((pgamd.DT_INT32, pgamd.OP_SUM), (pgamd.DT_DOUBLE, pgamd.OP_SUM),
                   (pgamd.DT_INT32, pgamd.OP_PROD), (pgamd.DT_DOUBLE, pgamd.OP_PROD)):
        tag = ("i32_" if dt == pgamd.DT_INT32 else "f64_") + ("sum" if op == pgamd.OP_SUM else "prod")
        if dt == pgamd.DT_INT32:
            x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=gen)
        elif op == pgamd.OP_SUM:
            x = torch.rand(n, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
        else:
            x = 1 + (torch.rand(n, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1) * 2.0**-10
        ln = n // world
        ours = torch.empty(ln, dtype=x.dtype, device="cuda")
        nat = torch.empty(ln, dtype=x.dtype, device="cuda")
        rop = dist.ReduceOp.SUM if op == pgamd.OP_SUM else dist.ReduceOp.PRODUCT
        torch.cuda.synchronize()
        pgamd.check(lib.pg_reduce_scatter(x.data_ptr(), ours.data_ptr(), n, dt, op, h), "RS")
        dist.reduce_scatter_tensor(nat, x, op=rop, group=grp)
        torch.cuda.synchronize()
        if dt == pgamd.DT_INT32:
            ok = bool(torch.equal(ours, nat))
            res[tag + "_bit_exact"] = sum_over_ranks(1.0 if ok else 0.0, world) == world
        else:
            if op == pgamd.OP_SUM:
                sabs = torch.empty_like(nat)
                dist.reduce_scatter_tensor(sabs, x.abs(), group=grp)
                torch.cuda.synchronize()
                tol = 2 * g * sabs
            else:
                tol = 2 * g / (1 - g) * nat.abs()
            diff = (ours - nat).abs()
            worst = float((diff / tol.clamp_min(1e-300)).max())
            ident = float((ours == nat).double().mean())
            res[tag + "_within_tol"] = sum_over_ranks(1.0 if worst <= 1.0 else 0.0, world) == world
            res[tag + "_max_diff_over_tol"] = round(max_over_ranks(worst, world), 4)
            res[tag + "_bit_identical_frac"] = round(sum_over_ranks(ident, world) / world, 4)
        del x, ours, nat
    res["f64_sum_tolerance"] = "|ours - rccl| <= 2*g*sum|x|, g = (W-1)*2^-53/(1-(W-1)*2^-53)"
    res["f64_prod_tolerance"] = "|ours - rccl| <= 2*g/(1-g)*|rccl|, g as above"
    # the other two collectives on int32 (order-independent, so bit-exact):
    # pg_all_reduce against RCCL's all-reduce, pg_all_gather against its all-gather
    x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=gen)
    ours = torch.empty_like(x)
    torch.cuda.synchronize()
    pgamd.check(lib.pg_all_reduce(x.data_ptr(), ours.data_ptr(), n, pgamd.DT_INT32, pgamd.OP_SUM, h), "AR")
    nat = x.clone()
    dist.all_reduce(nat, group=grp)
    torch.cuda.synchronize()
    res["i32_all_reduce_bit_exact"] = sum_over_ranks(1.0 if torch.equal(ours, nat) else 0.0, world) == world
    del ours, nat
    m = n // world
    ours = torch.empty(m * world, dtype=torch.int32, device="cuda")
    nat = torch.empty_like(ours)
    pgamd.check(lib.pg_all_gather(x.data_ptr(), ours.data_ptr(), m, pgamd.DT_INT32, h), "AG")
    dist.all_gather_into_tensor(nat, x[:m], group=grp)
    torch.cuda.synchronize()
    res["i32_all_gather_bit_exact"] = sum_over_ranks(1.0 if torch.equal(ours, nat) else 0.0, world) == world
    del x, ours, nat
    # RCCL's own reduce-scatter on the leg's full input, timed like ours
    m = (x_full.numel() // world) * world
    nat = torch.empty(m // world, dtype=x_full.dtype, device="cuda")
    dist.reduce_scatter_tensor(nat, x_full[:m], group=grp)         # warm
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(3):
        dist.reduce_scatter_tensor(nat, x_full[:m], group=grp)
    torch.cuda.synchronize()
    barrier(world)
    res["rccl_reduce_scatter_ms"] = round(max_over_ranks(time.perf_counter() - t0, world) / 3 * 1e3, 3)
    del nat
    torch.cuda.empty_cache()
    return res


def _phases(h, rank, world):
    """pg_get_stats of the last call, slowest rank per field: where the time of
    one reduce-scatter goes (device part of the ring, or the xgmi transport's
    sync / copy / barrier / fold phases) and the bytes a rank received."""
    st = pgamd.stats(h)
    keys = ("wall_us", "ring_us", "sync_us", "copy_us", "barrier_us", "kernel_us")
    out = {k: round(max_over_ranks(float(st[k]), world), 1) for k in keys}
    out["bytes_recv_per_rank"] = int(st["bytes_recv"])
    out["zero_copy"] = bool(st["zero_copy"])
    # an xgmi call whose peer input failed to map is redone with the slot copy:
    # correct, but it must show up in the record, not only as a slower number
    out["redone"] = sum_over_ranks(float(st["retried"]), world) > 0
    out["calls_redone_total"] = int(sum_over_ranks(float(st["calls_redone"]), world))
    t = out["kernel_us"] or out["ring_us"]
    out["recv_gbs_per_rank"] = round(st["bytes_recv"] / t / 1e3, 1) if t else None
    # the data path this handle actually runs, from the library itself (pg_get_stats)
    names = {pgamd.PG_TRANSPORT_RCCL: "rccl", pgamd.PG_TRANSPORT_XGMI: "xgmi"}
    out["path"] = {"transport": names.get(st["transport"], str(st["transport"])),
                   "schedule": ("push" if st["xgmi_push"] else "read") if st["transport"] == pgamd.PG_TRANSPORT_XGMI
                   else ("direct" if st["algo_direct"] else "ring"),
                   "chosen_by_probe": bool(st["xgmi_mode_auto"]),
                   "probe_read_gbs": round(st["probe_read_gbs"], 1), "probe_write_gbs": round(st["probe_write_gbs"], 1)}
    return out


def _small_calls(lib, h, rank, world, reps=50):
    """Config 5's eager-size calls on their own: 4 KiB per rank (512 doubles,
    product), reduce-scatter and all-reduce on device buffers, `reps` calls
    each; per-call wall time (median / p90 over calls, slowest rank) and the
    phase breakdown of the last call (pg_get_stats: wall, device part, and
    the xgmi transport's producer wait / barrier / kernel phases)."""
    count = 512
    x = _pattern(count, rank, world, pgamd.DT_DOUBLE, pgamd.OP_PROD)
    off, ln = pgamd.block_range(count, world, rank)
    out = {}
    for name in ("reduce_scatter", "all_reduce"):
        y = torch.empty(count if name == "all_reduce" else max(ln, 1), dtype=torch.float64, device="cuda")
        fn = lib.pg_all_reduce if name == "all_reduce" else lib.pg_reduce_scatter
        for _ in range(5):
            pgamd.check(fn(x.data_ptr(), y.data_ptr(), count, pgamd.DT_DOUBLE, pgamd.OP_PROD, h), name)
        barrier(world)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            pgamd.check(fn(x.data_ptr(), y.data_ptr(), count, pgamd.DT_DOUBLE, pgamd.OP_PROD, h), name)
            ts.append((time.perf_counter() - t0) * 1e6)
        barrier(world)
        want = _expected_block(count, 0 if name == "all_reduce" else off, count if name == "all_reduce" else ln,
                               world, pgamd.DT_DOUBLE, pgamd.OP_PROD)
        ok = bool(torch.equal(y[:want.numel()], want))
        st = pgamd.stats(h)
        out[name] = {"us_median": round(max_over_ranks(float(np.median(ts)), world), 1),
                     "us_p90": round(max_over_ranks(float(np.percentile(ts, 90)), world), 1),
                     "ok": sum_over_ranks(1.0 if ok else 0.0, world) == world,
                     "last_call": {k: round(max_over_ranks(float(st[k]), world), 1)
                                   for k in ("wall_us", "ring_us", "sync_us", "copy_us", "barrier_us", "kernel_us")}}
    out["shape"] = "512 doubles (4 KiB) per rank, OP_PROD, device buffers; per-call host wall time"
    return out


def _in_ring_reduce(lib, h, x, out, count, dt, rank, world):
    """The reduce launches inside the ring, measured: one more reduce-scatter
    with PG_KERNEL_TIMING=1, which stamps every executor launch with its own
    kernel begin/end (pg_exec.c); per rank, GB/s = 3 x reduced bytes / summed
    kernel time.  Untimed call: stamping costs a few us per launch."""
    os.environ["PG_KERNEL_TIMING"] = "1"
    try:
        pgamd.check(lib.pg_reduce_scatter(x.data_ptr(), out.data_ptr(), count, dt, pgamd.OP_SUM, h),
                    "ring RS (kernel-stamped)")
    finally:
        os.environ.pop("PG_KERNEL_TIMING", None)
    st = pgamd.stats(h)
    us = float(st["red_kernel_us"])
    moved = int(st["red_kernel_bytes"])       # 3*n*es per ring reduce, (W+1)*n*es per direct fold
    gbs = moved / us / 1e3 if us > 0 else 0.0
    per = gather_over_ranks(gbs, rank, world)
    launches = int(st["reduce_launches"])
    return {"launches_per_rank": launches, "kernel_us_per_rank": round(max_over_ranks(us, world), 1),
            "bytes_per_launch": int(moved / max(launches, 1)),
            "gbs_per_rank": {"min": round(min(per), 1), "median": round(float(np.median(per)), 1),
                             "max": round(max(per), 1)},
            "frac_min": round(min(per) / HBM_PEAK_GBS, 4),
            "timing": "PG_KERNEL_TIMING=1: each reduce launch kernel-stamped (pgk_reduce_ranges on the ring, "
                      "pgk_reduce_multi on the direct exchange and in the xgmi transport's fold); algorithmic bytes "
                      "(3*n*es per ring reduce, (W+1)*n*es per fold) / summed kernel time, one untimed reduce-scatter"}


SWEEP_COLUMNS = ["size", "rounds", "inflight", "time_us", "GB/s", "chunk_bytes", "is_default", "algo",
                 "in_ring_reduce_frac"]


def _sweep(lib, h, x, out, count, dt, rank, world, knob, values, algo):
    """One knob of one handle (one schedule) swept: PG_CHUNK_BYTES (config 3)
    or PG_INFLIGHT (config 4), set through the public struct pg fields as a
    reference harness would (include/pg.h).  Rows follow the reference's CSV
    discipline (README.md:85: size, rounds, inflight, time_us, GB/s) plus the
    knob, the schedule (`algo`) and the roofline fraction of the reduce launches
    inside that very configuration (one extra untimed call with
    PG_KERNEL_TIMING=1: slowest rank).  Stops early, marked, when the time
    budget runs out."""
    hd = pgamd.head(h)
    payload = count * pgamd.ELEM_SIZE[dt]
    default = int(getattr(hd, knob))
    rows, truncated = [], False
    for v in values:
        if past_budget(world):
            truncated = True
            break
        setattr(hd, knob, v)
        t = _timed_rs(lib, h, x, out, count, dt, pgamd.OP_SUM, 2, world)
        frac = _in_ring_reduce(lib, h, x, out, count, dt, rank, world)["frac_min"]
        rows.append([payload, world - 1, int(hd.inflight), round(t * 1e6, 1), round(payload / t / 1e9, 2),
                     int(hd.chunk_bytes), int(v == default), algo, frac])
    setattr(hd, knob, default)
    return rows, truncated


def _sweep_summary(rows, knob_col):
    """Per schedule: the fastest row and its gain over the default row."""
    out = {}
    for algo in sorted({r[7] for r in rows}):
        mine = [r for r in rows if r[7] == algo]
        best = max(mine, key=lambda r: r[4])
        dflt = [r for r in mine if r[6]]
        out[algo] = {"fastest": best[knob_col], "fastest_GBps": best[4],
                     "fastest_over_default": round(best[4] / dflt[0][4], 3) if dflt else None,
                     "in_ring_reduce_frac_at_default": dflt[0][8] if dflt else None}
    return out


def _ring_variant(lib, rank, world, x, out, count, dt, env, port_off, sweep=None):
    """The same timed reduce-scatter on a second handle (and RCCL communicator)
    opened with `env` (PG_ALGO / PG_RINGS): the W-1 round ring beside the
    default direct exchange, one clockwise ring (what the counter-rotating
    second ring buys), four rings (what two more rings of step +3 / -3 add).
    int32 results are checked against the default handle's.  sweep = (knob,
    values): also sweep that knob on this handle (rows under "sweep_rows")."""
    keys = ("PG_RINGS", "PG_PORT", "PG_ALGO")
    saved = {k: os.environ.get(k) for k in keys}
    os.environ.update(env)
    os.environ["PG_PORT"] = str(int(saved["PG_PORT"]) + port_off)   # no other leg uses it
    h1 = ctypes.c_void_p()
    try:
        if lib.connect_process_group(" ".join(["127.0.0.1"] * world).encode(), ctypes.byref(h1)) != 0:
            return {"error": "connect_process_group: " + pgamd.last_error()}
        ref = out.clone()
        wall = _timed_rs(lib, h1, x, out, count, dt, pgamd.OP_SUM, 3, world)
        same = bool(torch.equal(out, ref)) if dt == pgamd.DT_INT32 else None
        payload = count * pgamd.ELEM_SIZE[dt]
        rings = int(env.get("PG_RINGS", "2"))
        res = {"algo": env.get("PG_ALGO", "default"), "rings": rings,
               "steps": [pgamd.ring_offset(world, rings, g) for g in range(rings)],
               "ms_per_reduce_scatter": round(wall * 1e3, 3), "algbw_gibs": round(payload / wall / GIB, 2),
               "busbw_gibs": round(payload * (world - 1) / world / wall / GIB, 2)}
        if same is not None:
            res["int32_equal_to_default"] = sum_over_ranks(1.0 if same else 0.0, world) == world
        del ref
        res["in_ring_reduce"] = _in_ring_reduce(lib, h1, x, out, count, dt, rank, world)
        if sweep:
            res["sweep_rows"], res["sweep_truncated"] = _sweep(lib, h1, x, out, count, dt, rank, world, sweep[0],
                                                               sweep[1], env.get("PG_ALGO", "default"))
        return res
    finally:
        if h1.value:
            lib.pg_close(h1)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _link_probe(lib, h, rank, world, nbytes=256 << 20, reps=5):
    """Copy rates of this node's xGMI links as the xgmi transport uses them
    (pgx_xgmi_link_probe): one link pulled / pushed, all links pulled /
    pushed at once; GB/s per rank, min / median / max over ranks."""
    g = (ctypes.c_double * 4)()
    if lib.pgx_xgmi_link_probe(h, nbytes, reps, g) != 0:
        return {"error": pgamd.last_error()}
    out = {"bytes": nbytes, "reps": reps, "unit": "GB/s per rank (1e9 B/s moved by the rank)"}
    for i, name in enumerate(("read_one_link", "write_one_link", "read_all_links", "write_all_links")):
        per = gather_over_ranks(g[i], rank, world)
        out[name] = {"min": round(min(per), 1), "median": round(float(np.median(per)), 1), "max": round(max(per), 1)}
    return out


_PORT_OFFSET = {"rccl": 17, "xgmi": 19, "xgmi_push": 21, "xgmi_read": 23}


def _transport_env(transport, rank, world, port_shift=0):
    """Point the library's environment at one ring-leg transport; returns the
    server list for connect_process_group."""
    os.environ["PG_RANK"] = str(rank)
    os.environ["PG_TRANSPORT"] = "xgmi" if transport.startswith("xgmi") else transport
    os.environ["PG_XGMI_MODE"] = {"xgmi_push": "push", "xgmi_read": "read"}.get(transport, "auto")
    os.environ["PG_PORT"] = str(int(os.environ.get("MASTER_PORT", "29500")) + _PORT_OFFSET[transport] + port_shift)
    return " ".join(["127.0.0.1"] * world).encode()


# ---------------------------------------------------------------------------
# Preflight: the first exchange of every transport happens in a child process.
# A run on a node is the first time a rank's kernel reads (or writes) memory of
# another DEVICE; if that faulted inside the measuring process, the fault would
# end it and every rank with it, and the primary line would never print.  So
# each rank, BEFORE it touches the GPU itself (a process that has initialised
# the GPU starts no other program here), starts one child that makes two small
# checked calls per transport (4 KiB: the one-shot path; 8 MiB: the large
# path), reduce-scatter and all-reduce; the children are gone before the
# parents' first HIP call, and only transports whose children all finished
# clean get a leg.
PREFLIGHT_COUNTS = (512, 1 << 20)            # doubles
PREFLIGHT_TIMEOUT_S = 90.0
_PF_OK, _PF_NOT_REACHED, _PF_FAILED = 0, 1, 2


def preflight_child(args):
    """`bench.py --preflight a,b,c`: for each transport in turn print "start t",
    connect, run the checked calls, close, print "ok t" ("bad t: why" on a wrong
    result or an error return).  Exit 0 only if every transport was ok."""
    rank, world, local = rank_setup(args)
    torch.cuda.set_device(local)
    lib = pgamd.load()
    bad = 0
    for transport in args.preflight.split(","):
        print(f"start {transport}", flush=True)
        hosts = _transport_env(transport, rank, world, port_shift=40)
        why = None
        h = ctypes.c_void_p()
        if lib.connect_process_group(hosts, ctypes.byref(h)) != 0:
            why = "connect_process_group: " + pgamd.last_error()
        else:
            for count in PREFLIGHT_COUNTS:
                x = _pattern(count, rank, world, DT, OP)
                off, ln = pgamd.block_range(count, world, rank)
                out = torch.zeros(count, dtype=x.dtype, device="cuda")
                torch.cuda.synchronize()
                for name, fn, o, n in (("reduce_scatter", lib.pg_reduce_scatter, off, ln),
                                       ("all_reduce", lib.pg_all_reduce, 0, count)):
                    if fn(x.data_ptr(), out.data_ptr(), count, DT, OP, h) != 0:
                        why = why or f"{name}({count}): {pgamd.last_error()}"
                    elif not torch.equal(out[:n], _expected_block(count, o, n, world, DT, OP)):
                        why = why or f"{name}({count}): wrong result"
            lib.pg_close(h)
        print(f"ok {transport}" if why is None else f"bad {transport}: {why}", flush=True)
        bad += why is not None
    return 1 if bad else 0


def _run_preflight_child(transports, args):
    """Start this rank's child for `transports` and read what it got through:
    {transport: (code, detail)}.  The transport a child died in (signal, time
    limit, error exit before its "ok"/"bad" line) counts as failed.  Only ever
    called before this process has made its first GPU call."""
    import subprocess
    assert not torch.cuda.is_initialized(), "preflight children are started before the parent touches the GPU"
    cmd = [sys.executable, str(pathlib.Path(__file__).resolve()), "--preflight", ",".join(transports),
           "--gpus", str(args.gpus)]
    try:
        cp = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=PREFLIGHT_TIMEOUT_S,
                            text=True, errors="replace")
        lines, rc, err = cp.stdout.splitlines(), cp.returncode, cp.stderr
    except subprocess.TimeoutExpired as e:      # subprocess.run has killed the child
        raw = e.stdout or ""
        lines = (raw.decode(errors="replace") if isinstance(raw, bytes) else raw).splitlines()
        raw = e.stderr or ""
        rc, err = "time limit", raw.decode(errors="replace") if isinstance(raw, bytes) else raw
    return _read_preflight(transports, lines, rc, err)


def _read_preflight(transports, lines, rc, err=""):
    got = {t: (_PF_NOT_REACHED, "not reached") for t in transports}
    running = None
    for ln in lines:
        word, _, rest = ln.partition(" ")
        name = rest.split(":")[0]
        if word == "start" and name in got:
            running = name
        elif word == "ok" and name in got:
            got[name], running = (_PF_OK, "ok"), None
        elif word == "bad" and name in got:
            got[name], running = (_PF_FAILED, rest), None
    if running is not None:
        tail = [ln for ln in err.splitlines() if ln.strip()][-1:] or [""]
        end = f"signal {-rc}" if isinstance(rc, int) and rc < 0 else f"exit {rc}"
        got[running] = (_PF_FAILED, f"child ended in it ({end}): {tail[0][:200]}")
    return got


def preflight(args, rank, world, transports, run_child=_run_preflight_child):
    """{transport: None (every rank's child finished it clean) | reason}.  The
    ranks agree after each round of children (one max-reduce of the codes): the
    transports before the first one that failed anywhere are settled, that one
    is out, and the ones after it go to a fresh round of children, so one
    transport's fault does not cost the others their legs."""
    verdict, left = {}, list(transports)
    while left:
        got = run_child(left, args)
        codes = [got[t][0] for t in left]
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor(codes, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            worst = [int(v) for v in t]
        else:
            worst = codes
        cut = next((i for i, c in enumerate(worst) if c != _PF_OK), len(left))
        for t in left[:cut]:
            verdict[t] = None
        if cut < len(left):
            mine = got[left[cut]]
            verdict[left[cut]] = ("preflight failed on some rank; this rank: " + mine[1]) if mine[0] != _PF_OK \
                else "preflight failed on another rank (this rank's child finished it)"
        left = left[cut + 1:]
    return verdict


def ring_leg(lib, args, rank, world, transport, sink):
    """pg_reduce_scatter across the ranks, device-resident, BASELINE configs 3-5.
    transport: "rccl" (P2P ring over xGMI) or "xgmi" (direct peer reads).
    Rows of the sweeps follow the reference's CSV discipline (README.md:85):
    size, rounds, inflight, time_us, GB/s (GB/s = payload bytes per rank / time)."""
    if world == 4:
        dt, count, cfg = pgamd.DT_INT32, 1 << 28, "config3: 4-GPU ring, int32 sum, 1 GiB/rank"
    elif world == 8:
        dt, count, cfg = pgamd.DT_DOUBLE, 1 << 29, "config4: 8-GPU ring, double sum, 4 GiB/rank"
    else:
        dt, count, cfg = pgamd.DT_DOUBLE, 1 << 27, f"{world}-GPU ring, double sum, 1 GiB/rank"
    if args.ring_div > 1:
        count //= args.ring_div
        cfg += f" / {args.ring_div} (rehearsal size)"
    es = pgamd.ELEM_SIZE[dt]
    hosts = _transport_env(transport, rank, world)
    core_only = transport in ("xgmi_push", "xgmi_read")    # the correctness probe and the timed call
    h = ctypes.c_void_p()
    progress(rank, f"  {transport}: connect_process_group")
    if lib.connect_process_group(hosts, ctypes.byref(h)) != 0:
        raise RuntimeError("connect_process_group: " + pgamd.last_error())
    try:
        hd = pgamd.head(h)
        res = {"workload": cfg, "transport": {
            "rccl": "RCCL point-to-point over xGMI (PG_ALGO default: direct one-hop exchange on one node)",
            "xgmi": "direct peer access (HIP IPC) over xGMI, ring fold order; read or push chosen by the library's "
                    "connect-time link probe (PG_XGMI_MODE=auto)",
            "xgmi_read": "direct peer reads (HIP IPC) over xGMI, ring fold order (PG_XGMI_MODE=read)",
            "xgmi_push": "each block written to its owner over xGMI (HIP IPC), folded locally in ring order "
                         "(PG_XGMI_MODE=push)"}[transport]}
        if transport == "xgmi":
            push, rg, wg = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
            if lib.pgx_xgmi_mode(h, ctypes.byref(push), ctypes.byref(rg), ctypes.byref(wg)) == 0:
                res["mode"] = {"chosen": "push" if push.value else "read", "probe_read_gbs": round(rg.value, 1),
                               "probe_write_gbs": round(wg.value, 1),
                               "rule": "push when all-links write >= 1.15 x all-links read (32 MiB probe at connect)"}
        if os.environ.get("PG_BENCH_ONE_GPU") == "1":
            res["rehearsal"] = ("all ranks share one GPU; rccl runs over RCCL's socket transport on loopback "
                                "(NCCL_HOSTID per rank), xgmi's links are the one device's HBM: rates are not a node's")
        sink[transport] = res          # visible to the watchdog's print while the leg runs
        # every leg reads the SAME input allocation: a fresh tensor after the
        # previous leg's empty_cache() lands at the freed address under a new HIP
        # buffer id, and the xgmi transport never exports such a range (an importer may
        # still hold a mapping of the freed one): the forced-mode legs would then time the slot
        # copy instead of the zero-copy read they are there to compare
        x = _LEG_INPUT.get((count, dt))
        if x is None:
            _LEG_INPUT.clear()
            x = _LEG_INPUT[(count, dt)] = _pattern(count, rank, world, dt, pgamd.OP_SUM)
        off, ln = pgamd.block_range(count, world, rank)
        out = torch.empty(max(ln, 1), dtype=x.dtype, device="cuda")
        torch.cuda.synchronize()
        progress(rank, f"  {transport}: correctness probe, {count} elements")
        pgamd.check(lib.pg_reduce_scatter(x.data_ptr(), out.data_ptr(), count, dt, pgamd.OP_SUM, h), "ring RS")
        ok = bool(torch.equal(out[:ln], _expected_block(count, off, ln, world, dt, pgamd.OP_SUM)))
        res["ok"] = sum_over_ranks(1.0 if ok else 0.0, world) == world
        progress(rank, f"  {transport}: timed reduce-scatter")
        wall = _timed_rs(lib, h, x, out, count, dt, pgamd.OP_SUM, args.ring_steps, world)
        payload = count * es                       # per rank
        res["last_call_phases"] = _phases(h, rank, world)
        # the reduce launches inside this very call, kernel-stamped: the executor's
        # (rccl) or the transport's own multi-source fold (xgmi, whose sources are
        # its peers' memory: on a node this rate is the links', not local HBM's)
        res["in_ring_reduce"] = _in_ring_reduce(lib, h, x, out, count, dt, rank, world)
        res.update({"ms_per_reduce_scatter": round(wall * 1e3, 3),
                    "algbw_gibs": round(payload / wall / GIB, 2),
                    "busbw_gibs": round(payload * (world - 1) / world / wall / GIB, 2),
                    "reduced_traffic_gibs_per_gpu": round(3 * payload * (world - 1) / world / wall / GIB, 2),
                    "chunk_bytes": int(hd.chunk_bytes), "inflight": int(hd.inflight),
                    "algo": (os.environ.get("PG_ALGO") or "default") if transport == "rccl" else None,
                    "rings": int(os.environ.get("PG_RINGS", "2"))})
        if core_only:
            return res

        def optional(key, fn):
            """One optional part of the leg: skipped (and recorded as such) once the
            time budget is spent, timed, and never fatal for the leg."""
            if past_budget(world):
                res[key] = {"skipped": "time budget"}
                return
            progress(rank, f"  {transport}: {key}")
            with leg_clock(f"ring.{transport}.{key}"):
                try:
                    res[key] = fn()
                except Exception as e:  # noqa: BLE001 -- reported; the watchdog covers hangs
                    res[key] = {"error": f"{type(e).__name__}: {e}"}

        # 1. What BASELINE's configs 3 and 4 name: a RING with a PG_CHUNK_BYTES /
        # PG_INFLIGHT sweep.  The knobs exist on the point-to-point transport only
        # (xgmi reads whole blocks), and each sweep runs on both of its schedules:
        # the direct exchange (this handle, the default on one node) and the W-1
        # round ring (PG_ALGO=ring, two counter-rotating rings, a second handle).
        # Every row names its schedule and carries the roofline fraction of the
        # reduce launches inside it; by_algo names each schedule's fastest row and
        # its gain over that schedule's default row.
        sweep = None
        if transport == "rccl" and world == 4:
            sweep = ("chunk_bytes", [1 << e for e in range(16, 29)], "chunk_sweep", 5)   # 64 KiB .. 256 MiB
        if transport == "rccl" and world == 8:
            sweep = ("inflight", [1, 2, 4, 8, 16], "inflight_sweep", 2)
        own_algo = os.environ.get("PG_ALGO") or "direct"       # one node: the library's default schedule
        if sweep:
            def default_sweep():
                rows, cut = _sweep(lib, h, x, out, count, dt, rank, world, sweep[0], sweep[1], own_algo)
                return {"columns": SWEEP_COLUMNS, "rows": rows, "truncated_by_time_budget": cut}
            optional(sweep[2], default_sweep)
        if transport == "rccl" and os.environ.get("PG_RINGS", "2") == "2":
            optional("ring_algo", lambda: _ring_variant(lib, rank, world, x, out, count, dt,
                                                        {"PG_ALGO": "ring", "PG_RINGS": "2"}, 4,
                                                        (sweep[0], sweep[1]) if sweep else None))
            if sweep and "sweep_rows" in res["ring_algo"]:
                table = res[sweep[2]] if "rows" in res.get(sweep[2], {}) else {
                    "columns": SWEEP_COLUMNS, "rows": [], "truncated_by_time_budget": True}
                table["rows"] = table["rows"] + res["ring_algo"].pop("sweep_rows")
                table["truncated_by_time_budget"] |= res["ring_algo"].pop("sweep_truncated")
                res[sweep[2]] = table
        if sweep and res.get(sweep[2], {}).get("rows"):
            res[sweep[2]]["by_algo"] = _sweep_summary(res[sweep[2]]["rows"], sweep[3])

        # 2. config 5 (N = 8): products, eager size and 2 GiB mixed
        if world == 8:
            def config5():
                cfg5 = []
                for dt5, big in ((pgamd.DT_DOUBLE, 1 << 28), (pgamd.DT_INT32, 1 << 29)):
                    big //= max(args.ring_div, 1)              # 2 GiB per rank unless rehearsing
                    small = 4096 // pgamd.ELEM_SIZE[dt5]
                    for cnt in (small, big, small):
                        xv = _pattern(cnt, rank, world, dt5, pgamd.OP_PROD)
                        o5, l5 = pgamd.block_range(cnt, world, rank)
                        ov = torch.empty(max(l5, 1), dtype=xv.dtype, device="cuda")
                        reps = 20 if cnt == small else 2
                        t = _timed_rs(lib, h, xv, ov, cnt, dt5, pgamd.OP_PROD, reps, world)
                        good = bool(torch.equal(ov[:l5], _expected_block(cnt, o5, l5, world, dt5, pgamd.OP_PROD)))
                        good = sum_over_ranks(1.0 if good else 0.0, world) == world
                        row = {"dtype": "f64" if dt5 == pgamd.DT_DOUBLE else "i32", "count": cnt,
                               "bytes": cnt * pgamd.ELEM_SIZE[dt5], "time_us": round(t * 1e6, 1), "ok": good}
                        if cnt == small and transport == "rccl":
                            # eager one-shot (default) vs the W-1 round ring: eager_max = 0 disables it
                            hd.eager_max = 0
                            tr = _timed_rs(lib, h, xv, ov, cnt, dt5, pgamd.OP_PROD, reps, world)
                            hd.eager_max = 4096
                            row["time_us_ring_rounds"] = round(tr * 1e6, 1)
                        cfg5.append(row)
                        del xv, ov
                return cfg5
            optional("config5_prod_mixed", config5)

        # 3. the small calls, the links, the independent cross-check, host buffers
        optional("eager_4KiB", lambda: _small_calls(lib, h, rank, world))
        if transport == "xgmi":          # (one-GPU rehearsal: every "link" is the same device)
            optional("link_probe", lambda: _link_probe(lib, h, rank, world))
        optional("rccl_native", lambda: native_crosscheck(lib, h, rank, world, x, dt))

        def host_buffers():
            """The host-memory form of the same call: PCIe-inclusive (H2D + ring + D2H)."""
            xh = x.cpu().numpy()
            oh = np.empty(max(ln, 1), dtype=xh.dtype)
            barrier(world)
            t0 = time.perf_counter()
            pgamd.check(lib.pg_reduce_scatter(xh.ctypes.data, oh.ctypes.data, count, dt, pgamd.OP_SUM, h), "host RS")
            barrier(world)
            th = max_over_ranks(time.perf_counter() - t0, world)
            same = np.array_equal(oh[:ln], _expected_block(count, off, ln, world, dt, pgamd.OP_SUM).cpu().numpy())
            return {"ms": round(th * 1e3, 2), "ok": sum_over_ranks(1.0 if same else 0.0, world) == world}
        optional("host_buffers", host_buffers)

        # 4. what the second ring and further rings buy (P2P ring schedule)
        if transport == "rccl" and os.environ.get("PG_RINGS", "2") == "2":
            optional("one_ring", lambda: _ring_variant(lib, rank, world, x, out, count, dt,
                                                       {"PG_ALGO": "ring", "PG_RINGS": "1"}, 6))
            if world >= 5:
                optional("four_rings", lambda: _ring_variant(lib, rank, world, x, out, count, dt,
                                                             {"PG_ALGO": "ring", "PG_RINGS": "4"}, 8))
        del x, out
        torch.cuda.empty_cache()
        return res
    finally:
        lib.pg_close(h)


def main():
    global _BUDGET_S
    args = parse()
    if args.preflight:
        sys.exit(preflight_child(args))
    _BUDGET_S = args.time_budget if args.time_budget > 0 else None
    rank, world, local = rank_setup(args)
    dist_setup(rank, world)
    # the ring legs' preflight children run now, while this process has not made
    # a single GPU call (see "Preflight" above), and have ended before it does
    pf = None
    if world > 1 and not args.no_ring and not args.no_preflight:
        progress(rank, "preflight children (two small checked calls per ring transport)")
        with leg_clock("ring.preflight"):
            pf = preflight(args, rank, world, args.transports.split(","))
    torch.cuda.set_device(local)
    lib = pgamd.load()
    # the size table first: the primary measurement then starts on a GPU already at its streaming clocks
    sizes = None
    if not args.no_sizes:
        progress(rank, "kernel size table")
        with leg_clock("kernel_sizes"):
            try:
                sizes = size_leg(lib, rank, world)
            except Exception as e:  # noqa: BLE001 -- reported, never fatal for the primary line
                sizes = {"error": f"{type(e).__name__}: {e}"}

    progress(rank, f"kernel leg (world {world}, device {local})")
    with leg_clock("kernel_leg"):
        wall, region_mean_ms, stamped_ms = kernel_leg(lib, args, rank, world)
    wall_max = max_over_ranks(wall, world)
    bytes_per_step = 3 * N_ELEMS * 8
    per_rank_ms = gather_over_ranks(region_mean_ms, rank, world)
    mean_launch_ms = sum(per_rank_ms) / world
    achieved_gbs = bytes_per_step / (mean_launch_ms * 1e-3) / 1e9
    value = world * bytes_per_step * args.steps / wall_max / GIB

    sustained = None
    if not args.no_sizes:
        progress(rank, "sustained kernel leg")
        with leg_clock("kernel_sustained"):
            try:
                sustained = sustained_leg(lib, rank, world)
            except Exception as e:  # noqa: BLE001 -- reported, never fatal for the primary line
                sustained = {"error": f"{type(e).__name__}: {e}"}

    cpu = None
    host = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        progress(rank, "cpu baseline")
        with leg_clock("cpu_baseline"):
            cpu = cpu_baseline(args)
    if world == 1 and not args.no_host:
        progress(rank, "host-memory leg")
        with leg_clock("host_staged"):
            try:
                host = host_leg(lib)
            except Exception as e:
                host = {"error": f"{type(e).__name__}: {e}"}
    cfg1 = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        with leg_clock("config1"):
            try:
                cfg1 = config1_leg(lib)
            except Exception as e:
                cfg1 = {"error": f"{type(e).__name__}: {e}"}

    line = None
    if rank == 0:
        traffic = load_traffic()
        line = {
            "metric": "GiB/s device-resident chunk reduce (int32 sum, double sum) at 1/2/4/8 GPU",
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (uniform [-1,1) doubles, HBM-resident, 4 rotating 256 MiB dst/src pairs carved from one 2 GiB allocation)",
            "config": {"workload": "BASELINE config 2: pgk_reduce DT_DOUBLE OP_SUM, 256 MiB chunk per GPU "
                                   "(dst op= src), one reduce per step per GPU",
                       "chunk_bytes": N_ELEMS * 8, "bytes_per_step_per_gpu": bytes_per_step,
                       "parallelism": f"replicated per GPU x{world}"},
            "payload_gibs": round(value / 3, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel_mean_ms": round(mean_launch_ms, 5),
                         "timing": "HIP events bracketing the K timed launches on the launch stream, / K "
                                   "(includes the ~1 us kernel boundaries)",
                         "kernel_stamped_mean_ms": round(float(np.mean(stamped_ms)), 5),
                         "kernel_stamped_min_ms": round(float(np.min(stamped_ms)), 5),
                         "bytes_per_launch": bytes_per_step,
                         "per_gpu_gbs": None if world == 1 else {
                             "min": round(bytes_per_step / max(per_rank_ms) / 1e6, 1),
                             "median": round(bytes_per_step / float(np.median(per_rank_ms)) / 1e6, 1),
                             "max": round(bytes_per_step / min(per_rank_ms) / 1e6, 1)}},
            "kernel_sizes": sizes,
            "kernel_sustained": sustained,
            "cpu_baseline": cpu,
            "host_staged": host,
            "config1": cfg1,
            "ring": None,
            "kernel": lib.pgk_version().decode(),
            "one_gpu_rehearsal": (None if os.environ.get("PG_BENCH_ONE_GPU") != "1" else
                                  "every rank shares GPU 0" + (" (chosen by bench.py: fewer GPUs than ranks)"
                                                               if os.environ.get("PG_BENCH_ONE_GPU_AUTO") else "")
                                  + ": value, roofline and ring rates are not a node's"),
            "elapsed_s": _ELAPSED,       # per leg, filled in place; "total" is set just before printing
            "time_budget_s": _BUDGET_S,
        }

    if world > 1 and not args.no_ring:
        # the ring leg must never cost the primary line: a watchdog prints it
        # and ends every rank if the ring (RCCL init, a transfer) stalls
        import threading

        ring = {}
        if line is not None:
            line["ring"] = ring        # filled in place: a watchdog print keeps finished legs

        def _expire():
            if line is not None:
                ring["watchdog"] = (f"ring leg exceeded {args.ring_timeout} s; the leg that was running is "
                                    "reported up to where it stopped, later ones are omitted")
                _ELAPSED["total"] = round(time.perf_counter() - _T0, 2)
                txt = None
                for _ in range(20):          # the main thread may be adding to the ring dict right now
                    try:
                        txt = json.dumps(line)
                        break
                    except (RuntimeError, ValueError):
                        time.sleep(0.05)
                if txt is None:
                    txt = json.dumps({k: v for k, v in line.items() if k != "ring"})
                print(txt, flush=True)
            # a stalled ring is a failed run, whatever was printed: every rank
            # exits non-zero so the driver never records it as clean
            print(f"[bench r{rank}] ring watchdog expired after {args.ring_timeout} s", file=sys.stderr, flush=True)
            os._exit(3)

        dog = threading.Timer(args.ring_timeout, _expire)
        dog.daemon = True
        dog.start()
        if pf is not None and line is not None:
            line["ring_preflight"] = {t: ("ok" if why is None else why) for t, why in pf.items()}
        for transport in args.transports.split(","):
            if pf is not None and pf[transport] is not None:
                ring[transport] = {"error": "no leg: " + pf[transport]}
                continue
            if past_budget(world):           # the same answer on every rank
                ring[transport] = {"skipped": "time budget"}
                continue
            progress(rank, f"ring leg: {transport}")
            with leg_clock(f"ring.{transport}"):
                try:
                    ring_leg(lib, args, rank, world, transport, ring)
                except Exception as e:  # the primary measurement stands on its own
                    ring.setdefault(transport, {})["error"] = f"{type(e).__name__}: {e}"
            barrier(world)
        dog.cancel()

    if line is not None:
        _ELAPSED["total"] = round(time.perf_counter() - _T0, 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
