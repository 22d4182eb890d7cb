#!/usr/bin/env python3
"""EXPERIMENTS ONLY: where one reduce launch's time goes, from per-workgroup
timestamps (tools/lab/timeline_lab.hip, s_memrealtime at 100 MHz).

For each operand size and tile shape, over a 4 GiB pool (HBM-resident), the
diagnostic build is launched kernel-stamped (hipExtLaunchKernelGGL events, the
figure rocprofv3 reports) and every block's entry / loads-returned /
stores-acknowledged times are read back.  Per launch:

  stamped     begin->end event time of the launch
  span        first block entry -> last block's stores acknowledged
  outside     stamped - span: dispatch of the first wave + end-of-kernel
              completion (nothing of the kernel runs)
  dispatch    first -> last block entry of the first resident round
              (blocks that start before any block has finished)
  first_load  first block: entry -> its loads returned (one loaded HBM round trip)
  steady      bytes / time slope of block completions between 20% and 80%
  head        time before completions follow the steady line (ramp)
  tail        last completion minus the steady line's end (drain, incl. XCD imbalance)
  xcd_end     spread of the 8 XCDs' last completions

The shipped pgk_reduce is stamped beside it at the same size, so the build's
perturbation (its waits) is visible; the shares, not the diagnostic's length,
are the result.

    python tools/lab/run_timeline_lab.py [sizes in MiB ...]      (default 16 64 256)
"""
import ctypes
import pathlib
import statistics
import subprocess
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

so = HERE / "libtimelinelab.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    str(HERE / "timeline_lab.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
VP = ctypes.c_void_p
lab.tl_launch.argtypes = [ctypes.c_int, VP, VP, ctypes.c_size_t, VP, VP, VP, VP]
lab.tl_grid.argtypes = [ctypes.c_int, ctypes.c_size_t]
lab.tl_grid.restype = ctypes.c_uint
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
khz = ctypes.c_int()
assert lab.tl_clock_khz(ctypes.byref(khz)) == 0
TICK_US = 1e3 / khz.value                       # 100 MHz -> 0.01 us
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
SHAPES = {0: "512x2", 1: "1024x1", 2: "512x2 swapped", 3: "1024x1 swapped"}
REPS = 8


def elapsed_us():
    ms = ctypes.c_float()
    pgamd.check(lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)), "elapsed")
    return ms.value * 1e3


def analyse(ts, tile_bytes, stamped, factor=3.0):
    ent, ld, st, xcc = (ts[:, 0].astype(np.int64), ts[:, 1].astype(np.int64), ts[:, 2].astype(np.int64),
                        ts[:, 3].astype(np.int64))
    t0 = ent.min()
    ent, ld, st = (ent - t0) * TICK_US, (ld - t0) * TICK_US, (st - t0) * TICK_US
    span = st.max()
    first_done = st.min()
    first_round = ent < first_done
    order = np.argsort(st)
    done = st[order]
    cum = np.arange(1, len(done) + 1) * factor * tile_bytes
    lo, hi = int(0.2 * len(done)), int(0.8 * len(done))
    k, a = np.polyfit(cum[lo:hi], done[lo:hi], 1)          # t = a + k * bytes
    total = cum[-1]
    first_blk = np.argmin(ent)
    xcd_last = [st[xcc == x].max() for x in np.unique(xcc)]
    per_xcd = {int(x): (int((xcc == x).sum()), span - st[xcc == x].max(),
                        factor * tile_bytes * (xcc == x).sum() / (st[xcc == x].max() - ent[xcc == x].min()) / 1e3)
               for x in np.unique(xcc)}
    # block b -> XCD (b + c) mod 8 under strict round-robin dealing: the set of c over the launch
    cset = sorted(set(((xcc - np.arange(len(xcc))) % 8).tolist()))
    # streaming rate in each tenth of the span (completions' bytes / time): does it decay along a long launch?
    edges = np.linspace(0, span, 11)
    cnt = np.histogram(st, bins=edges)[0]
    deciles = (cnt * factor * tile_bytes / (span / 10) / 1e3).tolist()
    # how far apart in the buffer are the tiles finishing together?  5-95% range of the block
    # index (= tile index in the unswapped shapes) among the blocks completing in each tenth, in MiB
    # per operand: XCDs streaming at different rates drift apart over a launch
    which = np.digitize(st, edges[1:-1])
    bidx = np.arange(len(st))
    spread = [float(np.subtract(*np.percentile(bidx[which == k], [95, 5])) * tile_bytes / 2**20)
              if (which == k).sum() > 8 else 0.0 for k in range(10)]
    return {"cset": cset, "per_xcd": per_xcd, "deciles": deciles, "spread": spread, "stamped": stamped, "span": span, "outside": stamped - span,
            "resident": int(first_round.sum()), "dispatch": ent[first_round].max(),
            "first_load": ld[first_blk] - ent[first_blk],
            "load_med": float(np.median(ld - ent)), "store_med": float(np.median(st - ld)),
            "steady_gbs": 1.0 / k / 1e3, "head": a, "tail": span - (a + k * total),
            "xcd_end": max(xcd_last) - min(xcd_last), "n_xcc": len(xcd_last)}


STREAMS = "--streams" in sys.argv  # the 1024x1 reduce beside a loads-only and a stores-only build
if STREAMS:
    sys.argv.remove("--streams")
    SHAPES = {1: "1024x1", 4: "1024x1 loads only", 5: "1024x1 stores only"}
if "--swap-only" in sys.argv:        # only the parity-swapped shapes (and 512x2 for reference)
    sys.argv.remove("--swap-only")
    SHAPES = {0: "512x2", 2: "512x2 swapped", 3: "1024x1 swapped"}
PRE_ODD = "--pre-odd" in sys.argv    # a 3-block pgk_reduce launch before each stamped one: does dealing continue?
if PRE_ODD:
    sys.argv.remove("--pre-odd")
sizes = [int(a) << 20 for a in sys.argv[1:]] or [m << 20 for m in (16, 64, 256)]
k = 0
for size in sizes:
    n = size // 8
    pairs = POOL // (2 * size)
    for shape, sname in SHAPES.items():
        grid = lab.tl_grid(shape, n)
        ts_dev = torch.zeros(4 * grid, dtype=torch.int64, device="cuda")
        rows, shipped = [], []
        for rep in range(REPS + 1):
            d = base + 2 * size * (k % pairs)
            k += 1
            if PRE_ODD:
                pgamd.check(lib.pgk_reduce(base, base + (8 << 20), 3 * 2048, 1, 0, sh), "pre")
            assert lab.tl_launch(shape, d, d + size, n, ts_dev.data_ptr(), sh, ev[0], ev[1]) == 0
            torch.cuda.synchronize()
            st_us = elapsed_us()
            ts = ts_dev.view(grid, 4).cpu().numpy()
            d = base + 2 * size * (k % pairs)
            k += 1
            pgamd.check(lib.pgk_reduce_timed(d, d + size, n, 1, 0, sh, ev[0], ev[1]), "shipped")
            torch.cuda.synchronize()
            if rep:                                   # the first of each is a warm-up
                rows.append(analyse(ts, 1024 * 16, st_us, {4: 2.0, 5: 1.0}.get(shape, 3.0)))
                shipped.append(elapsed_us())
        per = [r.pop("per_xcd") for r in rows]
        csets = [r.pop("cset") for r in rows]
        dec = np.median(np.array([r.pop("deciles") for r in rows]), axis=0)
        spr = np.median(np.array([r.pop("spread") for r in rows]), axis=0)
        med = {key: statistics.median(r[key] for r in rows) for key in rows[0]}
        print(f"== {size >> 20} MiB per operand, {sname} tiles, {grid} blocks (medians of {REPS} launches, us) ==")
        print(f"  shipped pgk_reduce stamped {statistics.median(shipped):8.2f}   diagnostic build stamped "
              f"{med['stamped']:8.2f}")
        print(f"  span {med['span']:8.2f}  outside {med['outside']:6.2f}  | resident first round {med['resident']:.0f} "
              f"blocks, dispatched over {med['dispatch']:5.2f}")
        print(f"  first block loads {med['first_load']:5.2f}  median block: loads {med['load_med']:5.2f}, "
              f"stores acked {med['store_med']:5.2f}")
        print(f"  steady {med['steady_gbs']:7.1f} GB/s  head {med['head']:5.2f}  tail {med['tail']:5.2f}  "
              f"XCD last-completion spread {med['xcd_end']:5.2f} over {med['n_xcc']:.0f} XCDs", flush=True)
        # per XCD (HW_REG_XCC_ID): blocks, how long before the launch's last completion it finished
        # (median over launches; and in each launch), and its own rate over its span
        print("  GB/s by tenth of the span: " + " ".join(f"{v:6.0f}" for v in dec))
        print("  MiB apart (5-95%) of the tiles finishing in each tenth: " + " ".join(f"{v:6.1f}" for v in spr))
        print(f"  dealing: c in xcc = (b + c) mod 8, per launch: {csets}")
        ids = sorted(set().union(*[set(p) for p in per]))
        print("  per XCD: id blocks | finished early by (median; each launch) | GB/s over its own span")
        for x in ids:
            early = [p[x][1] for p in per if x in p]
            rate = [p[x][2] for p in per if x in p]
            print(f"    {x}  {per[0].get(x, (0,))[0]:6d} | {statistics.median(early):5.2f}; "
                  + " ".join(f"{e:4.1f}" for e in early) + f" | {statistics.median(rate):7.1f}")
        del ts_dev
