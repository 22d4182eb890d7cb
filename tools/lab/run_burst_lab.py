#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the 8-source fold with its stores gathered into bursts
(tools/lab/burst_lab.hip) against the shipped pgk_reduce_multi.  Kernel-stamped,
rotating over a 4 GiB pool, double sum; GB/s counts 9 x bytes per source.

    python tools/lab/run_burst_lab.py [MiB per source ...]     (default 64 256)
"""
import ctypes
import pathlib
import statistics
import subprocess
import sys

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

so = HERE / "libburstlab.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
                    str(HERE / "burst_lab.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
VP = ctypes.c_void_p
lab.burst_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_int,
                             VP, ctypes.POINTER(VP), ctypes.c_size_t, VP, VP, VP]
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")

# (label, unroll U, block, blocks per CU, period ticks (10 ns each; 0 = no gate), read ticks)
VARIANTS = [("shipped pgk_reduce_multi", 0, 0, 0, 0, 0)]
for u, b, bpc in ((4, 256, 8), (8, 256, 6), (8, 256, 4), (16, 256, 4), (16, 256, 2), (32, 256, 2), (8, 512, 3),
                  (16, 512, 2)):
    VARIANTS.append((f"burst U={u:2d} {b}x{bpc}/CU ({256 * bpc * b * u * 16 >> 20} MiB of results per burst)", u, b, bpc, 0, 0))
MAX_SPINS = 2000                     # x (s_sleep 16 ~ 1024 cycles) ~ 1 ms at most, then the wave stores anyway


def launch(var, b0, size, e0, e1):
    _, u, blk, bpc, period, rd = var
    n = size // 8
    srcs = (VP * 8)(*[b0 + size * j for j in range(8)])
    out = b0 + 8 * size
    if u == 0:
        return lib.pgk_reduce_multi_timed(out, srcs, 8, n, 1, 0, sh, e0, e1)
    return lab.burst_launch(u, blk, bpc, period, rd, MAX_SPINS, out, srcs, n, sh, e0, e1)


def check(var, size):
    n = size // 8
    pool[8 * n:9 * n].fill_(-7.0)
    assert launch(var, base, size, None, None) == 0, var
    torch.cuda.synchronize()
    acc = pool[:n].clone()
    for j in range(1, 8):
        acc += pool[j * n:(j + 1) * n]
    assert torch.equal(acc, pool[8 * n:9 * n]), var


for var in VARIANTS:
    for size in (4 << 20, (4 << 20) + 4096 + 16, 1 << 16):     # whole, ragged and tiny
        check(var, size)
print("every variant checked against torch", flush=True)


def measure(variants, size):
    times = {v[0]: [] for v in variants}
    k = 0
    sets = POOL // (9 * size)
    for rnd in range(4):
        for var in variants:
            for i in range(6):
                b0 = base + 9 * size * (k % sets)
                k += 1
                assert launch(var, b0, size, ev[0], ev[1]) == 0, var
                torch.cuda.synchronize()
                ms = ctypes.c_float()
                pgamd.check(lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)), "elapsed")
                if i:
                    times[var[0]].append(ms.value * 1e3)
    return {k: (statistics.median(v), min(v)) for k, v in times.items()}


for mib in [int(a) for a in sys.argv[1:]] or [64, 256]:
    size = mib << 20
    res = measure(VARIANTS, size)
    print(f"== 8 sources x {mib} MiB (kernel-stamped us: median / min; share of 8000 GB/s) ==", flush=True)
    for var in VARIANTS:
        m, lo = res[var[0]]
        print(f"  {m:9.2f} {lo:9.2f}  {9 * size / m / 8e4:5.1f}%  {var[0]}", flush=True)
    # the best ungated variant again, its bursts re-aligned to the clock: the period is what one of its
    # read-then-write rounds took ungated, the write window its last 15% / 25%
    best = min((v for v in VARIANTS if v[1]), key=lambda v: res[v[0]][0])
    _, u, blk, bpc, _, _ = best
    rounds = max(1, -(-(size // 16) // (256 * bpc * blk * u)))
    per_round_ticks = int(res[best[0]][0] * 100 / rounds)
    gated = []
    for scale in (0.9, 1.0, 1.1):
        for wr in (0.15, 0.25):
            period = max(200, int(per_round_ticks * scale))
            gated.append((f"  gated: period {period / 100:.1f} us x{scale}, writes in the last {int(wr * 100)}%", u, blk, bpc,
                          period, int(period * (1 - wr))))
    for var in gated:
        check(var, 4 << 20)
    res2 = measure(gated, size)
    print(f"  best ungated: {best[0]} ({rounds} rounds per launch); the same with the gate:", flush=True)
    for var in gated:
        m, lo = res2[var[0]]
        print(f"  {m:9.2f} {lo:9.2f}  {9 * size / m / 8e4:5.1f}%  {var[0]}", flush=True)
