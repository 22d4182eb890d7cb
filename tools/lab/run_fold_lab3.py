#!/usr/bin/env python3
"""EXPERIMENTS ONLY: store-side and turnover variants of the 8-source fold
(tools/lab/fold_lab3.hip), and the same shipped-shape kernel with its nine
regions skewed against each other (region j starts j * skew bytes later than a
power-of-two spacing would put it).  Kernel-stamped, rotating over a 4 GiB
pool, double sum; GB/s counts 9 x bytes per source.

    python tools/lab/run_fold_lab3.py [MiB per source ...]     (default 16 64)
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

so = HERE / "libfoldlab3.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
                    str(HERE / "fold_lab3.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
VP = ctypes.c_void_p
lab.fold3_launch.argtypes = [ctypes.c_int] * 4 + [VP, ctypes.POINTER(VP), ctypes.c_size_t, VP, VP, VP]
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")

# (label, kind, block, unroll, blocks per CU, skew bytes)
VARIANTS = [("shipped pgk_reduce_multi", -1, 0, 0, 0, 0),
            ("512x1 nt/nt (shipped shape)", 0, 512, 1, 0, 0),
            ("512x1 nt loads, plain store", 1, 512, 1, 0, 0),
            ("512x1 plain loads, nt store", 2, 512, 1, 0, 0),
            ("512x1 store after a block barrier", 4, 512, 1, 0, 0),
            ("64x1", 0, 64, 1, 0, 0), ("64x4", 0, 64, 4, 0, 0), ("128x1", 0, 128, 1, 0, 0),
            ("256x4", 0, 256, 4, 0, 0),
            ("resident 256 thr x 8/CU, next tile prefetched", 3, 256, 1, 8, 0),
            ("resident 512 thr x 4/CU, next tile prefetched", 3, 512, 1, 4, 0),
            ("resident 512 thr x 2/CU, next tile prefetched", 3, 512, 1, 2, 0)]
for skew in (256, 4096 + 256, 65536 + 4096 + 256, (2 << 20) + 8192 + 256, 1 << 20):
    VARIANTS.append((f"512x1 nt/nt, regions skewed by {skew} B", 0, 512, 1, 0, skew))


def launch(var, b0, size, e0, e1):
    _, kind, blk, unr, bpc, skew = var
    n = size // 8
    srcs = (VP * 8)(*[b0 + (size + skew) * j for j in range(8)])
    out = b0 + 8 * (size + skew)
    if kind < 0:
        return lib.pgk_reduce_multi_timed(out, srcs, 8, n, 1, 0, sh, e0, e1)
    return lab.fold3_launch(kind, blk, unr, bpc, out, srcs, n, sh, e0, e1)


# every variant computes the same sum (checked once at 4 MiB per source)
size = 4 << 20
n = size // 8
for var in VARIANTS:
    skew = var[5]
    assert launch(var, base, size, None, None) == 0, var
    torch.cuda.synchronize()
    st = (size + skew) // 8
    acc = pool[:n].clone()
    for j in range(1, 8):
        acc += pool[j * st:j * st + n]
    assert torch.equal(acc, pool[8 * st:8 * st + n]), var
print("every variant checked against torch", flush=True)

for mib in [int(a) for a in sys.argv[1:]] or [16, 64]:
    size = mib << 20
    times = {v[0]: [] for v in VARIANTS}
    k = 0
    for rnd in range(4):
        for var in VARIANTS:
            span = 9 * (size + var[5])
            sets = POOL // span
            for i in range(6):
                b0 = base + span * (k % sets)
                k += 1
                rc = launch(var, b0, size, ev[0], ev[1])
                assert rc == 0, (var, rc)
                torch.cuda.synchronize()
                ms = ctypes.c_float()
                pgamd.check(lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)), "elapsed")
                if i:
                    times[var[0]].append(ms.value * 1e3)
    print(f"== 8 sources x {mib} MiB (kernel-stamped us: median / min; GB/s and share of 8000) ==", flush=True)
    for var in VARIANTS:
        m = statistics.median(times[var[0]])
        print(f"  {m:9.2f} {min(times[var[0]]):9.2f}  {9 * size / m / 1e3:8.1f} GB/s {9 * size / m / 8e4:5.1f}%  {var[0]}",
              flush=True)
