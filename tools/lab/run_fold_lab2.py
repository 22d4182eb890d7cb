#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the 8-source fold with its sources in separate regions
(as shipped) against the same sources interleaved by granule inside one region
(tools/lab/fold_lab2.hip).  Kernel-stamped, rotating over a 4 GiB pool, double
sum; GB/s counts 9 x bytes per source (8 reads + 1 write; reads-only rows 8 x).

    python tools/lab/run_fold_lab2.py [MiB per source ...]     (default 16 64)
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

so = HERE / "libfoldlab2.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
                    str(HERE / "fold_lab2.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
VP = ctypes.c_void_p
lab.fold2_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, VP, VP, ctypes.POINTER(VP), ctypes.c_size_t,
                             ctypes.c_int, VP, VP, VP]
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")

GRAN = [16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20]
# (label, kind, block, unroll, granule bytes or 0)
VARIANTS = [("shipped pgk_reduce_multi (8 separate regions)", -1, 0, 0, 0),
            ("separate 512x1", 0, 512, 1, 0), ("separate 256x2", 0, 256, 2, 0), ("separate 1024x1", 0, 1024, 1, 0),
            ("separate 512x1, reads only", 1, 512, 1, 0)]
for g in GRAN:
    VARIANTS.append((f"8 interleaved @ {g >> 10} KiB, 512x1", 2, 512, 1, g))
for g in (64 << 10, 1 << 20):
    VARIANTS.append((f"8 interleaved @ {g >> 10} KiB, 1024x1", 2, 1024, 1, g))
    VARIANTS.append((f"7 interleaved @ {g >> 10} KiB + own block separate, 512x1", 3, 512, 1, g))


def launch(var, b0, size, e0, e1):
    _, kind, blk, unr, gran = var
    n = size // 8
    srcs = (VP * 8)(*[b0 + size * j for j in range(8)])
    out = b0 + 8 * size
    if kind < 0:
        return lib.pgk_reduce_multi_timed(out, srcs, 8, n, 1, 0, sh, e0, e1)
    lg = (gran // 16).bit_length() - 1 if gran else 0
    return lab.fold2_launch(kind, blk, unr, out, b0, srcs, n, lg, sh, e0, e1)


# correctness of the interleaved addressing, once, at 4 MiB per source
size = 4 << 20
for var in VARIANTS:
    _, kind, _, _, gran = var
    if kind not in (2, 3):
        continue
    assert launch(var, base, size, None, None) == 0
    torch.cuda.synchronize()
    n = size // 8
    ni = 8 if kind == 2 else 7
    il = pool[:ni * n].view(-1, ni, gran // 8)
    acc = il[:, 0].reshape(-1).clone()
    for j in range(1, ni):
        acc += il[:, j].reshape(-1)
    if ni == 7:
        acc += pool[7 * n:8 * n]
    assert torch.equal(acc, pool[8 * n:9 * n]), var
print("interleaved addressing checked against torch", flush=True)

for mib in [int(a) for a in sys.argv[1:]] or [16, 64]:
    size = mib << 20
    sets = POOL // (9 * size)
    times = {v[0]: [] for v in VARIANTS}
    k = 0
    for rnd in range(4):
        for var in VARIANTS:
            for i in range(6):
                b0 = base + 9 * size * (k % sets)
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
        traffic = (8 if var[1] == 1 else 9) * size
        print(f"  {m:9.2f} {min(times[var[0]]):9.2f}  {traffic / m / 1e3:8.1f} GB/s {traffic / m / 8e4:5.1f}%  {var[0]}",
              flush=True)
