#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the streaming rate against the read:write mix
(tools/lab/mix_lab.hip).  R read streams of `size` bytes each, one output
stream to which every M-th group of eight tiles writes its sums, packed (M = 0: none).  Kernel-stamped,
rotating over a 4 GiB pool; GB/s counts the bytes the launch really moves,
R x size + size / M.  The rows where the mix equals the shipped kernels'
(R = 2, M = 1: the reduce; R = 8, M = 1: the fold) are marked.

    python tools/lab/run_mix_lab.py [MiB per stream ...]     (default 64)
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

so = HERE / "libmixlab.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
                    str(HERE / "mix_lab.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
VP = ctypes.c_void_p
lab.mix_launch.argtypes = [ctypes.c_int, ctypes.c_int, VP, ctypes.POINTER(VP), ctypes.c_size_t, VP, VP, VP]
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")

READS = (1, 2, 3, 4, 6, 8)
EVERY = (0, 8, 4, 2, 1)

# the sums are right where they are stored, and nothing else is touched (4 MiB per stream)
size = 4 << 20
n = size // 8
for r in READS:
    for m in EVERY:
        srcs = (VP * 8)(*[base + size * j for j in range(8)])
        out = pool[8 * n:9 * n]
        out.fill_(-7.0)
        assert lab.mix_launch(r, m, out.data_ptr(), srcs, n, sh, None, None) == 0
        torch.cuda.synchronize()
        want = pool[:n].clone()
        for j in range(1, r):
            want += pool[j * n:(j + 1) * n]
        tile = torch.arange(n, device="cuda") // (512 * 2)            # 512 lanes x 2 doubles per tile
        kept = want[(tile // 8) % m == 0] if m else want[:0]          # the stored groups of 8 tiles, packed
        assert torch.equal(out[:kept.numel()], kept) and bool((out[kept.numel():] == -7.0).all()), (r, m)
print("every variant checked against torch", flush=True)

for mib in [int(a) for a in sys.argv[1:]] or [64]:
    size = mib << 20
    n = size // 8
    times = {}
    k = 0
    for rnd in range(4):
        for r in READS:
            for m in EVERY:
                span = (r + 1) * size
                sets = POOL // span
                for i in range(6):
                    b0 = base + span * (k % sets)
                    k += 1
                    srcs = (VP * 8)(*[b0 + size * min(j, r - 1) for j in range(8)])
                    assert lab.mix_launch(r, m, b0 + r * size, srcs, n, sh, ev[0], ev[1]) == 0
                    torch.cuda.synchronize()
                    ms = ctypes.c_float()
                    pgamd.check(lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)), "elapsed")
                    if i:
                        times.setdefault((r, m), []).append(ms.value * 1e3)
    print(f"== {mib} MiB per stream: share of 8000 GB/s by bytes really moved (median kernel-stamped us) ==", flush=True)
    print("  reads \\ groups stored:" + "".join(f"{'none' if m == 0 else '1 in ' + str(m):>18}" for m in EVERY), flush=True)
    for r in READS:
        row = f"  {r} read stream{'s' if r > 1 else ' '}      "
        for m in EVERY:
            t = statistics.median(times[(r, m)])
            moved = r * size + (size // m if m else 0)
            mark = "*" if m == 1 and r in (2, 8) else " "
            row += f"{moved / t / 8e4:7.1f}%{mark}({t:7.1f})"
        print(row, flush=True)
    print("  (* = the mix of the shipped two-operand reduce, R = 2, and of the 8-source fold, R = 8)", flush=True)
