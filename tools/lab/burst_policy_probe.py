#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the burst fold's dense run of stores under other cache
policies (tools/lab/burst_lab.hip, k_burst_pol: buffer stores with aux bits;
0 plain, 1 sc0, 2 nt, 16 sc1, 18 sc1 nt).  8 sources, one round per launch
(64 MiB at 32 tiles per wave, 32 MiB at 16).  Kernel-stamped, checked against
torch.

    python tools/lab/burst_policy_probe.py
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
lab.burst_policy_launch.argtypes = [ctypes.c_int, ctypes.c_int, VP, ctypes.POINTER(VP), ctypes.c_size_t, VP, VP, VP]
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
NAMES = {0: "plain", 1: "sc0", 2: "nt (shipped)", 16: "sc1", 18: "sc1 nt"}
for u, size, auxes in ((32, 64 << 20, (2, 0, 1, 16, 18)), (16, 32 << 20, (2, 0, 16))):
    n = size // 8
    for aux in auxes:                                   # correctness first, ragged
        m = n // 16 + 6
        srcs = (VP * 8)(*[base + size * j for j in range(8)])
        pool[8 * n:9 * n].fill_(-7.0)
        assert lab.burst_policy_launch(u, aux, base + 8 * size, srcs, m, sh, None, None) == 0
        torch.cuda.synchronize()
        acc = pool[:m].clone()
        for j in range(1, 8):
            acc += pool[j * n:j * n + m]
        assert torch.equal(acc, pool[8 * n:8 * n + m]) and bool((pool[8 * n + m:9 * n] == -7.0).all()), (u, aux)
    sets = POOL // (9 * size)
    res = {}
    k = 0
    for rnd in range(4):
        for aux in auxes:
            for i in range(6):
                b0 = base + 9 * size * (k % sets)
                k += 1
                srcs = (VP * 8)(*[b0 + size * j for j in range(8)])
                assert lab.burst_policy_launch(u, aux, b0 + 8 * size, srcs, n, sh, ev[0], ev[1]) == 0
                torch.cuda.synchronize()
                ms = ctypes.c_float()
                lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms))
                if i:
                    res.setdefault(aux, []).append(ms.value * 1e3)
    print(f"== 8 x {size >> 20} MiB, {u} tiles per wave (kernel-stamped us median / min; share of 8000 GB/s) ==", flush=True)
    for aux in auxes:
        m = statistics.median(res[aux])
        print(f"  {m:8.2f} {min(res[aux]):8.2f}  {9 * size / m / 8e4:5.1f}%  stores {NAMES[aux]}", flush=True)
