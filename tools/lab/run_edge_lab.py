#!/usr/bin/env python3
"""EXPERIMENTS ONLY: per-launch edge cost of the reduce (tools/lab/edge_lab.hip).

Every launch is kernel-stamped (hipExtLaunchKernelGGL start/stop events, the
figure rocprofv3 reports) and rotates over a 4 GiB pool of dst/src pairs, so
it streams from HBM.  For each variant a least-squares fit over the operand
sizes, t = t0 + traffic / bw, splits the launch into a fixed edge t0 and a
streaming rate bw (traffic: reduce/copy 3 or 2 bytes per operand byte, read 2,
write 1).  The shipped pgk_reduce is timed the same way beside them.

    python tools/lab/run_edge_lab.py [--lab edge|policy|wait|dyn] [--only TEXT] [--b2b] [--reduce-only] [sizes in MiB ...]
                                                            (default 8 16 32 64 128 256)
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

LAB = "edge"                    # --lab policy: tools/lab/policy_lab.hip (store cache policies), same API
if "--lab" in sys.argv:
    i = sys.argv.index("--lab")
    LAB = sys.argv[i + 1]
    del sys.argv[i:i + 2]
so = HERE / f"lib{LAB}lab.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    str(HERE / f"{LAB}_lab.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
lab.edge_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                            ctypes.c_void_p, ctypes.c_void_p]
lab.edge_name.restype = ctypes.c_char_p
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (ctypes.c_void_p(), ctypes.c_void_p())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
TRAFFIC = {0: 0, 1: 2, 2: 1, 3: 2, 4: 3}
KIND = {"empty": 0, "read": 1, "write": 2, "copy": 3, "reduce": 4}
variants = [-1] + [v for v in range(32) if lab.edge_name(v)]
B2B = "--b2b" in sys.argv       # events bracketing back-to-back launches (the bench's kernel_us) instead of stamps
if B2B:
    sys.argv.remove("--b2b")
if "--only" in sys.argv:                       # variants whose name contains this text (and the shipped kernel)
    i = sys.argv.index("--only")
    only = sys.argv[i + 1]
    del sys.argv[i:i + 2]
    variants = [v for v in variants if v < 0 or only in lab.edge_name(v).decode()]
if "--reduce-only" in sys.argv:
    sys.argv.remove("--reduce-only")
    variants = [v for v in variants if v < 0 or lab.edge_name(v).decode().startswith("reduce")]


def name(v):
    return "pgk_reduce (shipped)" if v < 0 else lab.edge_name(v).decode()


def kind(v):
    return 4 if v < 0 else KIND[name(v).split()[0]]


sizes = [int(a) << 20 for a in sys.argv[1:]] or [m << 20 for m in (8, 16, 32, 64, 128, 256)]
med = {}
k = 0
for size in sizes:
    n = size // 8
    pairs = POOL // (2 * size)
    times = {v: [] for v in variants}
    for rnd in range(4):
        for v in variants:
            if B2B:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for i in range(13):
                    if i == 1:
                        e0.record()
                    d = base + 2 * size * (k % pairs)
                    k += 1
                    rc = (lib.pgk_reduce(d, d + size, n, 1, 0, sh) if v < 0
                          else lab.edge_launch(v, d, d + size, n, sh, None, None))
                    assert rc == 0, (v, rc)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) * 1e3 / 12)
                continue
            for i in range(6):
                d = base + 2 * size * (k % pairs)
                k += 1
                rc = (lib.pgk_reduce_timed(d, d + size, n, 1, 0, sh, ev[0], ev[1]) if v < 0
                      else lab.edge_launch(v, d, d + size, n, sh, ev[0], ev[1]))
                assert rc == 0, (v, rc)
                torch.cuda.synchronize()
                ms = ctypes.c_float()
                pgamd.check(lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)), "elapsed")
                if i >= 1:
                    times[v].append(ms.value * 1e3)
    print(f"== {size >> 20} MiB per operand ({'back-to-back, events / launch' if B2B else 'kernel-stamped'} us: "
          "median / min) ==", flush=True)
    for v in variants:
        m = statistics.median(times[v])
        med[(v, size)] = m
        tr = TRAFFIC[kind(v)] * size
        rate = f"{tr / m / 1e3:8.1f} GB/s" if tr else " " * 13
        print(f"  {m:9.2f} {min(times[v]):9.2f}  {rate}  {name(v)}", flush=True)

print("== fit t = t0 + traffic/bw over the sizes ==")
for v in variants:
    tr = TRAFFIC[kind(v)]
    if not tr:
        print(f"  t0 {statistics.median([med[(v, s)] for s in sizes]):6.2f} us (no traffic)        {name(v)}")
        continue
    x = np.array([tr * s for s in sizes], dtype=np.float64)
    y = np.array([med[(v, s)] for s in sizes])
    A = np.vstack([np.ones_like(x), x]).T
    t0, inv = np.linalg.lstsq(A, y, rcond=None)[0]
    bw = 1.0 / inv / 1e3 if inv > 0 else float("nan")
    at64 = 3 * (64 << 20) / med.get((v, 64 << 20), float("nan")) / 1e3 if kind(v) == 4 else float("nan")
    print(f"  t0 {t0:6.2f} us  bw {bw:7.1f} GB/s  (64 MiB: {at64:7.1f} GB/s)  {name(v)}")
