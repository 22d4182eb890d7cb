#!/usr/bin/env python3
"""EXPERIMENTS ONLY: does cutting one reduce call into two half-launches on two
streams (tools/lab/split2_lab.hip) hide the per-launch edge?  Events on the
caller's stream bracketing 20 back-to-back calls (the bench's kernel_us), the
shipped pgk_reduce, double sum, operand pairs rotating over a 4 GiB pool.

    python tools/lab/run_split2_lab.py [MiB per operand ...]    (default 32 64 128 256)
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

so = HERE / "libsplit2lab.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    str(HERE / "split2_lab.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
lab.split2_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_size_t,
                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
lib = pgamd.load()
fn = ctypes.cast(lib.pgk_reduce, ctypes.c_void_p)
torch.cuda.set_device(0)
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1e-3, 1e-3)
base = pool.data_ptr()
MODES = {0: "one launch (shipped)", 1: "two halves on two streams, fork/join per call",
         2: "two halves on one stream", 3: "whole calls alternating between two streams (not a drop-in)"}
for mib in [int(a) for a in sys.argv[1:]] or [32, 64, 128, 256]:
    size = mib << 20
    pairs = POOL // (2 * size)
    res = {m: [] for m in MODES}
    for rnd in range(7):
        for m in MODES:
            us = ctypes.c_float()
            rc = lab.split2_run(fn, base, 2 * size, pairs, size // 8, 20, 3, m, ctypes.byref(us))
            assert rc == 0, (m, rc, pgamd.last_error())
            if rnd:
                res[m].append(us.value)
    print(f"== {mib} MiB per operand (us per call, events around 20 back-to-back calls: median / min; share of 8000 GB/s) ==",
          flush=True)
    for m, label in MODES.items():
        med = statistics.median(res[m])
        print(f"  {med:9.2f} {min(res[m]):9.2f}  {3 * size / med / 8e4:5.1f}%  {label}", flush=True)
