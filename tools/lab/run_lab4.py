#!/usr/bin/env python3
"""EXPERIMENTS ONLY: time tools/lab/reduce_lab4.hip variants against the shipped
pgk_reduce (f64 sum), interleaved rounds in one process, HBM-resident chunks."""
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

so = HERE / "libreducelab4.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    str(HERE / "reduce_lab4.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
lab.lab2_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
lab.lab2_name.restype = ctypes.c_char_p
lib = pgamd.load()
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
sh = stream.cuda_stream
POOL = 2 << 30
pd = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
ps = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
variants = [-1]
for v in range(64):                      # keep the variants that launch (LDS reservations may exceed the limit)
    if lab.lab2_name(v):
        rc = lab.lab2_launch(v, pd.data_ptr(), ps.data_ptr(), 1 << 24, sh)
        torch.cuda.synchronize()
        if rc == 0:
            variants.append(v)
        else:
            print(f"skip {lab.lab2_name(v).decode()}: launch rc {rc}", flush=True)
for size in tuple(int(a) << 20 for a in sys.argv[1:]) or (1 << 28, 1 << 30):
    n = size // 8
    nch = POOL // size
    times = {v: [] for v in variants}
    k = 0
    for rnd in range(5):
        for v in variants:
            evs = []
            for i in range(12):
                c = (k % nch) * n
                k += 1
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                dp, sp = pd.data_ptr() + c * 8, ps.data_ptr() + c * 8
                rc = lib.pgk_reduce(dp, sp, n, 1, 0, sh) if v < 0 else lab.lab2_launch(v, dp, sp, n, sh)
                assert rc == 0, (v, rc)
                b.record(stream)
                if i >= 2:
                    evs.append((a, b))
            torch.cuda.synchronize()
            times[v] += [a.elapsed_time(b) * 1e3 for a, b in evs]
    res = []
    for v in variants:
        med = statistics.median(times[v])
        name = "pgk_reduce (shipped)" if v < 0 else lab.lab2_name(v).decode()
        res.append((3 * size / med / 1e3, med, min(times[v]), name))
    print(f"== {size >> 20} MiB per operand, f64 sum ==")
    for gbs, med, mn, name in sorted(res, reverse=True):
        print(f"{gbs:8.1f} GB/s  median {med:8.2f} us  min {mn:8.2f} us  {name}")
