#!/usr/bin/env python3
"""EXPERIMENTS ONLY: tools/lab/reduce_lab3.hip (8-source fold shapes) against the
shipped pgk_reduce_multi, interleaved rounds, local sources, HBM traffic 9 x size.
    python tools/lab/run_lab3.py [MiB per source ...]"""
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

so = HERE / "libreducelab3.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    str(HERE / "reduce_lab3.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
lab.lab3_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
lab.lab3_name.restype = ctypes.c_char_p
lib = pgamd.load()
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
sh = stream.cuda_stream
variants = [-1] + [v for v in range(64) if lab.lab3_name(v)]
for size in tuple(int(a) << 20 for a in sys.argv[1:]) or (128 << 20, 512 << 20):
    n = size // 8
    pool = torch.empty(18 * n, dtype=torch.float64, device="cuda").uniform_(-1, 1)    # two sets of 8 srcs + out
    times = {v: [] for v in variants}
    k = 0
    for rnd in range(8):
        for v in variants:
            # consecutive launches alternate between the two sets, so no launch
            # finds its sources in the Infinity Cache after the previous variant
            base = pool.data_ptr() + (k % 2) * 9 * size
            k += 1
            srcs = (ctypes.c_void_p * 8)(*[base + j * size for j in range(8)])
            out = base + 8 * size
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            rc = lib.pgk_reduce_multi(out, srcs, 8, n, 1, 0, sh) if v < 0 else lab.lab3_launch(v, out, srcs, n, sh)
            assert rc == 0, (v, rc)
            b.record(stream)
            torch.cuda.synchronize()
            if rnd >= 2:
                times[v].append(a.elapsed_time(b) * 1e3)
    print(f"== {size >> 20} MiB per source, 8 sources, f64 sum ==")
    res = sorted(((9 * size / statistics.median(t) / 1e3, statistics.median(t),
                   "pgk_reduce_multi (shipped)" if v < 0 else lab.lab3_name(v).decode()) for v, t in times.items()),
                 reverse=True)
    for gbs, med, name in res:
        print(f"{gbs:8.1f} GB/s  median {med:8.2f} us  {name}", flush=True)
    del pool
    torch.cuda.empty_cache()
