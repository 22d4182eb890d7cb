#!/usr/bin/env python3
"""EXPERIMENTS ONLY: the 8-source fold (tools/lab/fold_lab.hip) against the
shipped pgk_reduce_multi, kernel-stamped, sources rotating over a 4 GiB pool
(HBM-resident), double sum.  GB/s counts 9 x bytes per source (8 reads + 1
write).

    python tools/lab/run_fold_lab.py [MiB per source ...]     (default 4 16 64)
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

so = HERE / "libfoldlab.so"
if not so.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    str(HERE / "fold_lab.hip"), "-o", str(so)], check=True)
lab = ctypes.CDLL(str(so))
VP = ctypes.c_void_p
lab.fold_launch.argtypes = [ctypes.c_int, VP, ctypes.POINTER(VP), ctypes.c_size_t, VP, VP, VP]
lab.fold_name.restype = ctypes.c_char_p
lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
variants = [-1] + [v for v in range(32) if lab.fold_name(v)]
for mib in [int(a) for a in sys.argv[1:]] or [4, 16, 64]:
    size = mib << 20
    n = size // 8
    sets = POOL // (9 * size)
    times = {v: [] for v in variants}
    k = 0
    for rnd in range(4):
        for v in variants:
            for i in range(6):
                b0 = base + 9 * size * (k % sets)
                k += 1
                srcs = (VP * 8)(*[b0 + size * j for j in range(8)])
                out = b0 + 8 * size
                rc = (lib.pgk_reduce_multi_timed(out, srcs, 8, n, 1, 0, sh, ev[0], ev[1]) if v < 0
                      else lab.fold_launch(v, out, srcs, n, sh, ev[0], ev[1]))
                assert rc == 0, (v, rc)
                torch.cuda.synchronize()
                ms = ctypes.c_float()
                pgamd.check(lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)), "elapsed")
                if i:
                    times[v].append(ms.value * 1e3)
    print(f"== 8 sources x {mib} MiB (kernel-stamped us: median / min; GB/s of 9 x size) ==", flush=True)
    for v in variants:
        m = statistics.median(times[v])
        name = "pgk_reduce_multi (shipped)" if v < 0 else lab.fold_name(v).decode()
        print(f"  {m:9.2f} {min(times[v]):9.2f}  {9 * size / m / 1e3:8.1f} GB/s  {name}", flush=True)
