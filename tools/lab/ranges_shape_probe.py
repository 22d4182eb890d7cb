#!/usr/bin/env python3
"""EXPERIMENTS ONLY: which tile shape for the executor's multi-range launch
(pgk_reduce_ranges)?  The shipped rule picks the shape from the LARGEST range;
a launch of R ranges streams like one launch of their sum.  Forces each
instantiated shape with pgk_tune_shape and times R ranges of S MiB
(kernel-stamped and back-to-back), ranges in separate regions of a 4 GiB pool,
rotating.  double sum.

    python tools/lab/ranges_shape_probe.py
"""
import ctypes
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1e-3, 1e-3)
base = pool.data_ptr()
VP, SZ = ctypes.c_void_p, ctypes.c_size_t
ev = (VP(), VP())
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[0])), "event")
pgamd.check(lib.pgk_event_create(ctypes.byref(ev[1])), "event")
SHAPES = [(0, 0), (512, 2), (256, 4), (1024, 1), (256, 2), (256, 8)]
for rings, mib in ((2, 64), (2, 32), (4, 32), (2, 128), (2, 16), (1, 128)):
    rng = mib << 20
    stride = max(64 << 20, rng)
    slots = (POOL // (2 * stride)) // rings
    print(f"== {rings} ranges x {mib} MiB per operand (stamped us median / back-to-back us; share of 8000 GB/s) ==", flush=True)
    res = {s: ([], []) for s in SHAPES}
    k = 0
    for rnd in range(3):
        for shape in SHAPES:
            pgamd.check(lib.pgk_tune_shape(*shape), "shape")

            def launch(i, e=(None, None)):
                outs, bs, ns = (VP * rings)(), (VP * rings)(), (SZ * rings)()
                for g in range(rings):
                    d = base + 2 * stride * ((i % slots) * rings + g)
                    outs[g], bs[g], ns[g] = d, d + stride, rng // 8
                assert lib.pgk_reduce_ranges(outs, outs, bs, ns, rings, 1, 0, sh, e[0], e[1]) == 0

            for i in range(7):
                launch(k, ev)
                k += 1
                torch.cuda.synchronize()
                ms = ctypes.c_float()
                lib.pgk_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms))
                if i:
                    res[shape][0].append(ms.value * 1e3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            launch(k)
            e0.record()
            for i in range(20):
                launch(k + i)
            e1.record()
            k += 20
            torch.cuda.synchronize()
            res[shape][1].append(e0.elapsed_time(e1) * 1e3 / 20)
    pgamd.check(lib.pgk_tune_shape(0, 0), "shape")
    tr = 3 * rng * rings
    for shape in SHAPES:
        st, bb = statistics.median(res[shape][0]), statistics.median(res[shape][1])
        name = "by size (shipped rule)" if shape == (0, 0) else f"{shape[0]}x{shape[1]}"
        print(f"  {st:8.2f} {tr / st / 8e4:5.1f}%   {bb:8.2f} {tr / bb / 8e4:5.1f}%   {name}", flush=True)
