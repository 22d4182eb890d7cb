#!/usr/bin/env python3
"""EXPERIMENTS ONLY: one block of `len` elements folded from W = 8 local
sources over R = 2 ring parts, two ways (the choice fold_block makes in the
xgmi transport, XG_FOLD_ONE_LAUNCH_MAX):
  parts  one pgk_reduce_multi launch per ring part (16-B vector kernel)
  one    one pgk_fold_blocks launch for all parts (element-wise kernel)
Each way: 200 back-to-back calls on one stream bracketed by events, then a
host wait (what a small xgmi call pays once).

    python tools/lab/fold_launch_probe.py
"""
import ctypes
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]

import torch  # noqa: E402

import pgamd  # noqa: E402


def main():
    lib = pgamd.load()
    W, R = 8, 2
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    for nbytes in (4 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20):
        n = nbytes // 8
        srcs = [torch.rand(n, dtype=torch.float64, device="cuda") for _ in range(W)]
        out1 = torch.empty(n, dtype=torch.float64, device="cuda")
        out2 = torch.empty(n, dtype=torch.float64, device="cuda")
        sp = (ctypes.c_void_p * W)(*[x.data_ptr() for x in srcs])
        parts = []
        for g in range(R):
            po, pl = pgamd.block_part(n, R, g)
            d = pgamd.ring_offset(W, R, g)
            order = [srcs[((j + 1) * d) % W] for j in range(W)]
            parts.append((po, pl, (ctypes.c_void_p * W)(*[x.data_ptr() + po * 8 for x in order])))

        def by_parts():
            for po, pl, ps in parts:
                assert lib.pgk_reduce_multi(out1.data_ptr() + po * 8, ps, W, pl, 1, 0, sh) == 0

        def one():
            assert lib.pgk_fold_blocks(out2.data_ptr(), sp, W, n, n, R, 1, 0, sh) == 0

        res = {}
        for name, fn in (("parts", by_parts), ("one", one)):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(200):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            dev_us = e0.elapsed_time(e1) / 200 * 1e3
            t = time.perf_counter()
            for _ in range(50):
                fn()
                torch.cuda.synchronize()
            host_us = (time.perf_counter() - t) / 50 * 1e6
            res[name] = (dev_us, host_us)
        same = torch.equal(out1.view(torch.int64), out2.view(torch.int64))
        print(f"{nbytes >> 10:6d} KiB  parts: {res['parts'][0]:7.1f} us device, {res['parts'][1]:7.1f} us call+wait"
              f"   one: {res['one'][0]:7.1f} us device, {res['one'][1]:7.1f} us call+wait   same_bits={same}",
              flush=True)
        del srcs, out1, out2


if __name__ == "__main__":
    main()
