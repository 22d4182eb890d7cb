#!/usr/bin/env python3
"""Sweep the gfx950 reduce kernel's launch knobs over chunk sizes (GPU box).

    python tools/sweep_kernel.py [--out gpurun_out/sweep_kernel.csv] [--quick]

Interleaved rounds in one process (guide §5.4 rule 24): every variant is timed
in each round, per-launch HIP events on the launch stream, median reported.
Chunks rotate through a 2 GiB pool per operand, so chunks >= 64 MiB come from
HBM, not the 256 MiB Infinity Cache.  CSV columns extend the reference's
measurement schema (README.md:85: size, rounds, inflight, time_us, GB/s).
"""
import argparse
import ctypes
import itertools
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]

import torch  # noqa: E402

import pgamd  # noqa: E402

POOL = 2 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/sweep_kernel.csv")
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sizes", default="", help="comma-separated byte sizes (default: 4 KiB .. 1 GiB)")
    ap.add_argument("--ab", action="store_true", help="only the one-shot nt shapes (A/B of block shape)")
    args = ap.parse_args()
    lib = pgamd.load()
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    pool_d = torch.empty(POOL, dtype=torch.uint8, device="cuda")
    pool_s = torch.empty(POOL, dtype=torch.uint8, device="cuda")
    EV = []
    for _ in range(args.reps + 2):
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        lib.pgk_event_create(ctypes.byref(a))
        lib.pgk_event_create(ctypes.byref(b))
        EV.append((a, b))
    pool_d.view(torch.float64).uniform_(-1, 1)
    pool_s.view(torch.float64).uniform_(-1, 1)
    sizes = [1 << 12, 1 << 16, 1 << 20, 1 << 24, 1 << 26, 1 << 28, 1 << 30]
    bpcs = [0, 2, 4, 8, 16]
    nts = [0, 1]
    shapes = [(256, 2), (256, 4), (256, 8), (512, 2), (1024, 1)]
    if args.quick:
        sizes = [1 << 20, 1 << 26, 1 << 28]
        bpcs = [0, 8]
        shapes = [(256, 4), (512, 2)]
    if args.sizes:
        sizes = [int(x) for x in args.sizes.split(",")]
    if args.ab:
        bpcs, nts = [0], [1]
    variants = [(b, nt, sh_) for b in bpcs for nt in nts for sh_ in shapes]
    rows = []
    out = pathlib.Path(args.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    with out.open("w") as f:
        f.write("size,rounds,inflight,time_us,GB/s,dtype,op,blocks_per_cu,nt,shape,min_us,grid\n")
        for size, (dt, op) in itertools.product(sizes, [(1, 0), (0, 0), (1, 1), (0, 1)]):
            if (dt, op) != (1, 0) and size not in (1 << 20, 1 << 28):
                continue
            es = 8 if dt == 1 else 4
            n = size // es
            nchunks = max(1, min(64, POOL // size))
            times = {v: [] for v in variants}
            k = 0
            for rnd in range(args.rounds):
                for v in variants:
                    lib.pgk_tune(v[0], v[1])
                    pgamd.check(lib.pgk_tune_shape(*v[2]), "tune")
                    evs = []
                    for i in range(args.reps + 2):
                        c = (k % nchunks) * size
                        k += 1
                        a, b = EV[i]
                        pgamd.check(lib.pgk_reduce_timed(pool_d.data_ptr() + c, pool_s.data_ptr() + c, n, dt, op, sh,
                                                         a, b), "reduce")
                        if i >= 2:
                            evs.append((a, b))
                    torch.cuda.synchronize()
                    for a, b in evs:
                        ms = ctypes.c_float()
                        lib.pgk_event_elapsed_ms(a, b, ctypes.byref(ms))
                        times[v].append(ms.value * 1e3)
            for v in variants:
                med = statistics.median(times[v])
                lib.pgk_tune(v[0], v[1])
                lib.pgk_tune_shape(*v[2])
                g = ctypes.c_uint()
                lib.pgk_launch_geometry(n, dt, ctypes.byref(g), None)
                gbs = 3 * size / (med * 1e-6) / 1e9
                row = (size, 1, 0, round(med, 3), round(gbs, 1), "f64" if dt else "i32", "sum" if op == 0 else "prod",
                       v[0], v[1], f"{v[2][0]}x{v[2][1]}", round(min(times[v]), 3), g.value)
                rows.append(row)
                f.write(",".join(map(str, row)) + "\n")
            f.flush()
            best = max((r for r in rows if r[0] == size and r[5] == ("f64" if dt else "i32") and r[6] == ("sum" if op == 0 else "prod")),
                       key=lambda r: r[4])
            print(f"size={size:>11} {best[5]} {best[6]}: best {best[4]:8.1f} GB/s "
                  f"(bpc={best[7]} nt={best[8]} shape={best[9]}, {best[3]} us)", flush=True)
    lib.pgk_tune(0, 1)
    lib.pgk_tune_shape(0, 0)


if __name__ == "__main__":
    main()
