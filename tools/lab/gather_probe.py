#!/usr/bin/env python3
"""EXPERIMENTS ONLY: pgk_gather (the all-gather / all-reduce copy kernel of the
xgmi transport and the link probe) as a local HBM copy on one GPU, against
hipMemcpy device-to-device and the reduce kernel's rate.

k sources of `size` bytes each are copied into one buffer of k*size bytes,
launches rotating over 4 such sets so the 256 MB Infinity Cache does not serve
them.  GB/s counts 2 bytes (read + write) per byte copied.

    python tools/lab/gather_probe.py [size_MiB ...]
"""
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]

import torch  # noqa: E402

import pgamd  # noqa: E402


def time_ms(fn, reps=20):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    e0.record(s)
    for i in range(reps):
        fn(i)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    lib = pgamd.load()
    sizes = [int(a) << 20 for a in sys.argv[1:]] or [8 << 20, 64 << 20, 256 << 20]
    sh = torch.cuda.current_stream().cuda_stream
    for k in (1, 4, 8):
        for size in sizes:
            sets = 4
            srcs = [[torch.empty(size, dtype=torch.uint8, device="cuda").fill_(j) for j in range(k)] for _ in range(sets)]
            dsts = [torch.empty(size * k, dtype=torch.uint8, device="cuda") for _ in range(sets)]
            arrays = []
            for t in range(sets):
                d = (ctypes.c_void_p * k)(*[dsts[t].data_ptr() + j * size for j in range(k)])
                s = (ctypes.c_void_p * k)(*[srcs[t][j].data_ptr() for j in range(k)])
                nb = (ctypes.c_size_t * k)(*([size] * k))
                arrays.append((d, s, nb))

            def gather(i):
                d, s, nb = arrays[i % sets]
                assert lib.pgk_gather(d, s, nb, k, sh) == 0

            def memcpy(i):
                t = i % sets
                for j in range(k):
                    dsts[t][j * size:(j + 1) * size].copy_(srcs[t][j])

            ms_g = time_ms(gather)
            ms_m = time_ms(memcpy)
            ok = all(torch.equal(dsts[t][j * size:(j + 1) * size], srcs[t][j]) for t in range(sets) for j in range(k))
            moved = 2 * k * size
            print(f"k={k} size={size >> 20:5d} MiB  pgk_gather {ms_g * 1e3:9.1f} us {moved / ms_g / 1e6:7.1f} GB/s"
                  f"   torch copy_ {ms_m * 1e3:9.1f} us {moved / ms_m / 1e6:7.1f} GB/s   ok={ok}", flush=True)
            del srcs, dsts, arrays
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
