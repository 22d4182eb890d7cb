#!/usr/bin/env python3
"""EXPERIMENTS ONLY: does kernel-argument preloading shorten the launch ramp?

Every wave of the shipped reduce starts with scalar loads of its kernel
arguments (the operand pointers and the vector count) and can issue no global
load before they return.  gfx950 can have the dispatcher place the first
kernel-argument dwords in user SGPRs instead (LLVM
`-amdgpu-kernarg-preload-count`; the code object keeps a 256-byte prologue
that loads them the old way for firmware that cannot preload).  This probe
builds the UNCHANGED csrc/pgk_reduce.hip a second time with that flag into
tools/lab/libpgk_preload.so and times both builds on the same operands, in
interleaved rounds over a 4 GiB pool:

  stamped : median of kernel-stamped launches (pgk_reduce_timed; what rocprofv3 reports)
  events  : 20 back-to-back launches bracketed by events (the size table's kernel_us)

    python tools/lab/preload_probe.py [MiB per operand ...]   (default 16 32 64 128 256)
    python tools/lab/preload_probe.py --build                  build the preload library only (on the CPU host)
"""
import ctypes
import pathlib
import statistics
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
LAB = pathlib.Path(__file__).resolve().parent
SO = LAB / "libpgk_preload.so"


def build():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fvisibility=hidden", f"-I{ROOT / 'include'}", "-mllvm", "-amdgpu-kernarg-preload-count=16",
           str(ROOT / "rdma-ring-collectives_amd/csrc/pgk_reduce.hip"), "-o", str(SO)]
    subprocess.run(cmd, check=True)
    for junk in LAB.glob(SO.name + ".0.*"):      # hipcc's offload-bundle leftovers
        junk.unlink()


if "--build" in sys.argv:
    build()
    sys.exit(0)
if not SO.exists():
    build()

sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

ship = pgamd.load()
pre = ctypes.CDLL(str(SO))
for lib in (pre,):
    lib.pgk_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p]
    lib.pgk_reduce_timed.argtypes = lib.pgk_reduce.argtypes + [ctypes.c_void_p, ctypes.c_void_p]
    lib.pgk_event_create.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    lib.pgk_event_elapsed_ms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    lib.pgk_last_error.restype = ctypes.c_char_p
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
base = pool.data_ptr()
sizes = [int(a) << 20 for a in sys.argv[1:] if a.isdigit()] or [m << 20 for m in (16, 32, 64, 128, 256)]
ROUNDS, BURST = 12, 20
LIBS = {"shipped": ship, "preload": pre}


def evpair(lib):
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.pgk_event_create(ctypes.byref(a)) == 0 and lib.pgk_event_create(ctypes.byref(b)) == 0
    return a, b


evs = {k: evpair(v) for k, v in LIBS.items()}
# bit-exactness of the preload build on one size (same inputs, both builds)
n = (16 << 20) // 8
x0 = pool[:n].clone()
y0 = pool[n:2 * n].clone()
xa, xb = x0.clone(), x0.clone()
assert ship.pgk_reduce(xa.data_ptr(), y0.data_ptr(), n, 1, 0, sh) == 0
assert pre.pgk_reduce(xb.data_ptr(), y0.data_ptr(), n, 1, 0, sh) == 0
torch.cuda.synchronize()
print(f"preload build bit-exact vs shipped: {bool(torch.equal(xa, xb))}", flush=True)
del x0, y0, xa, xb
for total in sizes:
    n = total // 8
    pairs = POOL // (2 * total)
    st = {k: [] for k in LIBS}
    ev = {k: [] for k in LIBS}
    i = 0
    for rnd in range(ROUNDS + 1):
        for name, lib in LIBS.items():
            # kernel-stamped single launch
            d = base + 2 * total * (i % pairs)
            i += 1
            e0, e1 = evs[name]
            assert lib.pgk_reduce_timed(d, d + total, n, 1, 0, sh, e0, e1) == 0
            torch.cuda.synchronize()
            ms = ctypes.c_float()
            assert lib.pgk_event_elapsed_ms(e0, e1, ctypes.byref(ms)) == 0
            # a burst of back-to-back launches bracketed by events
            b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b0.record()
            for _ in range(BURST):
                d = base + 2 * total * (i % pairs)
                i += 1
                assert lib.pgk_reduce(d, d + total, n, 1, 0, sh) == 0
            b1.record()
            torch.cuda.synchronize()
            if rnd:
                st[name].append(ms.value * 1e3)
                ev[name].append(b0.elapsed_time(b1) * 1e3 / BURST)
    print(f"== {total >> 20} MiB per operand (f64 sum), medians of {ROUNDS} rounds ==", flush=True)
    for name in LIBS:
        s, e = statistics.median(st[name]), statistics.median(ev[name])
        print(f"  {name:8s} stamped {s:8.2f} us ({3 * total / s / 1e3 / 80:5.1f}% of 8 TB/s)   "
              f"events {e:8.2f} us ({3 * total / e / 1e3 / 80:5.1f}%)", flush=True)
