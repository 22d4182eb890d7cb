"""libpg_amd.so loads on a machine without a GPU, exports every function its
headers declare, keeps the reference's struct pg prefix, and validates
arguments exactly where the reference does -- without touching a device."""
import ctypes
import os
import subprocess
import textwrap

import pgamd


def test_exports_every_declared_symbol(lib):
    names = pgamd.header_symbols()
    assert {"connect_process_group", "pg_close", "pg_all_reduce", "pg_reduce_scatter",
            "pg_all_gather", "pgk_reduce"} <= set(names)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_struct_pg_prefix_matches_reference(tmp_path):
    """Offsets of rank/world_size/chunk_bytes/eager_max/inflight equal those of
    the reference's struct pg (its pg.h:42-46: int, int, size_t, size_t, int)."""
    src = tmp_path / "off.c"
    src.write_text(textwrap.dedent("""
        #include <stdio.h>
        #include <stddef.h>
        #include "pg.h"
        struct ref_prefix { int rank; int world_size; size_t chunk_bytes; size_t eager_max; int inflight; };
        int main(void) {
          printf("%zu %zu %zu %zu %zu\\n", offsetof(struct pg, rank), offsetof(struct pg, world_size),
                 offsetof(struct pg, chunk_bytes), offsetof(struct pg, eager_max), offsetof(struct pg, inflight));
          printf("%zu %zu %zu %zu %zu\\n", offsetof(struct ref_prefix, rank), offsetof(struct ref_prefix, world_size),
                 offsetof(struct ref_prefix, chunk_bytes), offsetof(struct ref_prefix, eager_max),
                 offsetof(struct ref_prefix, inflight));
          printf("%d %d %d %d\\n", (int)DT_INT32, (int)DT_DOUBLE, (int)OP_SUM, (int)OP_PROD);
          return 0;
        }"""))
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", str(pgamd.REPO_ROOT / "include"), str(src), "-o", str(exe)], check=True)
    a, b, enums = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")[:3]
    assert a == b
    assert enums == "0 1 0 1"
    # and the ctypes mirror agrees with the C header
    assert [getattr(pgamd.PgHead, f).offset for f in ("rank", "world_size", "chunk_bytes", "eager_max", "inflight")] \
        == [int(x) for x in a.split()]


def test_validation_without_device(lib):
    buf = (ctypes.c_int * 8)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    # NULL handle / buffers / negative count / bad datatype -> -1 (reference src/pg.c:267,295,325)
    assert lib.pg_reduce_scatter(p, p, 8, 0, 0, None) == -1
    assert lib.pg_all_gather(p, p, 8, 0, None) == -1
    assert lib.pg_all_reduce(p, p, 8, 0, 0, None) == -1
    assert lib.pg_close(None) == 0
    assert lib.connect_process_group(None, None) == -1
    # the kernel ABI checks before touching HIP
    assert lib.pgk_reduce(p, p, 8, 7, 0, None) == -1
    assert b"datatype" in lib.pgk_last_error()
    assert lib.pgk_reduce(p, p, 8, 0, 9, None) == -1
    assert lib.pgk_reduce(None, None, 0, 0, 0, None) == 0     # n == 0: no-op
    assert lib.pgk_reduce(None, p, 5, 0, 0, None) == -1
    assert lib.pgk_version().startswith(b"pgk gfx950")


def test_launch_geometry(lib):
    g, b = ctypes.c_uint(), ctypes.c_uint()
    assert lib.pgk_launch_geometry(1 << 25, 1, ctypes.byref(g), ctypes.byref(b)) == 0
    assert b.value in (256, 512, 1024) and 1 <= g.value
    assert lib.pgk_launch_geometry(16, 7, None, None) == -1
    # the dispatch packet's grid size is 32-bit in work-items: any n stays below 2^32
    for n, dt in ((1 << 40, 1), (1 << 36, 0), ((1 << 31) - 1, 1), (1 << 33, 0)):
        assert lib.pgk_launch_geometry(n, dt, ctypes.byref(g), ctypes.byref(b)) == 0
        assert 1 <= g.value and g.value * b.value < 1 << 32, (n, dt, g.value, b.value)
    # above 512 MiB per operand the call is cut into <= 512 MiB launches: the first one's grid
    for n, dt, grid in ((1 << 26, 1, 32768), ((1 << 26) + 1, 1, 16385), (1 << 27, 1, 32768), (1 << 28, 0, 32768)):
        assert lib.pgk_launch_geometry(n, dt, ctypes.byref(g), ctypes.byref(b)) == 0
        assert (g.value, b.value) == (grid, 1024), (n, dt, g.value, b.value)


def test_connect_without_gpu_fails_cleanly(lib):
    if os.path.exists("/dev/kfd"):
        return  # a GPU machine: covered by the gpu tests
    h = ctypes.c_void_p()
    assert lib.connect_process_group(b"nosuchhost-xyz", ctypes.byref(h)) == -1


def test_headers_compile_as_c_and_cpp(tmp_path):
    """The three public headers are self-contained C and usable from C++
    (extern "C" guards), and `make install` lays out a drop-in prefix."""
    src = tmp_path / "h.c"
    src.write_text('#include "pg.h"\n#include "pg_ext.h"\n#include "pgk.h"\nint main(void){return 0;}\n')
    inc = str(pgamd.REPO_ROOT / "include")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", inc, str(src), "-o", str(tmp_path / "hc")], check=True)
    cpp = tmp_path / "h.cpp"
    cpp.write_text(src.read_text())
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", inc, str(cpp), "-o", str(tmp_path / "hcpp")], check=True)
    subprocess.run(["make", "-s", "-C", str(pgamd.PKG_DIR), "install", f"DESTDIR={tmp_path}", "PREFIX=/opt/pg"],
                   check=True)
    assert (tmp_path / "opt/pg/lib/libpg_amd.so").exists() and (tmp_path / "opt/pg/include/pg.h").exists()


def test_fold_launch_rule(lib):
    """How pgk_reduce_multi / pgk_fold_timed cut a fold into launches (host
    arithmetic, no device): the burst form from 5 to 8 sources and 32 MiB per
    source; 64 MiB launches of 32 tiles per wave and a last one of 32-64 MiB at
    16 tiles when the fold has the GPU to itself, 32 MiB launches beside other
    kernels, never for remote sources; the rest one tile per wave."""
    MiB = 1 << 20
    SZ, I = ctypes.c_size_t, ctypes.c_int

    def cut(nbytes, nsrc=8, flags=0, dt=pgamd.DT_DOUBLE):
        es = 8 if dt == pgamd.DT_DOUBLE else 4
        lb, lt, plain = (SZ * 8)(), (I * 8)(), SZ()
        k = lib.pgk_fold_geometry(nbytes // es, dt, nsrc, flags, lb, lt, 8, ctypes.byref(plain))
        assert k >= 0, pgamd.last_error()
        return [(lb[i] // MiB, lt[i]) for i in range(min(k, 8))], plain.value / MiB, k

    assert cut(64 * MiB) == ([(64, 32)], 0, 1)
    assert cut(64 * MiB, dt=pgamd.DT_INT32) == ([(64, 32)], 0, 1)
    assert cut(256 * MiB) == ([(64, 32)] * 4, 0, 4)
    assert cut(72 * MiB) == ([(64, 32)], 8, 1)                      # a rest under 32 MiB: one tile per wave
    assert cut(100 * MiB) == ([(64, 32), (36, 16)], 0, 2)           # a rest of 32-64 MiB: one 16-tile launch
    assert cut(40 * MiB) == ([(40, 16)], 0, 1)
    assert cut(32 * MiB) == ([(32, 16)], 0, 1)
    assert cut(31 * MiB) == ([], 31, 0)                             # under 32 MiB per source: plain
    assert cut(64 * MiB, nsrc=4) == ([], 64, 0) and cut(64 * MiB, nsrc=9) == ([], 64, 0)
    assert cut(64 * MiB, nsrc=5)[0] == [(64, 32)]
    shared = pgamd.FOLD_SHARED_GPU
    assert cut(64 * MiB, flags=shared) == ([(32, 16), (32, 16)], 0, 2)
    assert cut(100 * MiB, flags=shared) == ([(32, 16)] * 3, 4, 3)
    assert cut(256 * MiB, flags=pgamd.FOLD_REMOTE_SOURCES) == ([], 256, 0)
    assert cut(256 * MiB, flags=pgamd.FOLD_REMOTE_SOURCES | shared) == ([], 256, 0)
    # the API's largest double count: 256 launches, the first 8 reported
    first, plain, k = cut(((1 << 31) - 1) * 8)
    assert k == 256 and first == [(64, 32)] * 8 and plain < 1 / 1024 * 64
    assert lib.pgk_tune_fold(0) == 0
    try:
        assert cut(256 * MiB) == ([], 256, 0)
    finally:
        lib.pgk_tune_fold(1)
    assert lib.pgk_fold_geometry(8, 2, 8, 0, None, None, 0, None) == -1
