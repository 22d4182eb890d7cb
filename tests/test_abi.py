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
