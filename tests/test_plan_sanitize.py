"""Host C code under AddressSanitizer and UndefinedBehaviorSanitizer (GPU
sanitizers are not available on the MI355X pool):
  - the ring planner (pure C, csrc/pg_plan.c) over a grid of shapes
    (tests/c/plan_fuzz.c): no invalid access, no UB, every step's offsets
    inside its buffer;
  - the bootstrap star and shared-memory barrier (csrc/pg_boot.c) with 2, 3
    and 8 forked processes (tests/c/boot_fuzz.c)."""
import pathlib
import socket
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_planner_clean_under_asan_ubsan(tmp_path):
    exe = tmp_path / "plan_fuzz"
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    f"-I{ROOT / 'include'}", str(ROOT / "tests" / "c" / "plan_fuzz.c"),
                    str(ROOT / "rdma-ring-collectives_amd" / "csrc" / "pg_plan.c"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.returncode, r.stdout[-500:], r.stderr[-2000:])


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bootstrap_clean_under_asan_ubsan(tmp_path, world):
    exe = tmp_path / "boot_fuzz"
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'rdma-ring-collectives_amd' / 'csrc'}", str(ROOT / "tests" / "c" / "boot_fuzz.c"),
                    str(ROOT / "rdma-ring-collectives_amd" / "csrc" / "pg_boot.c"), "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), str(world), str(_port())], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.returncode, r.stdout[-500:], r.stderr[-2000:])
