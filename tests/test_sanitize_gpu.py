"""The host side of the ring path under AddressSanitizer + UndefinedBehavior-
Sanitizer, on the GPU (tests/c/sim_asan.c, built by tests/c/Makefile.asan from
__graft_entry__.build()): plan, executor, staging hooks, eager one-shot, the
direct exchange (PG_ALGO=direct), threads transport and the host-operand
reduce over 432 cases (1, 2 and 4 rings), every result bit for bit against the
oracle's ring simulator.  Host code only: the kernels are
built without sanitizers (GPU sanitizers are not available on this pool)."""
import os
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
EXE = ROOT / "build" / "asan" / "sim_asan"

pytestmark = pytest.mark.gpu


def test_ring_host_code_clean_under_asan_ubsan(gpu):
    if not EXE.exists():
        pytest.fail(f"{EXE} missing: run __graft_entry__.build() (make -f tests/c/Makefile.asan)")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(EXE)], capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
