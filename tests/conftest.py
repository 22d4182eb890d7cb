"""Shared fixtures.  `-m "not gpu"` runs everywhere; `-m gpu` needs an MI355X.

The oracle (oracle/) is test infrastructure: it is the checker here, never the
thing under test.  The product is rdma-ring-collectives_amd/libpg_amd.so,
reached through its C-ABI (pgamd.py is a ctypes binding, no implementation).
"""
import json
import pathlib
import subprocess
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "rdma-ring-collectives_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950); run with -m gpu")


def _make(args):
    subprocess.run(["make", "-s", "-j8"] + args, check=True, cwd=ROOT)


def pytest_sessionstart(session):
    # build what is missing (cheap no-op when __graft_entry__.build() already ran)
    if not (ROOT / "oracle" / "liboracle.so").exists():
        _make(["-C", "oracle", "liboracle.so"])
    if not (PKG / "libpg_amd.so").exists():
        _make(["-C", str(PKG)])


@pytest.fixture(scope="session")
def golden():
    manifest = json.loads((GOLDEN / "golden.json").read_text())
    arrays = np.load(GOLDEN / "golden.npz", allow_pickle=False)
    return manifest, arrays


@pytest.fixture(scope="session")
def oracle():
    from oracle.pyoracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def lib():
    import pgamd
    return pgamd.load()


@pytest.fixture(scope="session")
def gpu():
    """torch on cuda:0 -- device memory and streams only (plumbing)."""
    import torch
    assert torch.cuda.is_available(), "gpu tests need a visible MI355X"
    torch.cuda.set_device(0)
    import pgamd
    pgamd.load()
    return torch
