"""A plain C program written against include/pg.h (examples/pg_demo.c) builds
with gcc against libpg_amd.so -- the drop-in path for a reference caller --
and, on the GPU, runs as 1 rank and as 2 and 4 real processes (xgmi
transport), checking every element of all-reduce / reduce-scatter /
all-gather against the closed form."""
import os
import pathlib
import socket
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
LIBDIR = ROOT / "rdma-ring-collectives_amd"


def build(tmp_path):
    exe = tmp_path / "pg_demo"
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", f"-I{ROOT / 'include'}", str(ROOT / "examples" / "pg_demo.c"),
                    f"-L{LIBDIR}", "-lpg_amd", f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)], check=True)
    return exe


def test_demo_builds_against_the_drop_in_header(tmp_path):
    assert build(tmp_path).exists()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 4])
def test_demo_runs(tmp_path, world):
    exe = build(tmp_path)
    env = dict(os.environ, PG_DEVICE="0", PG_PORT=str(_port()), PG_TRANSPORT="xgmi")
    for k in ("RANK", "LOCAL_RANK", "PG_RANK"):
        env.pop(k, None)
    hosts = socket.gethostname() if world == 1 else " ".join(["127.0.0.1"] * world)
    procs = []
    for r in range(world):
        e = dict(env)
        if world > 1:
            e["PG_RANK"] = str(r)
        procs.append(subprocess.Popen([str(exe), hosts, "100003"], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=300)
        outs.append((p.returncode, out))
    for rc, out in outs:
        assert rc == 0 and "OK" in out, out
