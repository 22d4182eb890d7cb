"""Plain C programs written against include/pg.h (examples/pg_demo.c, the
Quick Start; examples/pg_sweep.c, the CSV size sweep) build with gcc against
libpg_amd.so -- the drop-in path for a reference caller -- and, on the GPU,
run as 1 rank and as 2 and 4 real processes (xgmi transport), checking every
element of all-reduce / reduce-scatter / all-gather against the closed form."""
import os
import pathlib
import socket
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
LIBDIR = ROOT / "rdma-ring-collectives_amd"


def build(tmp_path, name="pg_demo"):
    exe = tmp_path / name
    subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", f"-I{ROOT / 'include'}",
                    str(ROOT / "examples" / f"{name}.c"), f"-L{LIBDIR}", "-lpg_amd", f"-Wl,-rpath,{LIBDIR}",
                    "-o", str(exe)], check=True)
    return exe


def test_demo_builds_against_the_drop_in_header(tmp_path):
    assert build(tmp_path).exists()
    assert build(tmp_path, "pg_sweep").exists()


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


@pytest.mark.gpu
@pytest.mark.parametrize("coll,dt,op", [("allreduce", "int32", "sum"), ("reducescatter", "double", "prod"),
                                        ("allgather", "double", "sum")])
def test_sweep_harness_runs(tmp_path, coll, dt, op):
    """examples/pg_sweep.c: the reference's CSV perf discipline (README.md:83-85)
    over 2 real processes, every size checked against the closed form."""
    exe = build(tmp_path, "pg_sweep")
    env = dict(os.environ, PG_DEVICE="0", PG_PORT=str(_port()), PG_TRANSPORT="xgmi")
    for k in ("RANK", "LOCAL_RANK"):
        env.pop(k, None)
    procs = [subprocess.Popen([str(exe), "127.0.0.1 127.0.0.1", coll, dt, op, "4096", str(4 << 20), "2"],
                              env=dict(env, PG_RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(2)]
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 0 and "OK" in err, (out, err)
    rows = outs[0][0].strip().splitlines()
    assert rows[0] == "size,rounds,inflight,time_us,GB/s"
    assert [int(x.split(",")[0]) for x in rows[1:]] == [4096, 16384, 65536, 262144, 1048576, 4194304]
