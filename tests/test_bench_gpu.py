"""bench.py's RCCL-native cross-check, rehearsed at world 1.

The cross-check compares pg_reduce_scatter with RCCL's own reduce-scatter.  It
only means something at N > 1 (the driver's multi-GPU bench), and RCCL
refuses two ranks on one GPU, so here it runs at world 1 on the test GPU: the
RCCL group is created, both reduce-scatters run, the tolerance arithmetic is
evaluated, and every check must come out true.  A child process keeps the
torch.distributed state out of the test runner.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import ctypes, json, os, sys
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "rdma-ring-collectives_amd")]
import torch
import torch.distributed as dist
import bench, pgamd
torch.cuda.set_device(0)
dist.init_process_group("gloo", rank=0, world_size=1)
lib = pgamd.load()
h = ctypes.c_void_p()
pgamd.check(lib.connect_process_group(b"127.0.0.1", ctypes.byref(h)), "connect")
x = torch.arange(1 << 20, dtype=torch.float64, device="cuda")
res = bench.native_crosscheck(lib, h, 0, 1, x, pgamd.DT_DOUBLE)
lib.pg_close(h)
dist.destroy_process_group()
print(json.dumps(res))
"""


def test_native_crosscheck_world1():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29611", PG_RANK="0", PG_PORT="29612")
    r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["i32_sum_bit_exact"] is True, res
    assert res["f64_sum_within_tol"] is True, res
    assert res["i32_prod_bit_exact"] is True, res
    assert res["f64_prod_within_tol"] is True, res
    assert res["i32_all_reduce_bit_exact"] is True, res
    assert res["i32_all_gather_bit_exact"] is True, res
    assert res["f64_sum_bit_identical_frac"] == 1.0, res   # one rank: both are plain copies
    assert res["f64_prod_bit_identical_frac"] == 1.0, res
    assert res["rccl_reduce_scatter_ms"] > 0, res
