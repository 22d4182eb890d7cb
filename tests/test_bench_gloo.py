"""bench.py's N>1 bookkeeping on CPU: world_size 2 and 3 over torch.distributed gloo.

At N>1 every rank checks its reduce-scatter block on the device against
bench._expected_block (the sum/product of every rank's bench._pattern), and
rank 0 reports times and flags combined over ranks.  Here each process builds
its pattern on the CPU, the ranks all-gather them over gloo (the exchange the
ring performs), and the expected block must equal the oracle's ring
reduce-scatter (oracle/pg_oracle.c, pinned to the reference) bit for bit, for
both dtypes and both ops, 1 and 2 rings, ragged counts included.  The rank
aggregations (max, per-rank gather, sum) are checked on the same group."""
import os
import pathlib
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import pgamd
        from oracle.pyoracle import Oracle
        orc = Oracle()
        assert bench.max_over_ranks(rank + 0.5, world) == world - 0.5
        assert bench.gather_over_ranks(10.0 * rank, rank, world) == [10.0 * r for r in range(world)]
        assert bench.sum_over_ranks(1.0, world) == float(world)
        bench.barrier(world)
        checked = 0
        for dt in (pgamd.DT_INT32, pgamd.DT_DOUBLE):
            for op in (pgamd.OP_SUM, pgamd.OP_PROD):
                for count in (world, 1000, 4099, 65537):
                    x = bench._pattern(count, rank, world, dt, op, device="cpu")
                    parts = [torch.empty_like(x) for _ in range(world)]
                    dist.all_gather(parts, x)
                    sends = [p.numpy() for p in parts]
                    off, ln = pgamd.block_range(count, world, rank)
                    want = bench._expected_block(count, off, ln, world, dt, op, device="cpu").numpy()
                    for rings in (1, 2):
                        ring = orc.ring_reduce_scatter(sends, dt, op, rings)[rank]
                        assert ring.size == ln and ring.tobytes() == want.tobytes(), (dt, op, count, rings)
                        checked += 1
        ok = bench.sum_over_ranks(1.0, world) == world
        q.put((rank, checked, ok))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, -1, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_expected_blocks_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, checked, ok in results:
        assert checked == 2 * 2 * 4 * 2 and ok is True, (rank, checked, ok)
