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
import time

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
        # the time budget: one answer on every rank, decided by the slowest clock
        # (rank 1 started its clock "200 s ago"; the others just now)
        bench._T0 = time.perf_counter() - (200.0 if rank == 1 else 0.0)
        bench._BUDGET_S = None
        assert bench.past_budget(world) is False
        bench._BUDGET_S = 100.0
        assert bench.past_budget(world) is True
        bench._BUDGET_S = 1000.0
        assert bench.past_budget(world) is False
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


def test_sweep_summary_names_the_fastest_row_per_schedule():
    """bench._sweep_summary: per schedule, the fastest row of the knob and its
    gain over that schedule's default row."""
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    import bench
    cols = bench.SWEEP_COLUMNS
    assert cols[:5] == ["size", "rounds", "inflight", "time_us", "GB/s"] and "algo" in cols
    rows = [[1 << 30, 3, 4, 100.0, 10.0, 1 << 20, 0, "direct", 0.70], [1 << 30, 3, 4, 50.0, 20.0, 4 << 20, 1, "direct", 0.78],
            [1 << 30, 3, 4, 40.0, 25.0, 16 << 20, 0, "direct", 0.80], [1 << 30, 3, 4, 90.0, 11.0, 4 << 20, 1, "ring", 0.79],
            [1 << 30, 3, 4, 80.0, 12.1, 8 << 20, 0, "ring", 0.81]]
    s = bench._sweep_summary(rows, cols.index("chunk_bytes"))
    assert s["direct"] == {"fastest": 16 << 20, "fastest_GBps": 25.0, "fastest_over_default": 1.25,
                           "in_ring_reduce_frac_at_default": 0.78}
    assert s["ring"]["fastest"] == 8 << 20 and s["ring"]["fastest_over_default"] == 1.1


def test_preflight_reads_a_childs_output():
    """What a preflight child printed decides each transport: ok, bad (with its
    reason), the one it died in, and the ones it never reached."""
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    import bench
    names = ["xgmi", "xgmi_push", "rccl"]
    got = bench._read_preflight(names, ["start xgmi", "ok xgmi", "start xgmi_push", "ok xgmi_push", "start rccl",
                                        "ok rccl"], 0)
    assert [got[t][0] for t in names] == [bench._PF_OK] * 3
    got = bench._read_preflight(names, ["start xgmi", "ok xgmi", "start xgmi_push"], -6,
                                "warning\nMemory access fault by GPU node-2\n")
    assert got["xgmi"][0] == bench._PF_OK and got["rccl"][0] == bench._PF_NOT_REACHED
    assert got["xgmi_push"][0] == bench._PF_FAILED
    assert "signal 6" in got["xgmi_push"][1] and "Memory access fault" in got["xgmi_push"][1]
    got = bench._read_preflight(names, ["start xgmi", "bad xgmi: all_reduce(512): wrong result", "start xgmi_push",
                                        "ok xgmi_push", "start rccl"], "time limit")
    assert got["xgmi"] == (bench._PF_FAILED, "xgmi: all_reduce(512): wrong result")
    assert got["xgmi_push"][0] == bench._PF_OK
    assert got["rccl"][0] == bench._PF_FAILED and "time limit" in got["rccl"][1]
    assert bench._read_preflight(names, [], 1)["xgmi"][0] == bench._PF_NOT_REACHED


def _preflight_worker(rank, world, port, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        rounds = []

        def child(left, args):
            # rank 1's child dies inside xgmi_push (first round); everything else finishes clean
            rounds.append(list(left))
            lines = []
            for t in left:
                lines.append(f"start {t}")
                if t == "xgmi_push" and rank == 1:
                    return bench._read_preflight(left, lines, -6, "Memory access fault by GPU\n")
                lines.append(f"ok {t}")
            return bench._read_preflight(left, lines, 0)

        names = ["xgmi", "xgmi_push", "xgmi_read", "rccl"]
        verdict = bench.preflight(None, rank, world, names, run_child=child)
        q.put((rank, verdict, rounds))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_preflight_ranks_agree_and_later_transports_get_a_fresh_round():
    """One rank's child dies in the second transport: every rank drops exactly
    that transport, keeps the one before it, and sends the ones after it to a
    second round of children (where they pass)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_preflight_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, verdict, rounds in res:
        assert isinstance(verdict, dict), verdict
        assert verdict["xgmi"] is None and verdict["xgmi_read"] is None and verdict["rccl"] is None
        assert rounds == [["xgmi", "xgmi_push", "xgmi_read", "rccl"], ["xgmi_read", "rccl"]]
    assert "signal 6" in res[1][1]["xgmi_push"] and "another rank" in res[0][1]["xgmi_push"]


def test_more_ranks_than_gpus_becomes_the_one_gpu_rehearsal(monkeypatch):
    """Launched with more ranks on the node than it has GPUs, every rank takes
    the one-GPU rehearsal (device 0, per-rank RCCL host id, divided ring
    shapes) instead of failing on a device that does not exist.  The decision
    uses only the node's device count, so all ranks decide alike."""
    sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
    import argparse
    import bench
    import torch
    for k in ("PG_BENCH_ONE_GPU", "PG_BENCH_ONE_GPU_AUTO", "PG_DEVICE", "NCCL_HOSTID"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    for rank in (0, 3):
        monkeypatch.setenv("WORLD_SIZE", "4")
        monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
        monkeypatch.setenv("RANK", str(rank))
        monkeypatch.setenv("LOCAL_RANK", str(rank))
        monkeypatch.delenv("PG_BENCH_ONE_GPU", raising=False)
        args = argparse.Namespace(gpus=4, ring_div=1)
        assert bench.rank_setup(args) == (rank, 4, 0)
        assert os.environ["PG_BENCH_ONE_GPU"] == "1" and os.environ["PG_DEVICE"] == "0"
        assert os.environ["NCCL_HOSTID"].endswith(f"rank{rank}") and args.ring_div == 4
    # enough GPUs: nothing changes
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    for k in ("PG_BENCH_ONE_GPU", "PG_BENCH_ONE_GPU_AUTO", "PG_DEVICE", "NCCL_HOSTID"):
        monkeypatch.delenv(k, raising=False)
    args = argparse.Namespace(gpus=4, ring_div=1)
    assert bench.rank_setup(args) == (3, 4, 3) and "PG_BENCH_ONE_GPU" not in os.environ and args.ring_div == 1
