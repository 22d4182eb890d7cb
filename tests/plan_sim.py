"""Test-side executor of libpg_amd.so's ring plans (struct pg_step), in numpy.

Used to check the HOST SCHEDULE without a GPU: each rank's plan -- produced by
the library's pg_plan_* C functions -- is executed with per-edge FIFO channels
(the semantics of ncclSend/ncclRecv between ring neighbours) and the reduction
is done here with numpy's wrapping/IEEE arithmetic.  A step sends to rank
(r + send_peer) and receives from rank (r + recv_peer), one FIFO per directed
edge, so both ring directions are simulated.  This file is test
infrastructure; nothing in the library calls it.
"""
from __future__ import annotations

from collections import deque

import numpy as np

import pgamd

NP = {0: np.int32, 1: np.float64}


def np_reduce(dst: np.ndarray, src: np.ndarray, op: int, rev: int = 0) -> None:
    """dst op= src, or dst = src op dst (rev: a plan step's red_rev)."""
    if rev:
        tmp = src.copy()
        np_reduce(tmp, dst, op)
        dst[:] = tmp
        return
    if dst.dtype == np.int32:
        d, s = dst.view(np.uint32), src.view(np.uint32)
        if op == 0:
            np.add(d, s, out=d)
        else:
            np.multiply(d, s, out=d)
    else:
        if op == 0:
            np.add(dst, src, out=dst)
        else:
            np.multiply(dst, src, out=dst)


def _view(bufs, which, off, nbytes):
    b = bufs[which]
    return b[off:off + nbytes]


def direct_fold(bufs, s, rank, world, dt, op):
    """A fold step of a direct plan (include/pg_ext.h): OUT = x[r+d] op x[r+2d]
    op ... op x[r], x[q] = slot q of STAGE0, x[r] = this rank's own block in SRC;
    bufs["ctx"] = (rings, full block elements, block offset)."""
    rings, full, boff = bufs["ctx"]
    es = 4 if dt == 0 else 8
    n = s["red_elems"] * es
    d = pgamd.ring_offset(world, rings, s["seg"])
    acc = None
    for k in range(world):
        q = (rank + (k + 1) * d) % world
        if q == rank:
            x = _view(bufs, pgamd.PG_BUF_SRC, boff * es + s["red_src_off"], n)
        else:
            x = _view(bufs, pgamd.PG_BUF_STAGE0, q * full * es + s["red_src_off"], n)
        x = x.view(NP[dt])
        if acc is None:
            acc = x.copy()
        else:
            np_reduce(acc, x, op)
    _view(bufs, s["red_dst_buf"], s["red_dst_off"], n).view(NP[dt])[:] = acc


def _reduce_ranges(bufs, steps, es, dt, op):
    """One reduce launch of the executor over `steps`: the library's own
    pg_plan_coalesce lists the ranges, numpy reduces each."""
    total = 0
    for g in pgamd.plan_coalesce(steps, es):
        d = _view(bufs, g["dst_buf"], g["dst_off"], g["elems"] * es).view(NP[dt])
        src = _view(bufs, g["src_buf"], g["src_off"], g["elems"] * es).view(NP[dt])
        np_reduce(d, src, op, g["rev"])
        total += g["elems"]
    assert total == sum(s["red_elems"] for s in steps)          # nothing lost, nothing twice
    return len(steps)


def run_plans(plans, bufs_per_rank, dt, op, red_bytes=None):
    """Execute every rank's step list.  bufs_per_rank[r][PG_BUF_*] = uint8 arrays.
    A step runs once all its receives are available; sends snapshot the bytes
    at send time (a rank's steps run in order, so a forwarded partial is
    already reduced, as the executor's red_ev wait guarantees).
    red_bytes = None: every step reduces on arrival.  Otherwise the executor's
    rule (csrc/pg_exec.c, PG_REDUCE_BYTES): a batch's reduce steps wait until
    red_bytes per operand are pending, or the round or the plan ends, and are
    then reduced range by range as pg_plan_coalesce lists them.  Returns the
    number of reduce launches per rank (ring steps only)."""
    world = len(plans)
    chans = {(a, b): deque() for a in range(world) for b in range(world)}     # directed edge a -> b
    pos = [0] * world
    # group steps into batches per rank
    batches = []
    for st in plans:
        bl, cur = [], None
        for s in st:
            if cur is None or s["batch"] != cur[0]["batch"]:
                cur = []
                bl.append(cur)
            cur.append(s)
        batches.append(bl)
    es = 4 if dt == 0 else 8
    pending = [None] * world      # sends of a batch are posted before its receives
    waiting = [[] for _ in range(world)]          # reduce steps not launched yet (red_bytes mode)
    launches = [0] * world
    progress = True
    while progress:
        progress = False
        for r in range(world):
            if pos[r] >= len(batches[r]):
                continue
            batch = batches[r][pos[r]]
            bufs = bufs_per_rank[r]
            if pending[r] is None:
                for s in batch:
                    # a forwarded partial was reduced in the previous round: no step of an
                    # earlier round may still wait for its launch when this round sends
                    assert not (s["send_bytes"] and s.get("send_wait") and
                                any(w["round"] < s["round"] for w in waiting[r])), (r, s)
                    if s["send_bytes"]:
                        chans[(r, (r + s["send_peer"]) % world)].append(
                            _view(bufs, s["send_buf"], s["send_off"], s["send_bytes"]).copy())
                pending[r] = True
                progress = True
            need = {}
            for s in batch:
                if s["recv_bytes"]:
                    q = (r + s["recv_peer"]) % world
                    need[q] = need.get(q, 0) + 1
            if any(len(chans[(q, r)]) < k for q, k in need.items()):
                continue
            for s in batch:
                if s["recv_bytes"]:
                    msg = chans[((r + s["recv_peer"]) % world, r)].popleft()
                    assert msg.size == s["recv_bytes"], (r, s, msg.size)
                    _view(bufs, s["recv_buf"], s["recv_off"], s["recv_bytes"])[:] = msg
            for s in batch:
                if s.get("red_fold"):
                    direct_fold(bufs, s, r, world, dt, op)
                elif s["red_elems"] and red_bytes is None:
                    d = _view(bufs, s["red_dst_buf"], s["red_dst_off"], s["red_elems"] * es).view(NP[dt])
                    src = _view(bufs, s["red_src_buf"], s["red_src_off"], s["red_elems"] * es).view(NP[dt])
                    np_reduce(d, src, op, s.get("red_rev", 0))
                    launches[r] += 1
                elif s["red_elems"]:
                    waiting[r].append(s)
            if waiting[r]:
                last = pos[r] + 1 == len(batches[r])
                round_ends = last or batches[r][pos[r] + 1][0]["round"] != batch[0]["round"]
                if round_ends or sum(s["red_elems"] for s in waiting[r]) * es >= red_bytes:
                    _reduce_ranges(bufs, waiting[r], es, dt, op)
                    launches[r] += 1
                    waiting[r] = []
            pos[r] += 1
            pending[r] = None
            progress = True
    assert all(pos[r] == len(batches[r]) for r in range(world)), "deadlock"
    assert all(len(c) == 0 for c in chans.values()), "unconsumed messages"
    assert not any(waiting), "reduce steps left pending"
    return launches


def ring_reduce_scatter(sends, dt, op, chunk_bytes, eager_max=4096, inflight=4, alias=False, rings=2, red_bytes=None,
                        launches_out=None):
    world, count = len(sends), sends[0].size
    es = 4 if dt == 0 else 8
    blk = -(-count // world) if count else 0
    bmax = rings * -(-blk // rings) * es          # staging block: R * ceil(B/R) elements (include/pg_ext.h)
    plans, bufs = [], []
    for r in range(world):
        plans.append(pgamd.plan_reduce_scatter(r, world, count, dt, chunk_bytes, eager_max, inflight, int(alias),
                                               rings))
        off, ln = pgamd.block_range(count, world, r)
        src = sends[r].copy().view(np.uint8)
        if alias:
            out = src[off * es:(off + ln) * es]
        else:
            out = np.zeros(ln * es, np.uint8)
        bufs.append({pgamd.PG_BUF_SRC: src, pgamd.PG_BUF_OUT: out,
                     pgamd.PG_BUF_STAGE0: np.zeros(bmax, np.uint8), pgamd.PG_BUF_STAGE1: np.zeros(bmax, np.uint8)})
    launches = run_plans(plans, bufs, dt, op, red_bytes)
    if launches_out is not None:
        launches_out[:] = launches
    return [bufs[r][pgamd.PG_BUF_OUT].view(NP[dt]).copy() for r in range(world)], bufs


def ring_all_gather(sends, dt, rings=2):
    world, count = len(sends), sends[0].size
    es = 4 if dt == 0 else 8
    plans, bufs = [], []
    for r in range(world):
        plans.append(pgamd.plan_all_gather(r, world, count, dt, 1, rings))
        full = np.zeros(count * world * es, np.uint8)
        full[r * count * es:(r + 1) * count * es] = sends[r].view(np.uint8)
        bufs.append({pgamd.PG_BUF_OUT: full})
    run_plans(plans, bufs, dt, 0)
    return [b[pgamd.PG_BUF_OUT].view(NP[dt]).copy() for b in bufs]


def ring_all_reduce(sends, dt, op, chunk_bytes, eager_max=4096, inflight=4, rings=2, red_bytes=None):
    world, count = len(sends), sends[0].size
    _, bufs = ring_reduce_scatter(sends, dt, op, chunk_bytes, eager_max, inflight, alias=True, rings=rings,
                                  red_bytes=red_bytes)
    plans = [pgamd.plan_all_gather(r, world, count, dt, 0, rings) for r in range(world)]
    agbufs = [{pgamd.PG_BUF_OUT: bufs[r][pgamd.PG_BUF_SRC]} for r in range(world)]
    run_plans(plans, agbufs, dt, 0)
    return [agbufs[r][pgamd.PG_BUF_OUT].view(NP[dt]).copy() for r in range(world)]


def direct_reduce_scatter(sends, dt, op, chunk_bytes, inflight=4, rings=2):
    """PG_ALGO=direct: every rank's pg_plan_direct_reduce_scatter steps run
    together (one hop per block over every link, folds in ring order)."""
    world, count = len(sends), sends[0].size
    es = 4 if dt == 0 else 8
    full = -(-count // world) if count else 0
    plans, bufs = [], []
    for r in range(world):
        plans.append(pgamd.plan_direct_reduce_scatter(r, world, count, dt, chunk_bytes, inflight, rings))
        off, ln = pgamd.block_range(count, world, r)
        bufs.append({pgamd.PG_BUF_SRC: sends[r].copy().view(np.uint8), pgamd.PG_BUF_OUT: np.zeros(ln * es, np.uint8),
                     pgamd.PG_BUF_STAGE0: np.zeros(world * full * es, np.uint8), "ctx": (rings, full, off)})
    run_plans(plans, bufs, dt, op)
    return [bufs[r][pgamd.PG_BUF_OUT].view(NP[dt]).copy() for r in range(world)]
