/*
 * pg_exec.c -- executes a ring plan (pg_plan.c) on one rank.
 *
 * Two HIP streams per rank:
 *   comm : transport groups (RCCL ncclSend/ncclRecv over xGMI), in plan order
 *   red  : the reduce launches
 * and two kinds of events:
 *   recv_ev[batch]  comm -> red : the batch's segments have landed
 *   red_ev[seg]     red -> comm : the segment's partial is reduced and may be
 *                                 forwarded in the next round
 * so segment j of round k+1 is on the wire while later segments of round k
 * are still arriving.  This is the pipelining that the reference describes
 * for its RDMA path (README.md:17,74-77) and mocks with one synchronous local
 * call per chunk (src/pg.c:276-289).
 *
 * The link segment and the reduce launch are separate sizes.  A transport
 * group carries chunk_bytes x inflight per ring (what the links like); the
 * arrived segments of a round wait until red_bytes per operand are pending
 * (PG_REDUCE_BYTES, default 128 MiB) or the round ends, and are then reduced
 * by ONE pgk_reduce_ranges launch, one contiguous range per ring.  A launch of
 * that size streams at 80-82% of the HBM peak where a 32 MiB one reaches
 * 71-73%.  Forwarding is not held up: a round's first sends need the previous
 * round's first launch only, which ran long before the round's last arrival.
 *
 * One reduce stream on purpose.  Alternating the launches between two streams
 * lets one launch's drain overlap the next one's ramp, which helps launches of
 * 32 MiB per operand and less (+7 points of the HBM peak back to back) and
 * costs 2-4 points at 128-256 MiB, the size the launches have here
 * (tools/lab/split2_lab.hip, "whole calls alternating between two streams").
 *
 * Buffer reuse is safe by construction: a staging segment is overwritten by a
 * receive two rounds later, which the comm stream orders after the send of
 * the intervening round, and that send waited on the segment's reduce.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pg_impl.h"

static int ensure_red_events(struct pg_impl *im, int need) {
  if (need <= im->n_red_ev) return 0;
  int cap = im->n_red_ev ? im->n_red_ev : 16;
  while (cap < need) cap *= 2;
  hipEvent_t *ev = (hipEvent_t *)realloc(im->red_ev, sizeof(hipEvent_t) * (size_t)cap);
  if (!ev) { pg_set_error("pg_exec: out of host memory"); return -1; }
  im->red_ev = ev;
  for (int i = im->n_red_ev; i < cap; ++i) {
    hipError_t e = hipEventCreateWithFlags(&im->red_ev[i], hipEventDisableTiming);
    if (e != hipSuccess) {
      im->n_red_ev = i;
      pg_set_error("pg_exec: hipEventCreate: %s", hipGetErrorString(e));
      return -1;
    }
  }
  im->n_red_ev = cap;
  return 0;
}

static int pg_world_of(const struct pg_impl *im) { return im->pg->world_size; }

static inline char *at(void *const bufs[5], int which, int64_t off) {
  return (char *)bufs[which] + off;
}

static int ensure_round_events(struct pg_impl *im, int need) {
  if (need <= im->n_round_ev) return 0;
  hipEvent_t *ev = (hipEvent_t *)realloc(im->round_ev, sizeof(hipEvent_t) * (size_t)need);
  if (!ev) { pg_set_error("pg_exec: out of host memory"); return -1; }
  im->round_ev = ev;
  for (int i = im->n_round_ev; i < need; ++i) {
    hipError_t e = hipEventCreateWithFlags(&im->round_ev[i], hipEventDisableTiming);
    if (e != hipSuccess) {
      im->n_round_ev = i;
      pg_set_error("pg_exec: hipEventCreate: %s", hipGetErrorString(e));
      return -1;
    }
  }
  im->n_round_ev = need;
  return 0;
}

/* The reduce launches of one batch: up to PG_RED_RANGES ranges per
 * pgk_reduce_ranges call. */
#define PG_RED_RANGES 8
struct red_batch {
  void *out[PG_RED_RANGES];
  const void *a[PG_RED_RANGES], *b[PG_RED_RANGES];
  size_t n[PG_RED_RANGES];
  int k;
};

/* Next start/stop event pair for a stamped launch (PG_KERNEL_TIMING=1). */
int pg_kt_pair(struct pg_impl *im, void **t0, void **t1) {
  if (2 * (im->kt_used + 1) > im->n_kt_ev) {
    int cap = im->n_kt_ev ? 2 * im->n_kt_ev : 64;
    hipEvent_t *ev = (hipEvent_t *)realloc(im->kt_ev, sizeof(hipEvent_t) * (size_t)cap);
    if (!ev) { pg_set_error("pg_exec: out of host memory"); return -1; }
    im->kt_ev = ev;
    for (int i = im->n_kt_ev; i < cap; ++i) {
      hipError_t e = hipEventCreate(&im->kt_ev[i]);
      if (e != hipSuccess) {
        if (i & 1) hipEventDestroy(im->kt_ev[i - 1]);     /* keep whole pairs */
        im->n_kt_ev = i & ~1;
        pg_set_error("pg_exec: hipEventCreate: %s", hipGetErrorString(e));
        return -1;
      }
    }
    im->n_kt_ev = cap;
  }
  *t0 = (void *)im->kt_ev[2 * im->kt_used];
  *t1 = (void *)im->kt_ev[2 * im->kt_used + 1];
  im->kt_used++;
  return 0;
}

static int red_flush(struct pg_impl *im, struct red_batch *rb, int dt, int op, hipStream_t rs) {
  if (!rb->k) return 0;
  void *t0 = NULL, *t1 = NULL;
  if (im->kt_on && pg_kt_pair(im, &t0, &t1)) return -1;
  if (pgk_reduce_ranges(rb->out, rb->a, rb->b, rb->n, rb->k, dt, op, (void *)rs, t0, t1)) {
    pg_set_error("pg_exec: %s", pgk_last_error());
    return -1;
  }
  im->stats.reduce_launches += 1;
  if (im->kt_on)
    for (int j = 0; j < rb->k; ++j) im->stats.red_kernel_bytes += (int64_t)(3 * rb->n[j] * pg_elem_size(dt));
  rb->k = 0;
  return 0;
}

/* Reduce every pending step: the comm stream's position (behind the last
 * group that carried any of them) gates the reduce stream, pg_plan_coalesce
 * turns the steps into ranges contiguous in both operands -- the segments of
 * one ring over consecutive groups are neighbours in the same block -- and all
 * ranges go out in one pgk_reduce_ranges launch (eight ranges at most per
 * launch).  Then every step's red_ev is recorded behind it. */
static int reduce_pending(struct pg_impl *im, const struct pg_step *st, int npend, int nb, void *const bufs[5],
                          int dt, int op) {
  if (!npend) return 0;
  hipStream_t rs = im->red;
  hipEvent_t rev = im->recv_ev[nb % PG_RECV_EVENTS];
  PG_CHECK_HIP(hipEventRecord(rev, im->comm));
  PG_CHECK_HIP(hipStreamWaitEvent(rs, rev, 0));
  if (npend > im->ranges_cap) {
    struct pg_red_range *rr = (struct pg_red_range *)realloc(im->ranges, sizeof(*rr) * (size_t)npend);
    if (!rr) { pg_set_error("pg_exec: out of host memory"); return -1; }
    im->ranges = rr;
    im->ranges_cap = npend;
  }
  const int nr = pg_plan_coalesce(st, im->pend, npend, pg_elem_size(dt), im->ranges, im->ranges_cap);
  if (nr < 0) { pg_set_error("pg_exec: could not list the pending reduces"); return -1; }
  struct red_batch rb;
  rb.k = 0;
  for (int u = 0; u < nr; ++u) {
    const struct pg_red_range *g = &im->ranges[u];
    char *dst = at(bufs, g->dst_buf, g->dst_off);
    const char *src = at(bufs, g->src_buf, g->src_off);
    /* the arrival is the left operand: dst = dst op src, or with rev (the
     * arrival sits in src) dst = src op dst */
    rb.out[rb.k] = dst;
    rb.a[rb.k] = g->rev ? src : dst;
    rb.b[rb.k] = g->rev ? dst : src;
    rb.n[rb.k] = (size_t)g->elems;
    im->stats.reduce_elems += g->elems;
    if (++rb.k == PG_RED_RANGES && red_flush(im, &rb, dt, op, rs)) return -1;
  }
  if (red_flush(im, &rb, dt, op, rs)) return -1;
  for (int u = 0; u < npend; ++u) PG_CHECK_HIP(hipEventRecord(im->red_ev[st[im->pend[u]].seg], rs));
  return 0;
}

int pg_exec_plan(struct pg_impl *im, const struct pg_step *st, int n,
                 void *const bufs[5], int dt, int op, pg_round_hook hook, void *hook_ctx) {
  if (n <= 0) {
    im->last_round_rec = -1;
    return hook ? hook(im, hook_ctx, pg_world_of(im) - 1) : 0;
  }
  const struct pg *pg = im->pg;
  const int W = pg->world_size;

  int max_seg = 0;
  for (int i = 0; i < n; ++i) if (st[i].seg > max_seg) max_seg = st[i].seg;
  if (ensure_red_events(im, max_seg + 1)) return -1;
  if (n > im->pend_cap) {
    int *pd = (int *)realloc(im->pend, sizeof(int) * (size_t)n);
    if (!pd) { pg_set_error("pg_exec: out of host memory"); return -1; }
    im->pend = pd;
    im->pend_cap = n;
  }

  int rounds = st[n - 1].round + 1;
  if (hook && ensure_round_events(im, rounds)) return -1;
  im->last_round_rec = -1;
  const int64_t es = pg_elem_size(dt);
  int i = 0, nb = 0, cur_round = -1, npend = 0;
  int64_t pend_bytes = 0;
  while (i < n) {
    int b = st[i].batch, j = i;
    while (j < n && st[j].batch == b) ++j;          /* steps [i, j) = one batch */
    if (hook && st[i].round != cur_round) {
      if (cur_round >= 0) {
        PG_CHECK_HIP(hipEventRecord(im->round_ev[cur_round], im->comm));
        im->last_round_rec = cur_round;
      }
      cur_round = st[i].round;
      if (hook(im, hook_ctx, cur_round)) return -1;
    }

    /* forwarded partials must be reduced before they go on the wire */
    for (int s = i; s < j; ++s)
      if (st[s].send_bytes && st[s].send_wait)
        PG_CHECK_HIP(hipStreamWaitEvent(im->comm, im->red_ev[st[s].seg], 0));

    if (im->ops->group_start(im)) return -1;
    for (int s = i; s < j; ++s) {
      const int to = ((pg->rank + st[s].send_peer) % W + W) % W;
      const int from = ((pg->rank + st[s].recv_peer) % W + W) % W;
      if (st[s].send_bytes &&
          im->ops->send(im, at(bufs, st[s].send_buf, st[s].send_off), (size_t)st[s].send_bytes,
                        to, im->comm))
        return -1;
      if (st[s].recv_bytes &&
          im->ops->recv(im, at(bufs, st[s].recv_buf, st[s].recv_off), (size_t)st[s].recv_bytes,
                        from, im->comm))
        return -1;
      im->stats.bytes_sent += st[s].send_bytes;
      im->stats.bytes_recv += st[s].recv_bytes;
    }
    if (im->ops->group_end(im, im->comm)) return -1;

    for (int s = i; s < j; ++s)
      if (st[s].red_elems > 0) {
        im->pend[npend++] = s;
        pend_bytes += st[s].red_elems * es;
      }
    /* reduce now: enough is pending, or the round (or the plan) ends here --
     * the next round forwards what this one reduced */
    if (npend && ((size_t)pend_bytes >= im->red_bytes || j == n || st[j].round != st[i].round)) {
      if (reduce_pending(im, st, npend, nb, bufs, dt, op)) return -1;
      npend = 0;
      pend_bytes = 0;
    }
    ++nb;
    i = j;
  }
  if (hook) {
    PG_CHECK_HIP(hipEventRecord(im->round_ev[cur_round], im->comm));
    im->last_round_rec = cur_round;
    if (hook(im, hook_ctx, pg->world_size - 1)) return -1;   /* after the last round */
  }
  /* join: the comm stream observes the last reduce */
  PG_CHECK_HIP(hipEventRecord(im->join_ev, im->red));
  PG_CHECK_HIP(hipStreamWaitEvent(im->comm, im->join_ev, 0));
  return 0;
}
