/*
 * pg_direct.c -- PG_ALGO=direct: the point-to-point collectives as one-hop
 * exchanges over every link at once, for a fully connected node.
 *
 * The reference's ring (README.md:68-71, mocked at src/pg.c:277-289) moves
 * each block W-1 hops, one link direction per ring, and reduces it once per
 * hop.  On one MI355X node every GPU has its own xGMI link to each of its 7
 * peers, so the same reduce-scatter can send block q of this rank's input
 * straight to rank q -- all W-1 links busy, every byte crossing one link once
 * -- and fold the W contributions of block r in ONE multi-source launch per
 * segment batch.  The fold keeps each ring part's order
 *     part g of block r:  x[r+d] op x[r+2d] op ... op x[r]     (d = step of ring g)
 * so the result is bit-identical to the ring (and to the oracle) for the same
 * PG_RINGS, doubles included.  HBM traffic drops too: (W+1)·B·es for the fold
 * instead of 3·(W-1)·B·es for W-1 ring reduces.
 *
 * Pipelining: block r is cut into the ring's parts, each part into
 * chunk_bytes segments; one transport group per `inflight` segments carries
 * that batch from every peer (and the matching segments of every peer's block
 * to it), and the reduce stream folds a batch as soon as its group has landed
 * while the next batch is on the wire.  Every block uses the segment layout of
 * the full block (empty segments in a short last block), so every rank builds
 * the same groups and per-peer send/receive order matches.  The received
 * segments go to a gather area of W block-sized slots, never reused inside a
 * call, so the comm stream never waits for a fold.
 *
 * The schedule is data: pg_plan_direct_reduce_scatter (pg_plan.c) lists the
 * transfer and fold steps, so tests/test_plan_gloo.py runs the same plan over
 * gloo processes without a GPU.
 *
 * All-gather and the all-reduce's gather half: one group, every rank sending
 * its block (slot) to every peer.
 *
 * Default for the point-to-point transports when every rank is on one node and
 * W <= 16 (PG_ALGO unset); PG_ALGO=ring keeps the W-1 round ring.
 */
#include <stdlib.h>
#include <string.h>

#include "pg_impl.h"

#define DIRECT_MAX_WORLD 16

int pg_direct_applies(const struct pg *pg, int count) {
  const struct pg_impl *im = (const struct pg_impl *)pg->impl;
  return im->algo == PG_ALGO_DIRECT && pg->world_size > 1 && pg->world_size <= DIRECT_MAX_WORLD && count > 0;
}

/* The comm stream observes the last fold. */
static int join_folds(struct pg_impl *im) {
  PG_CHECK_HIP(hipEventRecord(im->join_ev, im->red));
  PG_CHECK_HIP(hipStreamWaitEvent(im->comm, im->join_ev, 0));
  return 0;
}

/* The gather area holds W full blocks -- as much as the whole input, where the
 * ring stages about two blocks.  When it has to grow and some rank cannot
 * allocate it, every rank takes the ring for this call instead (the ranks agree
 * over the bootstrap star; growth happens in the same call on every rank,
 * because every rank sees the same counts).  Returns 1: run the direct
 * exchange, 0: use the ring (agreed by all ranks), -1: failed.  Test hook
 * PG_TEST_FAIL_STAGE_ALLOC=r: rank r's allocation fails. */
int pg_direct_prepare(struct pg *pg, int count, int dt) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const size_t W = (size_t)pg->world_size, full = ((size_t)count + W - 1) / W;
  const size_t need = W * full * pg_elem_size(dt);
  if (im->ebuf && need <= im->ebuf_cap) return 1;
  int ok = pg_ensure(&im->ebuf, &im->ebuf_cap, need) == 0;
  const char *h = getenv("PG_TEST_FAIL_STAGE_ALLOC");
  if (h && *h && atoi(h) == pg->rank) ok = 0;
  if (!ok) (void)hipGetLastError();
  if (!im->boot_fds) return ok ? 1 : -1;          /* in-process ranks: nothing to agree over */
  char mine = (char)ok, all[DIRECT_MAX_WORLD];
  if (pg_boot_allgather(pg, im->boot_fds, &mine, all, 1)) return -1;
  for (int q = 0; q < pg->world_size; ++q) ok &= all[q] != 0;
  if (ok) return 1;
  /* every rank drops the area, so that all of them see "has to grow" alike next time */
  if (im->ebuf) { hipFree(im->ebuf); im->ebuf = NULL; }
  im->ebuf_cap = 0;
  pg_trace(pg, "direct: %zu bytes of gather area not available on every rank; falling back to the ring", need);
  return 0;
}

static int direct_finish(struct pg_impl *im) {
  if (join_folds(im)) return -1;
  PG_CHECK_HIP(hipEventRecord(im->t1, im->comm));
  if (pg_stream_wait(im->comm) || pg_stream_wait(im->red)) return -1;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, im->t0, im->t1) == hipSuccess) im->stats.ring_us += (double)ms * 1e3;
  pg_kt_collect(im);
  return 0;
}

/* Reduce-scatter core: block `rank` of the reduction of every rank's `src`
 * (device, count elements) into `out` (device, the block's length), running
 * the plan of pg_plan_direct_reduce_scatter (pg_plan.c; include/pg_ext.h). */
static int direct_rs_core(struct pg *pg, const char *src, char *out, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const int W = pg->world_size, r = pg->rank;
  const size_t es = pg_elem_size(dt), full = ((size_t)count + (size_t)W - 1) / (size_t)W;
  size_t boff, blen;
  pg_block_range(count, W, r, &boff, &blen);
  if (pg_ensure(&im->ebuf, &im->ebuf_cap, (size_t)W * full * es)) return -1;
  char *gat = (char *)im->ebuf;                      /* STAGE0: slot q = rank q's copy of block r */
  int n = pg_plan_direct_reduce_scatter(r, W, count, dt, pg->chunk_bytes, pg->inflight, im->rings, NULL, 0);
  if (n < 0) { pg_set_error("direct: bad plan arguments, or chunk_bytes too small for this count"); return -1; }
  if (n > im->steps_cap) {
    struct pg_step *st = (struct pg_step *)realloc(im->steps, sizeof(*st) * (size_t)n);
    if (!st) { pg_set_error("direct: out of host memory"); return -1; }
    im->steps = st;
    im->steps_cap = n;
  }
  pg_plan_direct_reduce_scatter(r, W, count, dt, pg->chunk_bytes, pg->inflight, im->rings, im->steps, n);
  const struct pg_step *st = im->steps;
  int dsteps[PG_MAX_RINGS];
  for (int g = 0; g < im->rings; ++g) dsteps[g] = pg_ring_offset(W, im->rings, g);

  PG_CHECK_HIP(hipEventRecord(im->t0, im->comm));
  /* Transfers go out batch by batch; the folds of the landed batches wait until
   * red_bytes per source are pending (PG_REDUCE_BYTES) or the plan ends, and
   * then each ring's pending segments -- neighbours in every slot -- fold in one
   * launch.  The gather slots are never reused inside a call, so nothing waits
   * for a fold. */
  int64_t pend_bytes = 0;
  int pend_from = 0;                                    /* plan steps [pend_from, j) hold the pending folds */
  int i = 0, nb = 0;
  while (i < n) {
    int j = i;
    while (j < n && st[j].batch == st[i].batch) ++j;   /* steps [i, j) = one batch */
    if (im->ops->group_start(im)) return -1;
    for (int t = i; t < j; ++t) {
      const int q = (r + st[t].send_peer) % W;           /* send_peer == recv_peer in direct plans */
      if (st[t].send_bytes &&
          im->ops->send(im, src + st[t].send_off, (size_t)st[t].send_bytes, q, im->comm))
        return -1;
      if (st[t].recv_bytes &&
          im->ops->recv(im, gat + st[t].recv_off, (size_t)st[t].recv_bytes, (r + st[t].recv_peer) % W, im->comm))
        return -1;
      im->stats.bytes_sent += st[t].send_bytes;
      im->stats.bytes_recv += st[t].recv_bytes;
      if (st[t].red_fold) pend_bytes += st[t].red_elems * (int64_t)es;
    }
    if (im->ops->group_end(im, im->comm)) return -1;
    if (pend_bytes && ((size_t)pend_bytes >= im->red_bytes || j == n)) {
      hipEvent_t rev = im->recv_ev[nb++ % PG_RECV_EVENTS];
      PG_CHECK_HIP(hipEventRecord(rev, im->comm));
      PG_CHECK_HIP(hipStreamWaitEvent(im->red, rev, 0));
      for (int g = 0; g < im->rings; ++g) {
        int t = pend_from;
        while (t < j) {
          if (!st[t].red_fold || st[t].seg != g) { ++t; continue; }
          /* a run of ring g's fold steps, contiguous in the block */
          int64_t len = st[t].red_elems;
          int u = t + 1;
          for (; u < j; ++u) {
            if (!st[u].red_fold || st[u].seg != g) continue;
            if (st[u].red_src_off != st[t].red_src_off + len * (int64_t)es ||
                st[u].red_dst_off != st[t].red_dst_off + len * (int64_t)es)
              break;
            len += st[u].red_elems;
          }
          if (!len) { t = u; continue; }                 /* empty segments of a short last block */
          const size_t o = (size_t)st[t].red_src_off / es;
          const void *srcs[DIRECT_MAX_WORLD];
          for (int k = 0; k < W; ++k) {
            const int q = ((r + (k + 1) * dsteps[g]) % W + W) % W;   /* k = W-1: q = r */
            srcs[k] = q == r ? (const void *)(src + (boff + o) * es) : (const void *)(gat + ((size_t)q * full + o) * es);
          }
          void *t0 = NULL, *t1 = NULL;
          if (im->kt_on) {
            if (pg_kt_pair(im, &t0, &t1)) return -1;
            im->stats.red_kernel_bytes += (int64_t)((size_t)(W + 1) * (size_t)len * es);
          }
          /* every flush but the last runs beside the next batches' transport kernels */
          if (pgk_fold_timed(out + st[t].red_dst_off, srcs, W, (size_t)len, dt, op, j == n ? 0u : PGK_FOLD_SHARED_GPU,
                             (void *)im->red, t0, t1)) {
            pg_set_error("direct: %s", pgk_last_error());
            return -1;
          }
          im->stats.reduce_launches++;
          im->stats.reduce_elems += len * (W - 1);
          t = u;
        }
      }
      pend_bytes = 0;
      pend_from = j;
    }
    i = j;
  }
  return 0;
}

/* One group: this rank's block to every peer, every peer's block into `full`.
 * uniform: blocks of `count` elements (all-gather); else the reduce-scatter
 * partition of `count` (the all-reduce's second half). */
static int direct_gather_core(struct pg *pg, char *full, int count, int uniform, int dt) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const int W = pg->world_size, r = pg->rank;
  const size_t es = pg_elem_size(dt);
  size_t roff, rlen;
  if (uniform) { roff = (size_t)r * (size_t)count; rlen = (size_t)count; }
  else pg_block_range(count, W, r, &roff, &rlen);
  if (im->ops->group_start(im)) return -1;
  for (int k = 1; k < W; ++k) {
    const int to = (r + k) % W, from = ((r - k) % W + W) % W;
    size_t foff, flen;
    if (uniform) { foff = (size_t)from * (size_t)count; flen = (size_t)count; }
    else pg_block_range(count, W, from, &foff, &flen);
    if (rlen && im->ops->send(im, full + roff * es, rlen * es, to, im->comm)) return -1;
    if (flen && im->ops->recv(im, full + foff * es, flen * es, from, im->comm)) return -1;
    im->stats.bytes_sent += (int64_t)(rlen * es);
    im->stats.bytes_recv += (int64_t)(flen * es);
  }
  return im->ops->group_end(im, im->comm);
}

/* Device image of a (possibly host) input. */
static int device_src(struct pg_impl *im, const void *buf, int dev, size_t bytes, const char **out) {
  if (dev) { *out = (const char *)buf; return 0; }
  if (pg_ensure(&im->dsrc, &im->dsrc_cap, bytes)) return -1;
  if (pg_timed_copy(im->dsrc, buf, bytes, &im->stats.h2d_us)) return -1;
  *out = (const char *)im->dsrc;
  return 0;
}

int pg_direct_reduce_scatter(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const size_t es = pg_elem_size(dt), bytes = (size_t)count * es;
  size_t boff, blen;
  pg_block_range(count, pg->world_size, pg->rank, &boff, &blen);
  int sd = pg_is_device_ptr(sendbuf), rd = pg_is_device_ptr(recvbuf);
  if ((sd || rd) && pg_wait_producers(im, 0)) return -1;
  const char *src;
  if (device_src(im, sendbuf, sd, bytes, &src)) return -1;
  char *out = (char *)recvbuf;
  int post_copy = 0;
  if (!rd || pg_ranges_overlap(recvbuf, blen * es, src, bytes)) {
    if (pg_ensure(&im->dout, &im->dout_cap, blen * es)) return -1;
    out = (char *)im->dout;
    post_copy = 1;
  }
  if (direct_rs_core(pg, src, out, count, dt, op) || direct_finish(im)) return -1;
  if (post_copy && blen && pg_timed_copy(recvbuf, out, blen * es, &im->stats.d2h_us)) return -1;
  return 0;
}

int pg_direct_all_gather(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const size_t slot = (size_t)count * pg_elem_size(dt), total = slot * (size_t)pg->world_size;
  int rd = pg_is_device_ptr(recvbuf), sd = sendbuf && pg_is_device_ptr(sendbuf);
  if ((rd || sd) && pg_wait_producers(im, 0)) return -1;
  char *full = (char *)recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, total)) return -1;
    full = (char *)im->dout;
  }
  char *own = full + (size_t)pg->rank * slot;
  const void *mine = sendbuf ? sendbuf : (const void *)((char *)recvbuf + (size_t)pg->rank * slot);
  if ((const char *)mine != own && pg_timed_copy(own, mine, slot, sd || rd ? &im->stats.copy_us : &im->stats.h2d_us))
    return -1;
  PG_CHECK_HIP(hipEventRecord(im->t0, im->comm));
  if (direct_gather_core(pg, full, count, 1, dt) || direct_finish(im)) return -1;
  if (!rd && pg_timed_copy(recvbuf, full, total, &im->stats.d2h_us)) return -1;
  return 0;
}

int pg_direct_all_reduce(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const size_t es = pg_elem_size(dt), bytes = (size_t)count * es;
  size_t boff, blen;
  pg_block_range(count, pg->world_size, pg->rank, &boff, &blen);
  int sd = pg_is_device_ptr(sendbuf), rd = pg_is_device_ptr(recvbuf);
  if ((sd || rd) && pg_wait_producers(im, 0)) return -1;
  char *work = (char *)recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, bytes)) return -1;
    work = (char *)im->dout;
  }
  if (sendbuf != (void *)work && pg_timed_copy(work, sendbuf, bytes, sd ? &im->stats.copy_us : &im->stats.h2d_us))
    return -1;
  /* block `rank` is folded in place: the fold reads this rank's own copy of the
   * block element by element before writing it, and the sends read the other
   * blocks only */
  if (direct_rs_core(pg, work, work + boff * es, count, dt, op)) return -1;
  if (join_folds(im)) return -1;                                /* the gather sends the folded block */
  if (direct_gather_core(pg, work, count, 0, dt) || direct_finish(im)) return -1;
  if (!rd && pg_timed_copy(recvbuf, work, bytes, &im->stats.d2h_us)) return -1;
  return 0;
}
