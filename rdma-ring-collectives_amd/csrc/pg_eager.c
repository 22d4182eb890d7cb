/*
 * pg_eager.c -- one-shot exchange for small messages (the eager path).
 *
 * The reference declares an eager threshold (eager_max, src/constants.h:75,
 * pg.h:44) but its ring always runs W-1 rounds (src/pg.c:277-289,
 * :309-319).  A 4 KiB call is pure latency: W-1 transport groups and W-1
 * kernel launches, each a few microseconds of fixed cost.  At or below
 * eager_max bytes per rank the collectives here use ONE transport group in
 * which every rank sends each peer what that peer needs, and ONE launch:
 *
 *   reduce-scatter  rank r receives block r of every peer's input and folds
 *                   them in ring order, every ring part in one launch
 *                   (pgk_fold_blocks; pgk_reduce_multi for one ring);
 *   all-gather      every rank sends its slot to every peer;
 *   all-reduce      every rank sends its whole input to every peer and
 *                   pgk_fold_blocks folds each block in its ring order.
 *
 * Fold order = the ring's (part g of block b: x[b+d] op x[b+2d] op ... op x[b]
 * with d = pg_ring_offset(W, rings, g): +1, -1, +3, -3; see
 * pg_plan.c and include/pg_ext.h), so results are bit-identical
 * to the ring path for int32 and double alike.  Used by the point-to-point transports (RCCL,
 * in-process threads) for W <= 16; xgmi has its own direct-read one-shot.
 * PG_EAGER_ONESHOT=0 turns it off.
 */
#include <stdlib.h>
#include <string.h>

#include "pg_impl.h"

#define EAGER_MAX_WORLD 16

int pg_eager_applies(const struct pg *pg, int count, int dt) {
  const struct pg_impl *im = (const struct pg_impl *)pg->impl;
  size_t bytes = (size_t)count * pg_elem_size(dt);
  return im->eager_oneshot && pg->world_size > 1 && pg->world_size <= EAGER_MAX_WORLD && count > 0 &&
         bytes <= pg->eager_max;
}

/* Device image of a (possibly host) input of `bytes`. */
static int device_input(struct pg_impl *im, const void *buf, int dev, size_t bytes, const void **out) {
  if (dev) { *out = buf; return 0; }
  if (pg_ensure(&im->dsrc, &im->dsrc_cap, bytes)) return -1;
  if (pg_timed_copy(im->dsrc, buf, bytes, &im->stats.h2d_us)) return -1;
  *out = im->dsrc;
  return 0;
}

static int finish(struct pg_impl *im) {
  PG_CHECK_HIP(hipEventRecord(im->t1, im->comm));
  if (pg_stream_wait(im->comm)) return -1;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, im->t0, im->t1) == hipSuccess) im->stats.ring_us += (double)ms * 1e3;
  return 0;
}

int pg_eager_reduce_scatter(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const int W = pg->world_size, r = pg->rank;
  size_t es = pg_elem_size(dt), bytes = (size_t)count * es, boff, blen;
  pg_block_range(count, W, r, &boff, &blen);
  int sd = pg_is_device_ptr(sendbuf), rd = pg_is_device_ptr(recvbuf);
  if ((sd || rd) && pg_wait_producers(im, 0)) return -1;
  const char *src;
  if (device_input(im, sendbuf, sd, bytes, (const void **)&src)) return -1;
  /* gather area: block r of every rank, one slot per rank; the output goes
   * behind it when recvbuf cannot take it directly */
  size_t slot = blen * es;
  if (pg_ensure(&im->ebuf, &im->ebuf_cap, slot * (size_t)(W + 1))) return -1;
  char *gat = (char *)im->ebuf;
  char *out = (char *)recvbuf;
  if (!rd || pg_ranges_overlap(recvbuf, slot, src, bytes)) out = gat + slot * (size_t)W;

  PG_CHECK_HIP(hipEventRecord(im->t0, im->comm));
  if (im->ops->group_start(im)) return -1;
  for (int q = 0; q < W; ++q) {
    if (q == r) continue;
    size_t qo, ql;
    pg_block_range(count, W, q, &qo, &ql);
    if (ql && im->ops->send(im, src + qo * es, ql * es, q, im->comm)) return -1;
    if (blen && im->ops->recv(im, gat + (size_t)q * slot, slot, q, im->comm)) return -1;
    im->stats.bytes_sent += (int64_t)(ql * es);
    im->stats.bytes_recv += (int64_t)slot;
  }
  if (im->ops->group_end(im, im->comm)) return -1;
  if (blen && im->rings > 1) {
    /* every ring part of block r in one launch: pgk_fold_blocks folds block 0
     * of its sources part by part in ring order, and source j is rank r+j's
     * block r (tools/lab/fold_launch_probe.py: 3.8 vs 6.6 us at these sizes) */
    const void *srcs[EAGER_MAX_WORLD];
    for (int j = 0; j < W; ++j) {
      int q = (r + j) % W;
      srcs[j] = q == r ? src + boff * es : gat + (size_t)q * slot;
    }
    if (pgk_fold_blocks(out, srcs, W, blen, blen, im->rings, dt, op, (void *)im->comm)) {
      pg_set_error("%s", pgk_last_error());
      return -1;
    }
    im->stats.reduce_launches++;
    im->stats.reduce_elems += (int64_t)(blen * (size_t)(W - 1));
  } else if (blen) {                                 /* one ring: the vector kernel */
    const void *srcs[EAGER_MAX_WORLD];
    for (int j = 0; j < W; ++j) {
      int q = (r + 1 + j) % W;                                          /* the ring order */
      srcs[j] = q == r ? src + boff * es : gat + (size_t)q * slot;
    }
    if (pgk_reduce_multi(out, srcs, W, blen, dt, op, (void *)im->comm)) {
      pg_set_error("%s", pgk_last_error());
      return -1;
    }
    im->stats.reduce_launches++;
    im->stats.reduce_elems += (int64_t)(blen * (size_t)(W - 1));
  }
  if (finish(im)) return -1;
  if (out != (char *)recvbuf && pg_timed_copy(recvbuf, out, slot, &im->stats.d2h_us)) return -1;
  return 0;
}

int pg_eager_all_gather(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const int W = pg->world_size, r = pg->rank;
  size_t slot = (size_t)count * pg_elem_size(dt), total = slot * (size_t)W;
  int rd = pg_is_device_ptr(recvbuf), sd = sendbuf && pg_is_device_ptr(sendbuf);
  if ((rd || sd) && pg_wait_producers(im, 0)) return -1;
  char *full = (char *)recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, total)) return -1;
    full = (char *)im->dout;
  }
  char *own = full + (size_t)r * slot;
  const void *mine = sendbuf ? sendbuf : (const void *)((char *)recvbuf + (size_t)r * slot);
  if ((char *)mine != own && pg_timed_copy(own, mine, slot, sd || rd ? &im->stats.copy_us : &im->stats.h2d_us))
    return -1;

  PG_CHECK_HIP(hipEventRecord(im->t0, im->comm));
  if (im->ops->group_start(im)) return -1;
  for (int q = 0; q < W; ++q) {
    if (q == r) continue;
    if (im->ops->send(im, own, slot, q, im->comm)) return -1;
    if (im->ops->recv(im, full + (size_t)q * slot, slot, q, im->comm)) return -1;
    im->stats.bytes_sent += (int64_t)slot;
    im->stats.bytes_recv += (int64_t)slot;
  }
  if (im->ops->group_end(im, im->comm)) return -1;
  if (finish(im)) return -1;
  if (!rd && pg_timed_copy(recvbuf, full, total, &im->stats.d2h_us)) return -1;
  return 0;
}

int pg_eager_all_reduce(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const int W = pg->world_size, r = pg->rank;
  size_t es = pg_elem_size(dt), bytes = (size_t)count * es;
  int sd = pg_is_device_ptr(sendbuf), rd = pg_is_device_ptr(recvbuf);
  if ((sd || rd) && pg_wait_producers(im, 0)) return -1;
  const char *src;
  if (device_input(im, sendbuf, sd, bytes, (const void **)&src)) return -1;
  /* every peer's whole input, plus an output slot when recvbuf is host
   * memory or is the input itself (the fold reads all of it) */
  if (pg_ensure(&im->ebuf, &im->ebuf_cap, bytes * (size_t)(W + 1))) return -1;
  char *gat = (char *)im->ebuf;
  char *out = (char *)recvbuf;
  if (!rd || pg_ranges_overlap(recvbuf, bytes, src, bytes)) out = gat + bytes * (size_t)W;

  PG_CHECK_HIP(hipEventRecord(im->t0, im->comm));
  if (im->ops->group_start(im)) return -1;
  for (int q = 0; q < W; ++q) {
    if (q == r) continue;
    if (im->ops->send(im, src, bytes, q, im->comm)) return -1;
    if (im->ops->recv(im, gat + (size_t)q * bytes, bytes, q, im->comm)) return -1;
    im->stats.bytes_sent += (int64_t)bytes;
    im->stats.bytes_recv += (int64_t)bytes;
  }
  if (im->ops->group_end(im, im->comm)) return -1;
  const void *srcs[EAGER_MAX_WORLD];
  for (int q = 0; q < W; ++q) srcs[q] = q == r ? (const void *)src : (const void *)(gat + (size_t)q * bytes);
  size_t blk = ((size_t)count + (size_t)W - 1) / (size_t)W;
  if (pgk_fold_blocks(out, srcs, W, (size_t)count, blk, im->rings, dt, op, (void *)im->comm)) {
    pg_set_error("%s", pgk_last_error());
    return -1;
  }
  im->stats.reduce_launches++;
  im->stats.reduce_elems += (int64_t)count * (W - 1);
  if (finish(im)) return -1;
  if (out != (char *)recvbuf && pg_timed_copy(recvbuf, out, bytes, rd ? &im->stats.copy_us : &im->stats.d2h_us))
    return -1;
  return 0;
}
