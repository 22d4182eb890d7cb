/*
 * pg_plan.c -- the ring schedule as data.  Pure C: no HIP, no transport.
 *
 * The reference computes its schedule inline in the collective loops
 * (src/pg.c:274-289 reduce-scatter, :309-318 all-gather) from four helpers:
 * elem_size (:109-115), chunk_elems_from_bytes (:118-123), chunk_offsets
 * (:126-138) and rs_send/recv_chunk_index (:141-148).  Here the same index
 * arithmetic produces an explicit list of steps that pg_exec.c executes, so
 * the schedule can be checked without a GPU (tests/test_plan_gloo.py runs it
 * over two gloo processes).
 *
 * Differences from the reference mock, all deliberate:
 *   - the ring partition unit is the block ceil(count/W), not chunk_bytes;
 *     chunk_bytes is the pipelining segment inside a block (README.md:17,75);
 *   - the index functions are evaluated at rank-1 so rank r ends with block r
 *     (pg.h:127-139 "each rank receives an equal-sized chunk");
 *   - each round both sends and receives for real: send length and receive
 *     length are those of their own blocks (the mock used recv_len for both,
 *     src/pg.c:282-287);
 *   - with rings = 2 (default) the second half of every block runs the mirror
 *     schedule in the other direction, so both directions of each link carry
 *     data (a bidirectional ring); rings = 3, 4 add rings of
 *     step +3 / -3 (world permitting: pg_ring_offset), each over its own pair
 *     of xGMI links (multi-ring); the reference's README describes one
 *     ring (README.md:68-71).
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pg.h"
#include "pg_ext.h"

#define PG_MAX_PLAN_STEPS (1 << 28)

static size_t plan_elem_size(int dt) {
  return dt == DT_INT32 ? 4 : dt == DT_DOUBLE ? 8 : 0;
}

static int ring_mod(int x, int w) { return ((x % w) + w) % w; }

int pg_block_range(int count, int world, int block, size_t *off, size_t *len) {
  if (count < 0 || world < 1 || block < 0 || block >= world || !off || !len) return -1;
  size_t n = (size_t)count;
  size_t be = (n + (size_t)world - 1) / (size_t)world;
  if (be == 0) be = 1;
  size_t first = (size_t)block * be;
  if (first >= n) { *off = 0; *len = 0; return 0; }
  size_t last = first + be;
  if (last > n) last = n;
  *off = first;
  *len = last - first;
  return 0;
}

/* Segment length (elements) for a block of `len` elements. */
static size_t seg_elems_for(size_t len, size_t es, size_t chunk_bytes, size_t eager_max) {
  if (len * es <= eager_max) return len ? len : 1;   /* eager: one segment */
  size_t s = chunk_bytes / es;                         /* src/pg.c:118-123 */
  return s ? s : 1;
}

static size_t nsegs(size_t len, size_t seg) { return len ? (len + seg - 1) / seg : 0; }

int pg_block_part(size_t len, int rings, int part, size_t *off, size_t *plen) {
  if (rings < 1 || rings > PG_MAX_RINGS || part < 0 || part >= rings || !off || !plen) return -1;
  /* part g = [ceil(g*len/R), ceil((g+1)*len/R)): part 0 is the largest */
  size_t a = ((size_t)part * len + (size_t)rings - 1) / (size_t)rings;
  size_t b = ((size_t)(part + 1) * len + (size_t)rings - 1) / (size_t)rings;
  *off = a;
  *plen = b - a;
  return 0;
}

static int gcd_int(int a, int b) {
  while (b) { int t = a % b; a = b; b = t; }
  return a;
}

int pg_ring_offset(int world, int rings, int part) {
  if (world < 1 || rings < 1 || rings > PG_MAX_RINGS || part < 0 || part >= rings) return 0;
  /* +1 and -1 (the bidirectional pair, also at world 2 where they coincide),
   * then +3, -3, +5, -5, ... kept when coprime with world and not already
   * used mod world; when those run out the list repeats (more segment streams
   * over the same links) */
  int offs[PG_MAX_RINGS] = {1, -1}, m = 2;
  for (int c = 3; m < PG_MAX_RINGS && c < 2 * world; c += 2) {
    for (int sgn = 1; sgn >= -1 && m < PG_MAX_RINGS; sgn -= 2) {
      int d = sgn * c, rd = ring_mod(d, world);
      if (rd == 0 || gcd_int(rd, world) != 1) continue;
      int dup = 0;
      for (int i = 0; i < m; ++i) dup |= ring_mod(offs[i], world) == rd;
      if (!dup) offs[m++] = d;
    }
  }
  return offs[part % m];
}

static void put(struct pg_step *steps, int max_steps, int n, const struct pg_step *s) {
  if (steps && n < max_steps) steps[n] = *s;
}

/* One ring's view of round k: the blocks it sends and receives (this rank's
 * parts of them) and how they are cut into segments. */
struct ring_round {
  int d;                        /* ring offset: send to rank+d, receive from rank-d */
  size_t so, sl, to, tl;        /* sent / received block: offset, length    */
  size_t sp, spl, tp, tpl;      /* this ring's part of each: offset, length */
  size_t sseg, tseg, ns, nt;    /* segment lengths and counts               */
  size_t stage_base;            /* element offset of this ring in staging   */
  int seg_base;                 /* first event slot of this ring            */
};

int pg_plan_reduce_scatter(int rank, int world, int count, int datatype,
                           size_t chunk_bytes, size_t eager_max, int inflight, int rings,
                           int out_aliases_src, struct pg_step *steps, int max_steps) {
  size_t es = plan_elem_size(datatype);
  if (!es || world < 1 || rank < 0 || rank >= world || count < 0 || rings < 1 || rings > PG_MAX_RINGS) return -1;
  if (inflight < 1) inflight = 1;
  size_t bfull = ((size_t)count + (size_t)world - 1) / (size_t)world;
  size_t bh, bhl;
  pg_block_part(bfull, rings, 0, &bh, &bhl);         /* part 0 of a full block: the largest part */
  const size_t segs = nsegs(bhl, seg_elems_for(bhl, es, chunk_bytes, eager_max));
  /* a plan is at most (world-1) rounds x rings x segs steps: refuse segment
   * sizes so small that the step count (an int, like the event slots) would
   * not fit -- the caller raises chunk_bytes */
  if (segs > (size_t)PG_MAX_PLAN_STEPS / ((size_t)world * (size_t)rings)) return -1;
  int seg_stride = (int)segs;
  int n = 0, batch = -1;
  for (int k = 0; k + 1 < world; ++k) {
    const int last = (k == world - 2);
    struct ring_round rr[PG_MAX_RINGS];
    size_t nj = 0;
    for (int g = 0; g < rings; ++g) {
      struct ring_round *q = &rr[g];
      q->d = pg_ring_offset(world, rings, g);
      /* d = +1: rs_send/recv_chunk_index(k, rank-1); other rings: the same walk
       * with step d (d = -1: the mirror, counter-clockwise ring) */
      int sb = ring_mod(rank - (k + 1) * q->d, world);
      int tb = ring_mod(rank - (k + 2) * q->d, world);
      pg_block_range(count, world, sb, &q->so, &q->sl);
      pg_block_range(count, world, tb, &q->to, &q->tl);
      pg_block_part(q->sl, rings, g, &q->sp, &q->spl);
      pg_block_part(q->tl, rings, g, &q->tp, &q->tpl);
      q->sseg = seg_elems_for(q->spl, es, chunk_bytes, eager_max);
      q->tseg = seg_elems_for(q->tpl, es, chunk_bytes, eager_max);
      q->ns = nsegs(q->spl, q->sseg);
      q->nt = nsegs(q->tpl, q->tseg);
      q->stage_base = (size_t)g * ((bfull + (size_t)rings - 1) / (size_t)rings);   /* parts <= ceil(B/R) */
      q->seg_base = g * seg_stride;
      size_t m = q->ns > q->nt ? q->ns : q->nt;
      if (m > nj) nj = m;
    }
    /* batches: segment indices [j0, j0 + inflight) of every ring, clockwise first */
    for (size_t j0 = 0; j0 < nj; j0 += (size_t)inflight) {
      ++batch;
      size_t j1 = j0 + (size_t)inflight < nj ? j0 + (size_t)inflight : nj;
      for (int g = 0; g < rings; ++g) {
        const struct ring_round *q = &rr[g];
        for (size_t j = j0; j < j1; ++j) {
          if (j >= q->ns && j >= q->nt) continue;
          struct pg_step st;
          memset(&st, 0, sizeof(st));
          st.round = k;
          st.batch = batch;
          st.seg = q->seg_base + (int32_t)j;
          st.send_peer = q->d;
          st.recv_peer = -q->d;
          if (j < q->ns) {
            size_t e0 = j * q->sseg, len = q->spl - e0 < q->sseg ? q->spl - e0 : q->sseg;
            if (k == 0) { st.send_buf = PG_BUF_SRC; st.send_off = (int64_t)((q->so + q->sp + e0) * es); }
            else {
              st.send_buf = ((k - 1) & 1) ? PG_BUF_STAGE1 : PG_BUF_STAGE0;
              st.send_off = (int64_t)((q->stage_base + e0) * es);
              st.send_wait = 1;                 /* previous round reduced it */
            }
            st.send_bytes = (int64_t)(len * es);
          }
          if (j < q->nt) {
            size_t e0 = j * q->tseg, len = q->tpl - e0 < q->tseg ? q->tpl - e0 : q->tseg;
            int stage = (k & 1) ? PG_BUF_STAGE1 : PG_BUF_STAGE0;
            int64_t stage_off = (int64_t)((q->stage_base + e0) * es);
            if (last && !out_aliases_src) {
              st.recv_buf = PG_BUF_OUT;
              st.recv_off = (int64_t)((q->tp + e0) * es);
            } else {
              st.recv_buf = stage;
              st.recv_off = stage_off;
            }
            st.recv_bytes = (int64_t)(len * es);
            st.red_elems = (int64_t)len;
            if (last && out_aliases_src) {
              /* OUT is block `rank` of SRC: fold the arrival into it in place,
               * arrival op own like every other round (red_rev): + and * commute
               * except in the payload of NaN op NaN, which is the left operand's */
              st.red_dst_buf = PG_BUF_OUT; st.red_dst_off = (int64_t)((q->tp + e0) * es);
              st.red_src_buf = stage;      st.red_src_off = stage_off;
              st.red_rev = 1;
            } else {
              /* arrival op= this rank's own contribution to the block */
              st.red_dst_buf = st.recv_buf; st.red_dst_off = st.recv_off;
              st.red_src_buf = PG_BUF_SRC;  st.red_src_off = (int64_t)((q->to + q->tp + e0) * es);
            }
          }
          put(steps, max_steps, n, &st);
          ++n;
        }
      }
    }
  }
  if (steps && n > max_steps) return -1;
  return n;
}

/* ---- the direct exchange (PG_ALGO=direct, pg_direct.c) ------------------------
 * Block r is cut into the ring parts (pg_block_part) and each part into
 * chunk_elems segments, counted on the FULL block so that every block -- and
 * so every rank -- has the same flat segment list (a short last block has
 * empty segments).  Batch b = segments [b*inflight, (b+1)*inflight).  For each
 * batch: for every peer q = rank+k (k = 1 .. W-1), one transfer step per
 * segment sending that segment of block q from SRC to q and receiving that
 * segment of block `rank` from q into slot q of STAGE0 (slots of the full
 * block); then one fold step per run of the batch's segments inside one part
 * (red_fold = 1, seg = the part's ring). */
struct dseg {
  int rings, total;
  size_t seg;
  int count[PG_MAX_RINGS];
};

static void dseg_init(struct dseg *d, size_t full, int rings, size_t seg) {
  memset(d, 0, sizeof(*d));
  d->rings = rings;
  d->seg = seg ? seg : 1;
  for (int g = 0; g < rings; ++g) {
    size_t po, pl;
    pg_block_part(full, rings, g, &po, &pl);
    d->count[g] = (int)((pl + d->seg - 1) / d->seg);
    d->total += d->count[g];
  }
}

/* segment s of a block of `len` elements: part and [*off, *off + *n) in the block */
static void dseg_get(const struct dseg *d, int s, size_t len, int *part, size_t *off, size_t *n) {
  int g = 0;
  while (g + 1 < d->rings && s >= d->count[g]) s -= d->count[g++];
  size_t po, pl;
  pg_block_part(len, d->rings, g, &po, &pl);
  size_t a = (size_t)s * d->seg, b = a + d->seg;
  if (a > pl) a = pl;
  if (b > pl) b = pl;
  *part = g;
  *off = po + a;
  *n = b - a;
}

int pg_plan_direct_reduce_scatter(int rank, int world, int count, int datatype, size_t chunk_bytes, int inflight,
                                  int rings, struct pg_step *steps, int max_steps) {
  size_t es = plan_elem_size(datatype);
  if (!es || world < 1 || rank < 0 || rank >= world || count < 0 || rings < 1 || rings > PG_MAX_RINGS) return -1;
  if (inflight < 1) inflight = 1;
  const size_t full = ((size_t)count + (size_t)world - 1) / (size_t)world;
  size_t boff, blen;
  pg_block_range(count, world, rank, &boff, &blen);
  const size_t seg = chunk_bytes / es ? chunk_bytes / es : 1;
  /* at most ceil(full/seg) + rings segments, each a transfer step per peer
   * plus a fold: refuse what would overflow the int step count */
  if (full / seg + (size_t)rings > (size_t)PG_MAX_PLAN_STEPS / ((size_t)world + 1)) return -1;
  struct dseg d;
  dseg_init(&d, full, rings, seg);
  int n = 0, batch = 0;
  for (int s0 = 0; s0 < d.total; s0 += inflight, ++batch) {
    const int s1 = s0 + inflight < d.total ? s0 + inflight : d.total;
    for (int k = 1; k < world; ++k) {
      const int q = (rank + k) % world;
      size_t qoff, qlen;
      pg_block_range(count, world, q, &qoff, &qlen);
      for (int s = s0; s < s1; ++s) {
        int part;
        size_t so, sn, ro, rn;
        dseg_get(&d, s, qlen, &part, &so, &sn);
        dseg_get(&d, s, blen, &part, &ro, &rn);
        if (!sn && !rn) continue;
        struct pg_step st;
        memset(&st, 0, sizeof(st));
        st.batch = batch;
        st.seg = s;
        st.send_peer = k;
        st.recv_peer = k;
        if (sn) { st.send_buf = PG_BUF_SRC; st.send_off = (int64_t)((qoff + so) * es); st.send_bytes = (int64_t)(sn * es); }
        if (rn) {
          st.recv_buf = PG_BUF_STAGE0;
          st.recv_off = (int64_t)(((size_t)q * full + ro) * es);
          st.recv_bytes = (int64_t)(rn * es);
        }
        put(steps, max_steps, n, &st);
        ++n;
      }
    }
    int s = s0;
    while (s < s1) {
      int part, part2;
      size_t o, len, o2, len2;
      dseg_get(&d, s, blen, &part, &o, &len);
      int e = s + 1;
      while (e < s1) {
        dseg_get(&d, e, blen, &part2, &o2, &len2);
        if (part2 != part || o2 != o + len) break;
        len += len2;
        ++e;
      }
      if (len) {
        struct pg_step st;
        memset(&st, 0, sizeof(st));
        st.batch = batch;
        st.seg = part;
        st.red_fold = 1;
        st.red_dst_buf = PG_BUF_OUT;
        st.red_dst_off = (int64_t)(o * es);
        st.red_src_buf = PG_BUF_STAGE0;
        st.red_src_off = (int64_t)(o * es);
        st.red_elems = (int64_t)len;
        put(steps, max_steps, n, &st);
        ++n;
      }
      s = e;
    }
  }
  if (steps && n > max_steps) return -1;
  return n;
}

int pg_plan_all_gather(int rank, int world, int count, int datatype, int uniform, int rings,
                       struct pg_step *steps, int max_steps) {
  size_t es = plan_elem_size(datatype);
  if (!es || world < 1 || rank < 0 || rank >= world || count < 0 || rings < 1 || rings > PG_MAX_RINGS) return -1;
  int n = 0;
  for (int k = 0; k + 1 < world; ++k) {
    for (int g = 0; g < rings; ++g) {
      const int d = pg_ring_offset(world, rings, g);
      int sb = ring_mod(rank - k * d, world);          /* d = +1: src/pg.c:310 */
      int rb = ring_mod(rank - (k + 1) * d, world);    /* d = +1: src/pg.c:311 */
      size_t so, sl, ro, rl, sp, spl, rp, rpl;
      if (uniform) { so = (size_t)sb * (size_t)count; sl = (size_t)count; ro = (size_t)rb * (size_t)count; rl = (size_t)count; }
      else { pg_block_range(count, world, sb, &so, &sl); pg_block_range(count, world, rb, &ro, &rl); }
      pg_block_part(sl, rings, g, &sp, &spl);
      pg_block_part(rl, rings, g, &rp, &rpl);
      if (!spl && !rpl) continue;
      struct pg_step st;
      memset(&st, 0, sizeof(st));
      st.round = k;
      st.batch = k;
      st.seg = g;
      st.send_peer = d;
      st.recv_peer = -d;
      if (spl) { st.send_buf = PG_BUF_OUT; st.send_off = (int64_t)((so + sp) * es); st.send_bytes = (int64_t)(spl * es); }
      if (rpl) { st.recv_buf = PG_BUF_OUT; st.recv_off = (int64_t)((ro + rp) * es); st.recv_bytes = (int64_t)(rpl * es); }
      put(steps, max_steps, n, &st);
      ++n;
    }
  }
  if (steps && n > max_steps) return -1;
  return n;
}

/* ---- which steps reduce together ---------------------------------------------- */

/* qsort has no context argument: the plan being sorted, per calling thread */
static __thread const struct pg_step *t_sort_steps;

static int red_order(const void *pa, const void *pb) {
  const struct pg_step *a = &t_sort_steps[*(const int *)pa], *b = &t_sort_steps[*(const int *)pb];
  if (a->red_dst_buf != b->red_dst_buf) return a->red_dst_buf < b->red_dst_buf ? -1 : 1;
  if (a->red_src_buf != b->red_src_buf) return a->red_src_buf < b->red_src_buf ? -1 : 1;
  if (a->red_rev != b->red_rev) return a->red_rev < b->red_rev ? -1 : 1;
  if (a->red_dst_off != b->red_dst_off) return a->red_dst_off < b->red_dst_off ? -1 : 1;
  return 0;
}

int pg_plan_coalesce(const struct pg_step *st, int *idx, int n, size_t elem_size,
                     struct pg_red_range *out, int max_out) {
  if (n < 0 || (n && (!st || !idx || !out)) || (elem_size != 4 && elem_size != 8)) return -1;
  t_sort_steps = st;
  qsort(idx, (size_t)n, sizeof(int), red_order);
  const int64_t es = (int64_t)elem_size;
  int k = 0, u = 0;
  while (u < n) {
    const struct pg_step *s0 = &st[idx[u]];
    int64_t elems = s0->red_elems;
    int v = u + 1;
    for (; v < n; ++v) {
      const struct pg_step *s1 = &st[idx[v]];
      if (s1->red_rev != s0->red_rev || s1->red_dst_buf != s0->red_dst_buf || s1->red_src_buf != s0->red_src_buf ||
          s1->red_dst_off != s0->red_dst_off + elems * es || s1->red_src_off != s0->red_src_off + elems * es)
        break;
      elems += s1->red_elems;
    }
    if (k == max_out) return -1;
    out[k].dst_buf = s0->red_dst_buf;
    out[k].src_buf = s0->red_src_buf;
    out[k].rev = s0->red_rev;
    out[k].pad = 0;
    out[k].dst_off = s0->red_dst_off;
    out[k].src_off = s0->red_src_off;
    out[k].elems = elems;
    ++k;
    u = v;
  }
  return k;
}
