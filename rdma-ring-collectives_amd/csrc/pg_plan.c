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
 *     src/pg.c:282-287).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "pg.h"
#include "pg_ext.h"

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

static void put(struct pg_step *steps, int max_steps, int n, const struct pg_step *s) {
  if (steps && n < max_steps) steps[n] = *s;
}

int pg_plan_reduce_scatter(int rank, int world, int count, int datatype,
                           size_t chunk_bytes, size_t eager_max, int inflight,
                           int out_aliases_src, struct pg_step *steps, int max_steps) {
  size_t es = plan_elem_size(datatype);
  if (!es || world < 1 || rank < 0 || rank >= world || count < 0) return -1;
  if (inflight < 1) inflight = 1;
  int n = 0, batch = -1;
  for (int k = 0; k + 1 < world; ++k) {
    int sb = ring_mod(rank - 1 - k, world);   /* rs_send_chunk_index(k, rank-1) */
    int tb = ring_mod(rank - 2 - k, world);   /* rs_recv_chunk_index(k, rank-1) */
    size_t so, sl, to, tl;
    pg_block_range(count, world, sb, &so, &sl);
    pg_block_range(count, world, tb, &to, &tl);
    int last = (k == world - 2);
    size_t sseg = seg_elems_for(sl, es, chunk_bytes, eager_max);
    size_t tseg = seg_elems_for(tl, es, chunk_bytes, eager_max);
    size_t ns = nsegs(sl, sseg), nt = nsegs(tl, tseg);
    size_t nj = ns > nt ? ns : nt;
    int in_batch = inflight;                  /* force a new batch per round */
    for (size_t j = 0; j < nj; ++j) {
      struct pg_step st;
      memset(&st, 0, sizeof(st));
      if (in_batch == inflight) { ++batch; in_batch = 0; }
      ++in_batch;
      st.round = k;
      st.batch = batch;
      st.seg = (int32_t)j;
      if (j < ns) {
        size_t e0 = j * sseg, len = sl - e0 < sseg ? sl - e0 : sseg;
        if (k == 0) { st.send_buf = PG_BUF_SRC; st.send_off = (int64_t)((so + e0) * es); }
        else {
          st.send_buf = ((k - 1) & 1) ? PG_BUF_STAGE1 : PG_BUF_STAGE0;
          st.send_off = (int64_t)(e0 * es);
          st.send_wait = 1;                   /* previous round reduced it */
        }
        st.send_bytes = (int64_t)(len * es);
      }
      if (j < nt) {
        size_t e0 = j * tseg, len = tl - e0 < tseg ? tl - e0 : tseg;
        int stage = (k & 1) ? PG_BUF_STAGE1 : PG_BUF_STAGE0;
        st.recv_buf = (last && !out_aliases_src) ? PG_BUF_OUT : stage;
        st.recv_off = (int64_t)(e0 * es);
        st.recv_bytes = (int64_t)(len * es);
        st.red_elems = (int64_t)len;
        if (last && out_aliases_src) {
          /* OUT is block `rank` of SRC: fold the arrival into it in place
           * (local op incoming == incoming op local bit for bit: + and * are
           * commutative in IEEE-754 and in two's complement) */
          st.red_dst_buf = PG_BUF_OUT; st.red_dst_off = st.recv_off;
          st.red_src_buf = stage;      st.red_src_off = st.recv_off;
        } else {
          /* arrival op= this rank's own contribution to the block */
          st.red_dst_buf = st.recv_buf; st.red_dst_off = st.recv_off;
          st.red_src_buf = PG_BUF_SRC;  st.red_src_off = (int64_t)((to + e0) * es);
        }
      }
      put(steps, max_steps, n, &st);
      ++n;
    }
  }
  if (steps && n > max_steps) return -1;
  return n;
}

int pg_plan_all_gather(int rank, int world, int count, int datatype, int uniform,
                       struct pg_step *steps, int max_steps) {
  size_t es = plan_elem_size(datatype);
  if (!es || world < 1 || rank < 0 || rank >= world || count < 0) return -1;
  int n = 0;
  for (int k = 0; k + 1 < world; ++k) {
    int sb = ring_mod(rank - k, world);       /* src/pg.c:310 */
    int rb = ring_mod(rank - k - 1, world);   /* src/pg.c:311 */
    size_t so, sl, ro, rl;
    if (uniform) { so = (size_t)sb * (size_t)count; sl = (size_t)count; ro = (size_t)rb * (size_t)count; rl = (size_t)count; }
    else { pg_block_range(count, world, sb, &so, &sl); pg_block_range(count, world, rb, &ro, &rl); }
    if (!sl && !rl) continue;
    struct pg_step st;
    memset(&st, 0, sizeof(st));
    st.round = k;
    st.batch = k;
    if (sl) { st.send_buf = PG_BUF_OUT; st.send_off = (int64_t)(so * es); st.send_bytes = (int64_t)(sl * es); }
    if (rl) { st.recv_buf = PG_BUF_OUT; st.recv_off = (int64_t)(ro * es); st.recv_bytes = (int64_t)(rl * es); }
    put(steps, max_steps, n, &st);
    ++n;
  }
  if (steps && n > max_steps) return -1;
  return n;
}
