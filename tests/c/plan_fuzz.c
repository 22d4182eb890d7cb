/* tests/c/plan_fuzz.c -- the ring planner (csrc/pg_plan.c, pure C) under
 * AddressSanitizer + UndefinedBehaviorSanitizer: every shape in the grid below
 * is planned for every rank, in one to four rings, reduce-scatter (plain and
 * in place), the direct exchange and all-gather, and every offset a step names
 * must lie inside the buffer it names.  Built and run by tests/test_plan_sanitize.py.  Exit 0 = ok. */
#include <stdio.h>
#include <stdlib.h>
#include "pg.h"
#include "pg_ext.h"
int main(void) {
  long total = 0;
  int counts[] = {0, 1, 2, 3, 5, 7, 8, 9, 63, 64, 65, 1000, 1001, 4099, 20011};
  size_t cbs[] = {4, 12, 100, 4096, 1 << 20};
  for (int W = 1; W <= 9; ++W)
    for (int ci = 0; ci < 15; ++ci)
      for (int dt = 0; dt < 2; ++dt)
        for (int cbi = 0; cbi < 5; ++cbi)
          for (int eager = 0; eager <= 4096; eager += 4096)
            for (int infl = 1; infl <= 3; ++infl)
              for (int rings = 1; rings <= 4; ++rings)
                for (int alias = 0; alias < 2; ++alias)
                  for (int r = 0; r < W; ++r) {
                    int n = pg_plan_reduce_scatter(r, W, counts[ci], dt, cbs[cbi], eager, infl, rings, alias, NULL, 0);
                    if (n < 0) { printf("fail %d %d\n", W, r); return 1; }
                    struct pg_step *st = malloc(sizeof(*st) * (n ? n : 1));
                    int m = pg_plan_reduce_scatter(r, W, counts[ci], dt, cbs[cbi], eager, infl, rings, alias, st, n);
                    if (m != n) return 2;
                    /* the plan must name only in-range offsets */
                    size_t es = dt ? 8 : 4, blk = ((size_t)counts[ci] + W - 1) / W;
                    size_t stage = (size_t)rings * ((blk + rings - 1) / rings);   /* staging block, elements */
                    for (int i = 0; i < n; ++i) {
                      if (st[i].send_buf == PG_BUF_SRC && (size_t)(st[i].send_off + st[i].send_bytes) > counts[ci] * es) return 3;
                      if ((st[i].send_buf == PG_BUF_STAGE0 || st[i].send_buf == PG_BUF_STAGE1) &&
                          (size_t)(st[i].send_off + st[i].send_bytes) > stage * es) return 4;
                      if ((st[i].recv_buf == PG_BUF_STAGE0 || st[i].recv_buf == PG_BUF_STAGE1) &&
                          (size_t)(st[i].recv_off + st[i].recv_bytes) > stage * es) return 5;
                      if (st[i].recv_buf == PG_BUF_OUT && (size_t)(st[i].recv_off + st[i].recv_bytes) > blk * es) return 6;
                    }
                    /* the reduce launches (pg_plan_coalesce): every round's reduce steps, handed over
                     * in reverse, must come back as ranges that cover each element once, inside the
                     * buffers, never more ranges than steps */
                    {
                      int *idx = malloc(sizeof(int) * (n ? n : 1));
                      struct pg_red_range *rr = malloc(sizeof(*rr) * (n ? n : 1));
                      for (int k = 0; k + 1 < W; ++k) {
                        int m2 = 0;
                        long long want = 0, got = 0;
                        for (int i = n - 1; i >= 0; --i)
                          if (st[i].round == k && st[i].red_elems > 0) { idx[m2++] = i; want += st[i].red_elems; }
                        int nr = pg_plan_coalesce(st, idx, m2, es, rr, m2 ? m2 : 1);
                        if (nr < 0 || nr > m2) return 12;
                        for (int u = 0; u < nr; ++u) {
                          got += rr[u].elems;
                          if (rr[u].elems <= 0 || rr[u].dst_off < 0 || rr[u].src_off < 0) return 13;
                          if (rr[u].src_buf == PG_BUF_SRC && (size_t)(rr[u].src_off + rr[u].elems * (long long)es) > counts[ci] * es) return 14;
                          if (u && rr[u].dst_buf == rr[u - 1].dst_buf && rr[u].src_buf == rr[u - 1].src_buf &&
                              rr[u].rev == rr[u - 1].rev && rr[u].dst_off < rr[u - 1].dst_off + rr[u - 1].elems * (long long)es)
                            return 15;                       /* sorted, not overlapping */
                        }
                        if (got != want) return 16;
                      }
                      if (pg_plan_coalesce(st, idx, 1, 3, rr, 1) != -1) return 17;    /* bad element size */
                      free(idx);
                      free(rr);
                    }
                    total += n;
                    free(st);
                    if (!alias && !eager) {           /* the direct exchange (no alias / eager knobs) */
                      n = pg_plan_direct_reduce_scatter(r, W, counts[ci], dt, cbs[cbi], infl, rings, NULL, 0);
                      if (n < 0) return 7;
                      st = malloc(sizeof(*st) * (n ? n : 1));
                      if (pg_plan_direct_reduce_scatter(r, W, counts[ci], dt, cbs[cbi], infl, rings, st, n) != n) return 8;
                      size_t boff, blen;
                      pg_block_range(counts[ci], W, r, &boff, &blen);
                      for (int i = 0; i < n; ++i) {
                        if (st[i].send_bytes && (size_t)(st[i].send_off + st[i].send_bytes) > counts[ci] * es) return 9;
                        if (st[i].recv_bytes && (size_t)(st[i].recv_off + st[i].recv_bytes) > (size_t)W * blk * es) return 10;
                        if (st[i].red_fold && ((size_t)st[i].red_dst_off + st[i].red_elems * es > blen * es ||
                                               (size_t)st[i].red_src_off + st[i].red_elems * es > blk * es))
                          return 11;
                      }
                      total += n;
                      free(st);
                    }
                    n = pg_plan_all_gather(r, W, counts[ci], dt, alias, rings, NULL, 0);
                    st = malloc(sizeof(*st) * (n ? n : 1));
                    pg_plan_all_gather(r, W, counts[ci], dt, alias, rings, st, n);
                    free(st);
                  }
  printf("ok %ld steps\n", total);
  return 0;
}
