/*
 * examples/pg_demo.c -- a plain C caller of the reference API (include/pg.h),
 * built exactly as a user of the reference would build theirs, but linked
 * against libpg_amd.so:
 *
 *   gcc -O2 -Iinclude examples/pg_demo.c -Lrdma-ring-collectives_amd -lpg_amd \
 *       -Wl,-rpath,$PWD/rdma-ring-collectives_amd -o pg_demo
 *   PG_RANK=r PG_TRANSPORT=xgmi ./pg_demo "127.0.0.1 127.0.0.1" [count]   (one process per rank)
 *   ./pg_demo "$(hostname)"                                                 (single rank)
 *
 * Mirrors the reference's Quick Start (README.md:37-45): connect, all-reduce,
 * close -- plus reduce-scatter and all-gather -- on host buffers, and checks
 * every element against the closed form of the reduction.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pg.h"

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s \"host1 host2 ...\" [count]\n", argv[0]);
    return 2;
  }
  int count = argc > 2 ? atoi(argv[2]) : 1 << 20;
  void *h = NULL;
  if (connect_process_group(argv[1], &h) != 0) return 1;
  struct pg *pg = (struct pg *)h;          /* the public leading fields, as in the reference */
  int W = pg->world_size, r = pg->rank, bad = 0;

  /* all-reduce, int32 sum: sum over ranks of (i % 97 + rank) */
  int32_t *a = malloc(sizeof(int32_t) * (size_t)count), *b = malloc(sizeof(int32_t) * (size_t)count);
  for (int i = 0; i < count; ++i) a[i] = i % 97 + r;
  if (pg_all_reduce(a, b, count, DT_INT32, OP_SUM, h) != 0) bad++;
  for (int i = 0; i < count && !bad; ++i)
    if (b[i] != W * (i % 97) + W * (W - 1) / 2) { fprintf(stderr, "all_reduce mismatch at %d\n", i); bad++; }

  /* reduce-scatter, double product of powers of two: block `rank` of the result */
  double *x = malloc(sizeof(double) * (size_t)count), *y = malloc(sizeof(double) * (size_t)count);
  for (int i = 0; i < count; ++i) x[i] = ((i + r) % 3 == 0) ? 0.5 : ((i + r) % 3 == 1 ? 1.0 : 2.0);
  if (pg_reduce_scatter(x, y, count, DT_DOUBLE, OP_PROD, h) != 0) bad++;
  int blk = W == 1 ? count : (count + W - 1) / W;
  int off = W == 1 ? 0 : r * blk, len = off >= count ? 0 : (off + blk > count ? count - off : blk);
  for (int i = 0; i < len && !bad; ++i) {
    double want = 1.0;
    for (int q = 0; q < W; ++q) {
      int k = (off + i + q) % 3;
      want *= k == 0 ? 0.5 : (k == 1 ? 1.0 : 2.0);
    }
    if (y[i] != want) { fprintf(stderr, "reduce_scatter mismatch at %d\n", i); bad++; }
  }

  /* all-gather, in place (sendbuf NULL): slot q holds rank q's values */
  int32_t *g = malloc(sizeof(int32_t) * (size_t)count * (size_t)W);
  for (int i = 0; i < count; ++i) g[(size_t)r * count + i] = 1000 * r + i % 13;
  if (pg_all_gather(NULL, g, count, DT_INT32, h) != 0) bad++;
  for (int q = 0; q < W && !bad; ++q)
    for (int i = 0; i < count; ++i)
      if (g[(size_t)q * count + i] != 1000 * q + i % 13) { fprintf(stderr, "all_gather mismatch\n"); bad++; break; }

  printf("rank %d/%d: %s\n", r, W, bad ? "FAIL" : "OK");
  free(a); free(b); free(x); free(y); free(g);
  pg_close(h);
  return bad ? 1 : 0;
}
