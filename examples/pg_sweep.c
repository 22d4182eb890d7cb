/*
 * examples/pg_sweep.c -- the reference's performance discipline as a plain C
 * caller of include/pg.h: "warm up once, log-sweep sizes, record
 * size, rounds, inflight, time_us, GB/s as CSV" (reference README.md:83-85),
 * with the "compare against a CPU reference" check of README.md:79-81 done on
 * every size (closed-form expected values, int32 exact, double exact because
 * the inputs are small integers / powers of two).
 *
 *   gcc -O2 -Iinclude examples/pg_sweep.c -Lrdma-ring-collectives_amd -lpg_amd \
 *       -Wl,-rpath,$PWD/rdma-ring-collectives_amd -o pg_sweep
 *   PG_RANK=r ./pg_sweep "127.0.0.1 127.0.0.1 ..." [allreduce|reducescatter|allgather]
 *                        [int32|double] [sum|prod] [min_bytes] [max_bytes] [reps]
 *
 * Buffers are host memory (malloc), as the reference's callers use them, so
 * the times include the PCIe copies.  size = bytes per rank (count * elem),
 * GB/s = size / time.  Rank 0 prints the CSV; every rank checks its results.
 * Exit status 0 = every size checked out.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pg.h"

static double now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e6 + (double)ts.tv_nsec * 1e-3;
}

/* Rank q's input element i: sums stay exact in int32 and double; products of
 * {1, 2, 1/2} (double) or {1, 2, -1} (int32) are exact too. */
static double in_val(int q, size_t i, int op) {
  if (op == OP_SUM) return (double)((i % 1000) + (size_t)q);
  int k = (int)((i + (size_t)q) % 3);
  return k == 0 ? 1.0 : (k == 1 ? 2.0 : 0.5);
}

static int32_t in_i32(int q, size_t i, int op) {
  if (op == OP_SUM) return (int32_t)((i % 1000) + (size_t)q);
  int k = (int)((i + (size_t)q) % 3);
  return k == 0 ? 1 : (k == 1 ? 2 : -1);
}

static double want_val(int W, size_t i, int op) {
  double acc = op == OP_SUM ? 0.0 : 1.0;
  for (int q = 0; q < W; ++q) acc = op == OP_SUM ? acc + in_val(q, i, op) : acc * in_val(q, i, op);
  return acc;
}

static int32_t want_i32(int W, size_t i, int op) {
  uint32_t acc = op == OP_SUM ? 0u : 1u;
  for (int q = 0; q < W; ++q) {
    uint32_t v = (uint32_t)in_i32(q, i, op);
    acc = op == OP_SUM ? acc + v : acc * v;
  }
  return (int32_t)acc;
}

static void fill(void *buf, size_t n, int dt, int q, int op) {
  for (size_t i = 0; i < n; ++i) {
    if (dt == DT_INT32) ((int32_t *)buf)[i] = in_i32(q, i, op);
    else ((double *)buf)[i] = in_val(q, i, op);
  }
}

/* result element i of the full reduction equals the closed form? */
static int check(const void *buf, size_t n, size_t first, int dt, int W, int op) {
  for (size_t i = 0; i < n; ++i) {
    size_t g = first + i;
    int ok = dt == DT_INT32 ? ((const int32_t *)buf)[i] == want_i32(W, g, op)
                            : ((const double *)buf)[i] == want_val(W, g, op);
    if (!ok) return 0;
  }
  return 1;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s \"host1 host2 ...\" [allreduce|reducescatter|allgather] [int32|double] "
                    "[sum|prod] [min_bytes] [max_bytes] [reps]\n", argv[0]);
    return 2;
  }
  const char *coll = argc > 2 ? argv[2] : "allreduce";
  DATATYPE dt = (argc > 3 && strcmp(argv[3], "double") == 0) ? DT_DOUBLE : DT_INT32;
  OPERATION op = (argc > 4 && strcmp(argv[4], "prod") == 0) ? OP_PROD : OP_SUM;
  size_t min_b = argc > 5 ? strtoull(argv[5], NULL, 0) : 4096;
  size_t max_b = argc > 6 ? strtoull(argv[6], NULL, 0) : (64u << 20);
  int reps = argc > 7 ? atoi(argv[7]) : 5;
  size_t es = dt == DT_INT32 ? 4 : 8;
  if (min_b < es) min_b = es;
  if (reps < 1) reps = 1;

  void *h = NULL;
  if (connect_process_group(argv[1], &h) != 0) return 1;
  struct pg *pg = (struct pg *)h;
  const int W = pg->world_size, r = pg->rank;
  int bad = 0;
  int32_t sync_in = 0, sync_out = 0;

  if (r == 0) printf("size,rounds,inflight,time_us,GB/s\n");
  for (size_t bytes = min_b; bytes <= max_b && !bad; bytes *= 4) {
    size_t count = bytes / es;
    size_t full = strcmp(coll, "allgather") == 0 ? count * (size_t)W : count;
    void *send = malloc(count * es), *recv = malloc(full * es);
    if (!send || !recv) { fprintf(stderr, "rank %d: out of host memory\n", r); return 1; }
    fill(send, count, dt, r, op);
    double t = 0.0;
    for (int it = 0; it <= reps; ++it) {           /* iteration 0 is the warm-up */
      if (pg_all_reduce(&sync_in, &sync_out, 1, DT_INT32, OP_SUM, h) != 0) { bad = 1; break; }  /* align ranks */
      double t0 = now_us();
      int rc;
      if (strcmp(coll, "reducescatter") == 0) rc = pg_reduce_scatter(send, recv, (int)count, dt, op, h);
      else if (strcmp(coll, "allgather") == 0) rc = pg_all_gather(send, recv, (int)count, dt, h);
      else rc = pg_all_reduce(send, recv, (int)count, dt, op, h);
      double t1 = now_us();
      if (rc != 0) { fprintf(stderr, "rank %d: %s failed at %zu bytes\n", r, coll, bytes); bad = 1; break; }
      if (it > 0) t += t1 - t0;
    }
    if (!bad) {
      int ok;
      if (strcmp(coll, "reducescatter") == 0) {
        size_t blk = W == 1 ? count : (count + (size_t)W - 1) / (size_t)W;
        size_t off = W == 1 ? 0 : (size_t)r * blk;
        size_t len = off >= count ? 0 : (off + blk > count ? count - off : blk);
        ok = check(recv, len, off, dt, W, op);
      } else if (strcmp(coll, "allgather") == 0) {
        ok = 1;
        for (int q = 0; q < W && ok; ++q) {
          void *mine = malloc(count * es);
          fill(mine, count, dt, q, op);
          ok = memcmp((char *)recv + (size_t)q * count * es, mine, count * es) == 0;
          free(mine);
        }
      } else {
        ok = check(recv, count, 0, dt, W, op);
      }
      if (!ok) { fprintf(stderr, "rank %d: %s result mismatch at %zu bytes\n", r, coll, bytes); bad = 1; }
    }
    if (r == 0 && !bad) {
      double us = t / reps;
      printf("%zu,%d,%d,%.1f,%.3f\n", bytes, W - 1, pg->inflight, us, (double)bytes / us * 1e-3);
      fflush(stdout);
    }
    free(send);
    free(recv);
  }
  fprintf(stderr, "rank %d/%d: %s\n", r, W, bad ? "FAIL" : "OK");
  pg_close(h);
  return bad ? 1 : 0;
}
