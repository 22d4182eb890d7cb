/*
 * pg_xport_xgmi.c -- PG_TRANSPORT=xgmi: the reduce-scatter as direct reads of
 * every peer's contribution over xGMI, folded in ring order by one kernel.
 *
 * The reference moves each chunk one hop per round and reduces it on arrival
 * (ring design README.md:68-71; mocked at src/pg.c:277-289).  On one MI355X
 * node every GPU has a direct xGMI link to each of its 7 peers, so rank r can
 * read block r of all W contributions at once -- W-1 links busy instead of one
 * -- and fold them in the exact order the ring would:
 *     out = x[r+1] op x[r+2] op ... op x[r]        (indices mod W)
 * which is bit-identical to the RCCL ring and to the oracle's ring simulator.
 * This is a fused receive-reduce over every link of the GPU at once.
 *
 * Memory: each rank owns up to two IPC-exportable HBM regions, each mapped
 * into every peer with hipIpcOpenMemHandle and double-buffered by call parity:
 * contribution slots X0/X1 (used only when an input cannot be read in place)
 * and all-reduce result slots R0/R1 (used only by the reduce-scatter + gather
 * form of the all-reduce).  A region is allocated the first time a call needs
 * it, so a zero-copy reduce-scatter holds no exchange memory at all.  A call
 * that uses X copies its input into X[parity], meets the others at a host
 * barrier (node-local shared memory, pg_boot.c), then reads.  Double
 * buffering makes one barrier per call enough: a slot is rewritten two calls
 * later, and every rank passed the intervening call's barrier only after
 * finishing its reads.
 *
 * Every call closes at a barrier that carries each rank's status (finish), so
 * outcomes are collective: a failure anywhere fails the call everywhere, and a
 * peer input that could not be mapped makes every rank redo the call with the
 * slot copy (xgmi_retry).  Descriptors carry the byte count, so ranks called
 * with different counts fail before reading anything.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#include "pg_impl.h"

#define XG_REG_X 0              /* contribution slots X0, X1 */
#define XG_REG_R 1              /* all-reduce result slots R0, R1 */
#define XG_IMPORTS 2            /* mapped input allocations cached per peer */
#define XG_FOLD_ONE_LAUNCH_MAX (1u << 20)   /* blocks up to this size fold all ring parts in one launch
                                               (profiles/r01_fold_launch_probe.txt: one launch wins to 1 MiB,
                                               ties at 4 MiB, loses at 16 MiB) */

struct xg_import {
  unsigned long long bid;
  uint64_t peer_base;           /* the allocation's address range in the      */
  uint64_t peer_size;           /* exporter                                   */
  void *base;                   /* its mapping here                           */
  unsigned long stamp;
};
#define XG_GRANULE (64ull << 20)
/* A cached mapping of a peer's input keeps that allocation's HBM alive in the
 * peer even after it frees it.  Mappings of allocations at least this large
 * are kept only while they are the peer's current input: the first call with
 * another input closes them (tests/test_xgmi_gpu.py::
 * test_xgmi_freed_large_input_is_released).  Small ones stay in the LRU. */
#define XG_KEEP_MAX (256ull << 20)

struct xg_hist {
  uint64_t base, size;
  unsigned long long bid;
};

struct xg_region {
  void *mem;                    /* my allocation: 2 slots of cap bytes      */
  size_t cap;                   /* bytes per slot (0: not allocated yet)    */
  void **peer;                  /* peer[q] = rank q's allocation, mapped    */
};

struct xgmi_ctx {
  struct xg_region reg[2];      /* XG_REG_X, XG_REG_R                       */
  size_t oneshot_max;           /* all-reduce at most this many bytes: one-shot */
  void *bar;                    /* node-local shm barrier (pg_boot.c), or NULL */
  int zc;                       /* zero-copy inputs allowed (PG_XGMI_ZERO_COPY) */
  int push;                     /* reduce-scatter writes (push), not reads: PG_XGMI_MODE */
  int mode_auto;                /* PG_XGMI_MODE=auto (default): chosen at init by a link probe */
  double probe_read_gbs, probe_write_gbs;   /* that probe: median over ranks, all links at once */
  int force_copy;               /* this call: no zero-copy (the retry after a failed import) */
  long fail_import_at;          /* test hook PG_XGMI_FAIL_IMPORT=n: the n-th import fails */
  long imports;                 /* imports attempted so far (for the hook)   */
  hipIpcMemHandle_t exp_h;      /* last export of a caller allocation       */
  unsigned long long exp_bid;
  void *exp_base;
  int exp_valid;
  struct xg_import *imp;        /* world * XG_IMPORTS mapped peer inputs     */
  unsigned long clock;
  unsigned long gen;            /* collective calls so far (slot parity)    */
};

static void drop_imports(struct pg *pg, struct xgmi_ctx *x);
static int choose_mode(struct pg *pg);

/* ROCm 7.2: hipIpcOpenMemHandle never returns for an allocation whose size has
 * bit 31 set (2 GiB, 2 GiB + 2 MiB, 3 GiB, 6 GiB stall; 2 GiB - 2 MiB, 4, 5,
 * 8, 12 GiB open in < 1 ms; measured on MI355X, tools/ipc_probe.py --mode sizes).  So no
 * allocation of that size is ever exported: our own slot memory is padded to
 * the next multiple of 4 GiB, and a caller's input living in such an
 * allocation takes the slot copy instead of zero-copy. */
static int ipc_size_ok(size_t bytes) { return (bytes & (1ull << 31)) == 0; }

static size_t ipc_safe_size(size_t bytes) {
  return ipc_size_ok(bytes) ? bytes : (bytes + (4ull << 30) - 1) & ~((4ull << 30) - 1);
}

static struct xgmi_ctx *ctx_of(struct pg *pg) {
  return (struct xgmi_ctx *)((struct pg_impl *)pg->impl)->xctx;
}

static double us_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e6 + (double)ts.tv_nsec * 1e-3;
}

/* Rank q's slot `parity` of region `reg` (NULL while the region is unallocated). */
static char *slot(struct xgmi_ctx *x, int reg, int q, int parity) {
  const struct xg_region *g = &x->reg[reg];
  return g->peer[q] ? (char *)g->peer[q] + (size_t)parity * g->cap : NULL;
}

/* All ranks of this transport share one node: shm barrier, TCP as fallback. */
static int barrier(struct pg *pg) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xgmi_ctx *x = (struct xgmi_ctx *)im->xctx;
  return x->bar ? pg_shm_barrier(pg, x->bar) : pg_boot_barrier(pg, im->boot_fds);
}

static void unmap_peers(struct pg *pg, struct xg_region *g) {
  if (!g->peer) return;
  for (int q = 0; q < pg->world_size; ++q)
    if (q != pg->rank && g->peer[q]) hipIpcCloseMemHandle(g->peer[q]);
  memset(g->peer, 0, sizeof(void *) * (size_t)pg->world_size);
}

static void unmap(struct pg *pg, struct xg_region *g) {
  unmap_peers(pg, g);
  if (g->mem) hipFree(g->mem);
  g->mem = NULL;
  g->cap = 0;
}

/* Region `reg` holds slots of at least `bytes`.  Collective: every rank calls
 * it at the same point of the same call with the same `bytes` (same count),
 * so every rank grows in the same call to the same size.
 *
 * Growth order matters (observed on ROCm 7.2, tests/test_xgmi_gpu.py::
 * test_xgmi_slot_growth): unmapping the peers' old slots, then allocating and
 * exporting the replacement failed with hipIpcGetMemHandle: invalid argument.
 * So the replacement is allocated and exported while every old import is
 * still mapped, and the old allocation is freed only after all ranks have
 * dropped their mappings of it. */
/* Every rank learns whether every rank's step succeeded (one TCP all-gather). */
static int all_ranks_ok(struct pg *pg, int ok) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  char mine = (char)(ok != 0), all[16];
  if (pg_boot_allgather(pg, im->boot_fds, &mine, all, 1)) return 0;
  for (int q = 0; q < pg->world_size; ++q)
    if (!all[q]) return 0;
  return 1;
}

struct xg_export {
  hipIpcMemHandle_t h;
  int32_t ok;
};

static int ensure(struct pg *pg, int reg, size_t bytes) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xg_region *g = &ctx_of(pg)->reg[reg];
  if (bytes <= g->cap && g->mem) return 0;
  size_t cap = g->cap ? g->cap : XG_GRANULE;
  while (cap < bytes) cap *= 2;
  pg_trace(pg, "xgmi ensure: region %d grows %zu -> %zu bytes per slot", reg, g->cap, cap);
  if (g->mem && barrier(pg)) return -1;      /* nobody still reads the old slots */
  /* allocate and export; every rank learns whether every rank managed to
   * before anything is torn down, so a failure (out of memory) is collective */
  void *fresh = NULL;
  struct xg_export mine, all[16];
  memset(&mine, 0, sizeof(mine));
  hipError_t e = hipMalloc(&fresh, ipc_safe_size(cap * 2));
  if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.h, fresh);
  mine.ok = e == hipSuccess;
  if (!mine.ok) {
    (void)hipGetLastError();
    pg_set_error("xgmi: allocating/exporting %zu bytes of slots: %s", cap * 2, hipGetErrorString(e));
  }
  pg_trace(pg, "xgmi ensure: allocated and exported: %d", mine.ok);
  if (pg_boot_allgather(pg, im->boot_fds, &mine, all, sizeof(mine))) {
    if (fresh) hipFree(fresh);
    return -1;
  }
  int ok = 1;
  for (int q = 0; q < pg->world_size; ++q) ok &= all[q].ok;
  if (!ok) {
    if (fresh) hipFree(fresh);
    if (mine.ok) pg_set_error("xgmi: a peer could not allocate %zu bytes of exchange slots", cap * 2);
    return -1;                                /* the old slots stay as they were, on every rank */
  }
  if (g->mem) {
    unmap_peers(pg, g);
    pg_trace(pg, "xgmi ensure: old peer slots unmapped");
    if (barrier(pg)) { hipFree(fresh); return -1; }   /* nobody maps my old slots */
    hipFree(g->mem);
    pg_trace(pg, "xgmi ensure: old slots freed");
  }
  g->mem = fresh;
  g->cap = cap;
  g->peer[pg->rank] = g->mem;
  int opened = 1;
  for (int q = 0; q < pg->world_size && opened; ++q) {
    if (q == pg->rank) continue;
    e = hipIpcOpenMemHandle(&g->peer[q], all[q].h, hipIpcMemLazyEnablePeerAccess);
    pg_trace(pg, "xgmi ensure: opened rank %d's slots: %s", q, hipGetErrorString(e));
    if (e != hipSuccess) {
      g->peer[q] = NULL;
      pg_set_error("xgmi: hipIpcOpenMemHandle(rank %d): %s", q, hipGetErrorString(e));
      opened = 0;
    }
  }
  if (!all_ranks_ok(pg, opened)) {
    /* undo on every rank: nobody keeps a region some peer cannot reach */
    unmap_peers(pg, g);
    if (barrier(pg) == 0) hipFree(g->mem);
    g->mem = NULL;
    g->cap = 0;
    if (opened) pg_set_error("xgmi: a peer could not map this rank's exchange slots");
    return -1;
  }
  return 0;
}

/* Can every rank map device memory of every other rank?  The server list only
 * says that the ranks share a host; GPUs without peer access to each other, or
 * processes confined to their own device, would fail at the first exchange.
 * Each rank exports a small allocation, opens every peer's, closes it again,
 * and the outcome is all-gathered: 1 = every rank reached every peer, 0 = some
 * rank could not (the same answer on every rank, nothing left mapped),
 * -1 = the bootstrap itself failed.  Test hook PG_XGMI_FAIL_REACH=r: rank r
 * (-1: every rank) reports that it could not. */
#define XG_REACH_BYTES (2u << 20)
static int reach_check(struct pg *pg) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  const int W = pg->world_size, r = pg->rank;
  void *probe = NULL;
  struct xg_export mine, all[16];
  memset(&mine, 0, sizeof(mine));
  hipError_t e = hipMalloc(&probe, XG_REACH_BYTES);
  if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.h, probe);
  mine.ok = e == hipSuccess;
  if (!mine.ok) (void)hipGetLastError();
  if (pg_boot_allgather(pg, im->boot_fds, &mine, all, sizeof(mine))) {
    if (probe) hipFree(probe);
    return -1;
  }
  int ok = 1;
  for (int q = 0; q < W; ++q) ok &= all[q].ok;
  for (int q = 0; q < W && ok; ++q) {
    if (q == r) continue;
    void *p = NULL;
    e = hipIpcOpenMemHandle(&p, all[q].h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      pg_trace(pg, "xgmi reach check: rank %d's memory does not map here: %s", q, hipGetErrorString(e));
      ok = 0;
    } else {
      hipIpcCloseMemHandle(p);
    }
  }
  const char *h = getenv("PG_XGMI_FAIL_REACH");
  if (h && *h && (atoi(h) == r || atoi(h) == -1)) ok = 0;
  /* the all-gather is also the point after which no peer maps my probe */
  ok = all_ranks_ok(pg, ok);
  if (probe) hipFree(probe);
  return ok;
}

/* Returns 0, -1 (failed), or 1: the ranks cannot reach each other's memory
 * (agreed by all of them; nothing of the transport is left set up except the
 * bootstrap star, which the caller may reuse for another transport). */
int pg_xport_xgmi_init(struct pg *pg) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  if (pg->world_size > 16) { pg_set_error("xgmi transport: at most 16 ranks"); return -1; }
  struct xgmi_ctx *x = (struct xgmi_ctx *)calloc(1, sizeof(*x));
  if (!x) return -1;
  im->xctx = x;
  for (int g = 0; g < 2; ++g) {
    x->reg[g].peer = (void **)calloc((size_t)pg->world_size, sizeof(void *));
    if (!x->reg[g].peer) { pg_set_error("xgmi: out of host memory"); return -1; }
  }
  x->oneshot_max = 1u << 20;
  const char *e = getenv("PG_ONESHOT_MAX");
  if (e && *e) x->oneshot_max = (size_t)strtoull(e, NULL, 0);
  e = getenv("PG_XGMI_ZERO_COPY");
  x->zc = !(e && *e == '0');
  e = getenv("PG_XGMI_MODE");
  if (e && *e && strcmp(e, "read") != 0 && strcmp(e, "push") != 0 && strcmp(e, "auto") != 0) {
    pg_set_error("PG_XGMI_MODE=%s: expected auto, read or push", e);
    return -1;
  }
  x->push = e && strcmp(e, "push") == 0;
  x->mode_auto = !(e && *e) || strcmp(e, "auto") == 0;
  e = getenv("PG_XGMI_FAIL_IMPORT");
  x->fail_import_at = (e && *e) ? atol(e) : 0;
  x->imp = (struct xg_import *)calloc((size_t)pg->world_size * XG_IMPORTS, sizeof(struct xg_import));
  if (!x->imp) { pg_set_error("xgmi: out of host memory"); return -1; }
  if (!im->boot_fds && pg_boot_open(pg, &im->boot_fds)) return -1;
  int reach = reach_check(pg);
  if (reach < 0) return -1;
  if (!reach) {
    pg_set_error("xgmi transport: some rank cannot map a peer's device memory (no peer access or IPC between the GPUs)");
    return 1;
  }
  const char *nb = getenv("PG_NO_SHM_BARRIER");
  if (!(nb && *nb == '1') && pg_shm_open(pg, im->boot_fds, &x->bar)) return -1;
  /* push mode publishes its per-call flags in the shm page's descriptor table:
   * without the page (PG_NO_SHM_BARRIER=1, or shm_open/mmap failed somewhere --
   * pg_shm_open falls back on every rank together) every rank reads instead */
  if (x->push && !x->bar) {
    pg_trace(pg, "xgmi: PG_XGMI_MODE=push needs the shared-memory page; using the read path");
    x->push = 0;
  }
  if (barrier(pg)) return -1;
  return x->mode_auto && x->bar ? choose_mode(pg) : 0;
}

/* PG_XGMI_MODE=auto: measure, don't guess.  Every rank pulls from all peers
 * at once, then pushes to all peers at once (pgx_xgmi_link_probe, 32 MiB, 3
 * launches per phase, two passes, the better of each); the medians over ranks
 * decide, on every rank alike
 * (one all-gather of the pairs): push when the links move pushed bytes at
 * least 15% faster than pulled ones, else read.  ~1 ms on a node; the probe's
 * exchange slots stay allocated for later calls. */
#define XG_PROBE_BYTES (32u << 20)
static int cmp_double(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

static int choose_mode(struct pg *pg) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xgmi_ctx *x = ctx_of(pg);
  /* two passes, the better rate of each direction.  A precaution, not a
   * response to an observed failure: the choice is made once per handle from
   * about a millisecond of traffic, and a second pass costs as little. */
  double g[4] = {0, 0, 0, 0}, best[2] = {0, 0};
  for (int pass = 0; pass < 2; ++pass) {
    if (pgx_xgmi_link_probe(pg, XG_PROBE_BYTES, 3, g)) return -1;
    if (g[2] > best[0]) best[0] = g[2];
    if (g[3] > best[1]) best[1] = g[3];
  }
  double mine[2] = {best[0], best[1]}, all[16][2], rd[16], wr[16];
  if (pg_boot_allgather(pg, im->boot_fds, mine, all, sizeof(mine))) return -1;
  const int W = pg->world_size;
  for (int q = 0; q < W; ++q) { rd[q] = all[q][0]; wr[q] = all[q][1]; }
  qsort(rd, (size_t)W, sizeof(double), cmp_double);
  qsort(wr, (size_t)W, sizeof(double), cmp_double);
  x->probe_read_gbs = rd[W / 2];
  x->probe_write_gbs = wr[W / 2];
  x->push = x->probe_write_gbs >= 1.15 * x->probe_read_gbs;
  pg_trace(pg, "xgmi auto mode: read %.1f GB/s, write %.1f GB/s -> %s", x->probe_read_gbs, x->probe_write_gbs,
           x->push ? "push" : "read");
  return 0;
}

int pgx_xgmi_mode(void *pg_handle, int *push, double *read_gbs, double *write_gbs) {
  struct pg *pg = (struct pg *)pg_handle;
  if (!pg || !pg->impl || pg->transport != PG_TRANSPORT_XGMI || !push) {
    pg_set_error("pgx_xgmi_mode: needs an xgmi handle");
    return -1;
  }
  struct xgmi_ctx *x = ctx_of(pg);
  *push = x->push;
  if (read_gbs) *read_gbs = x->mode_auto ? x->probe_read_gbs : 0.0;
  if (write_gbs) *write_gbs = x->mode_auto ? x->probe_write_gbs : 0.0;
  return 0;
}

void pg_xport_xgmi_destroy(struct pg *pg) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xgmi_ctx *x = ctx_of(pg);
  if (!x) return;
  /* peers may still be reading my last contribution: meet them first
   * (regions are allocated collectively, so every rank takes this branch alike) */
  if ((x->reg[XG_REG_X].mem || x->reg[XG_REG_R].mem) && im->boot_fds) barrier(pg);
  drop_imports(pg, x);
  free(x->imp);
  for (int g = 0; g < 2; ++g) {
    unmap(pg, &x->reg[g]);
    free(x->reg[g].peer);
  }
  pg_shm_close(x->bar);
  free(x);
  im->xctx = NULL;
}

static int is_dev(const void *p) {
  if (!p) return 0;
  hipPointerAttribute_t a;
  memset(&a, 0, sizeof(a));
  if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return 0; }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.isManaged;
}

/* ---- sharing the inputs -------------------------------------------------------
 * Every rank must be able to read every other rank's input.  Two ways:
 *  - zero-copy: the caller's own device allocation is exported through HIP
 *    IPC (cached by HIP buffer id on both sides), with descriptors in the
 *    node-local shm page; used when every rank's input is device memory that
 *    exports and the output does not overlap the input.  A closing barrier
 *    keeps inputs untouched until every peer has finished reading them.
 *  - slot copy: the input is copied into this rank's X[parity] slot.
 * The choice is collective: each rank flags whether its export worked, and
 * after the first barrier every rank sees the same flags. */
#define XG_DESC_OFF 256          /* descriptor table offset in the shm page */

struct xg_desc {
  hipIpcMemHandle_t h;
  uint64_t bid;                  /* HIP buffer id of the exported allocation */
  uint64_t base;                 /* its base address in the exporter          */
  uint64_t size;                 /* and its size                              */
  uint64_t off;                  /* input offset inside it                    */
  uint64_t nbytes;               /* the call's input bytes (must agree)       */
  int32_t ok;
  int32_t pad;
};

/* call-result flags, double-buffered by call parity, after the descriptors */
#define XG_FLAG_OFF (XG_DESC_OFF + 16 * (int)sizeof(struct xg_desc))
_Static_assert(XG_FLAG_OFF + 2 * 16 * 4 <= 4096, "shm page layout");

static struct xg_desc *descs(struct xgmi_ctx *x) {
  return (struct xg_desc *)((char *)x->bar + XG_DESC_OFF);
}

/* An IPC handle names (exporter pid, address, size), not the allocation
 * (tools/ipc_probe.py --mode reuse: a new allocation at a freed one's address exports
 * byte-identical handle bytes), and what hipIpcOpenMemHandle does in an
 * importer that opened that range before is not something this transport can
 * control: it may hand back a mapping of the freed allocation (stale data,
 * tools/xgmi_cfg5_probe.py and tests/test_xgmi_gpu.py::
 * test_xgmi_input_reallocated_at_same_address reproduced it), and it failed
 * once in 226 calls of the cfg5 probe.  So an allocation whose address range
 * overlaps one this process exported earlier under another buffer id is never
 * exported: the call takes the slot copy instead.  Buffer ids are never
 * reused, so the history check is exact. */
/* The history is per process, not per handle: the importer-side state it
 * guards lives in each peer's HIP runtime and outlives a pg handle. */
static struct {
  pthread_mutex_t mu;
  struct xg_hist *v;
  size_t n, cap;
} g_exported = {PTHREAD_MUTEX_INITIALIZER, NULL, 0, 0};

/* 1: [base, base+size) may be exported under `bid` (recorded if new); 0: it
 * overlaps an allocation exported before under another id, or out of memory. */
static int may_export(uint64_t base, uint64_t size, unsigned long long bid) {
  int ok = 1, seen = 0;
  pthread_mutex_lock(&g_exported.mu);
  for (size_t i = 0; i < g_exported.n && ok; ++i) {
    const struct xg_hist *h = &g_exported.v[i];
    if (h->bid == bid) seen = 1;
    else if (h->base < base + size && base < h->base + h->size) ok = 0;
  }
  if (ok && !seen) {
    if (g_exported.n == g_exported.cap) {
      size_t cap = g_exported.cap ? 2 * g_exported.cap : 64;
      struct xg_hist *v = (struct xg_hist *)realloc(g_exported.v, cap * sizeof(*v));
      if (v) { g_exported.v = v; g_exported.cap = cap; }
    }
    if (g_exported.n < g_exported.cap) {
      g_exported.v[g_exported.n].base = base;
      g_exported.v[g_exported.n].size = size;
      g_exported.v[g_exported.n].bid = bid;
      ++g_exported.n;
    } else {
      ok = 0;
    }
  }
  pthread_mutex_unlock(&g_exported.mu);
  return ok;
}

static int export_input(struct xgmi_ctx *x, const void *in, struct xg_desc *d) {
  memset(d, 0, sizeof(*d));
  void *base = NULL;
  size_t size = 0;
  unsigned long long bid = 0;
  if (hipMemGetAddressRange((hipDeviceptr_t *)&base, &size, (hipDeviceptr_t)in) != hipSuccess ||
      hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)in) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  if (!ipc_size_ok(size)) return 0;           /* peers could not open it: slot copy */
  if (!x->exp_valid || x->exp_bid != bid || x->exp_base != base) {
    if (!may_export((uint64_t)(uintptr_t)base, (uint64_t)size, bid)) return 0;
    x->exp_valid = 0;
    if (hipIpcGetMemHandle(&x->exp_h, base) != hipSuccess) { (void)hipGetLastError(); return 0; }
    x->exp_bid = bid;
    x->exp_base = base;
    x->exp_valid = 1;
  }
  d->h = x->exp_h;
  d->bid = bid;
  d->base = (uint64_t)(uintptr_t)base;
  d->size = (uint64_t)size;
  d->off = (uint64_t)((const char *)in - (const char *)base);
  d->ok = 1;
  return 1;
}

/* Peer q's input, mapped (LRU cache of XG_IMPORTS allocations per peer).  On
 * a miss, any cached mapping of this peer whose exporter range overlaps the
 * new one is closed first (its allocation has been freed: live allocations do
 * not overlap); with export_input's rule this should never find one. */
static const char *import_input(struct xgmi_ctx *x, int q, const struct xg_desc *d) {
  struct xg_import *e = &x->imp[q * XG_IMPORTS];
  ++x->clock;
  for (int i = 0; i < XG_IMPORTS; ++i)
    if (e[i].base && e[i].bid == d->bid) { e[i].stamp = x->clock; return (const char *)e[i].base + d->off; }
  for (int i = 0; i < XG_IMPORTS; ++i)
    if (e[i].base && e[i].peer_base < d->base + d->size && d->base < e[i].peer_base + e[i].peer_size) {
      hipIpcCloseMemHandle(e[i].base);
      e[i].base = NULL;
      e[i].stamp = 0;
    }
  int lru = 0;
  for (int i = 1; i < XG_IMPORTS; ++i)
    if (e[i].stamp < e[lru].stamp) lru = i;
  if (e[lru].base) { hipIpcCloseMemHandle(e[lru].base); e[lru].base = NULL; }
  void *p = NULL;
  hipError_t err = ++x->imports == x->fail_import_at ? hipErrorInvalidValue
                                                     : hipIpcOpenMemHandle(&p, d->h, hipIpcMemLazyEnablePeerAccess);
  if (err != hipSuccess) {
    (void)hipGetLastError();
    pg_set_error("xgmi: hipIpcOpenMemHandle(rank %d's input, bid %llu): %s", q, (unsigned long long)d->bid,
                 hipGetErrorString(err));
    return NULL;
  }
  e[lru].base = p;
  e[lru].bid = d->bid;
  e[lru].peer_base = d->base;
  e[lru].peer_size = d->size;
  e[lru].stamp = x->clock;
  return (const char *)p + d->off;
}

/* Close this peer's cached mappings of large allocations other than `bid`
 * (not read by the current call). */
static void release_stale_imports(struct xgmi_ctx *x, int q, unsigned long long bid) {
  struct xg_import *e = &x->imp[q * XG_IMPORTS];
  for (int i = 0; i < XG_IMPORTS; ++i)
    if (e[i].base && e[i].bid != bid && e[i].peer_size >= XG_KEEP_MAX) {
      hipIpcCloseMemHandle(e[i].base);
      e[i].base = NULL;
      e[i].stamp = 0;
    }
}

/* A pushed call reads no peer input: close every large cached mapping, as the
 * slot-copy path does, so that an input freed by its owner gives its memory
 * back at the owner's next call whatever path that call takes. */
static void release_unread_imports(struct pg *pg, struct xgmi_ctx *x) {
  for (int q = 0; q < pg->world_size; ++q)
    if (q != pg->rank) release_stale_imports(x, q, 0);
}

static void drop_imports(struct pg *pg, struct xgmi_ctx *x) {
  if (!x->imp) return;
  for (int i = 0; i < pg->world_size * XG_IMPORTS; ++i)
    if (x->imp[i].base) { hipIpcCloseMemHandle(x->imp[i].base); x->imp[i].base = NULL; }
}

/* Make every rank's input readable; by_rank[q] = where rank q's input starts.
 * *zero_copy tells the caller to close with barrier(); *fail = this rank could
 * not map a peer (it must still join that barrier, then report -1). */
static int share_inputs(struct pg *pg, const void *in, size_t bytes, int in_dev, int may_alias_out,
                        const char **by_rank, int *zero_copy, int *fail) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xgmi_ctx *x = ctx_of(pg);
  const int W = pg->world_size, r = pg->rank, which = (int)(x->gen & 1);
  *zero_copy = 0;
  *fail = 0;
  double t0 = us_now();
  if (in_dev && pg_wait_producers(im, 1)) return -1;        /* peers read it after the barrier */
  double t1 = us_now();
  im->stats.sync_us += t1 - t0;
  if (x->zc && x->bar && bytes) {
    struct xg_desc mine;
    if (!in_dev || may_alias_out || x->force_copy || !export_input(x, in, &mine)) memset(&mine, 0, sizeof(mine));
    mine.nbytes = bytes;
    pg_trace(pg, "xgmi share: input %p exported=%d (bid %llu base %#llx size %llu)", in, mine.ok,
             (unsigned long long)mine.bid, (unsigned long long)mine.base, (unsigned long long)mine.size);
    descs(x)[r] = mine;
    if (barrier(pg)) return -1;
    struct xg_desc all[16];
    memcpy(all, descs(x), sizeof(struct xg_desc) * (size_t)W);
    int all_ok = 1, agree = 1;
    for (int q = 0; q < W; ++q) {
      agree &= all[q].nbytes == bytes;
      all_ok &= all[q].ok && all[q].off <= all[q].size && bytes <= all[q].size - all[q].off;
    }
    pg_trace(pg, "xgmi share: call %lu, %zu bytes, zero-copy %d", x->gen, bytes, all_ok);
    if (!agree) {
      /* ranks called with different counts (or types): every rank sees the same
       * table, so every rank fails this call here -- before any peer memory is
       * read with the wrong extent.  Meet once more so that nobody rewrites the
       * table before all have read it. */
      for (int q = 0; q < W; ++q)
        if (all[q].nbytes != bytes) {
          pg_set_error("xgmi: rank %d called with %llu bytes, this rank with %zu (counts must agree)", q,
                       (unsigned long long)all[q].nbytes, bytes);
          break;
        }
      barrier(pg);
      return -1;
    }
    im->stats.barrier_us += us_now() - t1;
    if (all_ok) {
      for (int q = 0; q < W; ++q) {
        by_rank[q] = q == r ? (const char *)in : import_input(x, q, &all[q]);
        pg_trace(pg, "xgmi share: rank %d's input at %p (bid %llu base %#llx size %llu off %llu)", q,
                 (const void *)by_rank[q], (unsigned long long)all[q].bid, (unsigned long long)all[q].base,
                 (unsigned long long)all[q].size, (unsigned long long)all[q].off);
        if (!by_rank[q]) *fail = 2;           /* soft: every rank redoes the call with the slot copy */
        if (q != r) release_stale_imports(x, q, all[q].bid);
      }
      *zero_copy = 1;
      im->stats.zero_copy = !*fail;
      return 0;
    }
    /* somebody's input cannot be shared in place: everybody copies, and no
     * mapping of a peer's input is read by this call */
    for (int q = 0; q < W; ++q)
      if (q != r) release_stale_imports(x, q, 0);
  }
  /* every rank reaches this point in this call (the choice above is collective) */
  if (bytes && ensure(pg, XG_REG_X, bytes)) return -1;
  char *xs = slot(x, XG_REG_X, r, which);
  pg_trace(pg, "xgmi share: call %lu slot copy of %zu bytes into X%d at %p", x->gen, bytes, which, (void *)xs);
  double t2 = us_now();
  if (bytes) {
    if (in_dev && ((uintptr_t)in & 3) == 0 && (bytes & 3) == 0) {
      /* device input: a copy kernel (the DMA engine path costs ~50 us to
       * start for a small copy) */
      void *d[1] = {xs};
      const void *sv[1] = {in};
      size_t nb[1] = {bytes};
      if (pgk_gather(d, sv, nb, 1, (void *)im->red)) { pg_set_error("xgmi: %s", pgk_last_error()); return -1; }
    } else if (!in_dev) {
      if (pg_copy_parallel(xs, in, bytes)) return -1;
    } else {
      PG_CHECK_HIP(hipMemcpyAsync(xs, in, bytes, hipMemcpyDeviceToDevice, im->red));
    }
    if (pg_stream_wait(im->red)) return -1;
  }
  double t3 = us_now();
  int rc = barrier(pg);
  im->stats.copy_us += t3 - t2;
  im->stats.barrier_us += us_now() - t3;
  for (int q = 0; q < W; ++q) by_rank[q] = slot(x, XG_REG_X, q, which);
  return rc;
}

/* End of a call: zero-copy inputs stay untouched until every peer is done.
 * That closing barrier also carries each rank's status (0 ok, 1 failed, 2
 * could not map a peer's input), so a failure on one rank is seen by every
 * rank and the callers stay in step.  Returns 0, -1 (some rank failed), or 1
 * (some rank could not map a peer, none failed otherwise: the caller redoes
 * the call on every rank with the slot copy, see xgmi_retry).  Slot-copy
 * calls meet here too (one more node-local barrier, ~1 us); only the
 * TCP-barrier fallback (PG_NO_SHM_BARRIER=1, never zero-copy) leaves a local
 * failure local. */
static int finish(struct pg *pg, int zero_copy, int fail) {
  struct xgmi_ctx *x = ctx_of(pg);
  int rc = 0, hard = fail == 1, soft = fail == 2;
  if (x->bar) {
    struct pg_impl *im = (struct pg_impl *)pg->impl;
    volatile int32_t *flags = (volatile int32_t *)((char *)x->bar + XG_FLAG_OFF) + (x->gen & 1) * 16;
    flags[pg->rank] = fail;
    double t = us_now();
    rc = barrier(pg);
    im->stats.barrier_us += us_now() - t;
    for (int q = 0; q < pg->world_size && !rc; ++q) {
      hard |= flags[q] == 1;
      soft |= flags[q] == 2;
    }
    if (hard && fail != 1 && !rc) pg_set_error("xgmi: a peer failed this call");
  } else if (zero_copy) {
    rc = barrier(pg);
  }
  x->gen++;
  if (rc || hard) return -1;
  return soft ? 1 : 0;
}

/* out = fold over ranks of this rank's block (at off_elems, len elements),
 * each ring part in its ring's order (include/pg_ext.h): bit-identical to the
 * P2P ring with the same PG_RINGS.  local_sources: every by_rank[] is this
 * GPU's own memory (push mode), so the fold may take the form tuned for local
 * HBM; peers' memory read over the links keeps the plain streaming form. */
static int fold_block(struct pg *pg, void *out, const char *const *by_rank, size_t off_elems, size_t len, int dt,
                      int op, int local_sources) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  if (!len) return 0;
  int W = pg->world_size, r = pg->rank;
  size_t es = pg_elem_size(dt);
  double tk = us_now();
  pg_trace(pg, "xgmi fold: %zu elements from %d ranks", len, W);
  const int one_launch = im->rings > 1 && len * es <= XG_FOLD_ONE_LAUNCH_MAX;
  if (one_launch) {
    /* small block: every ring part in one launch.  pgk_fold_blocks folds block
     * 0 of its sources as src[d] op src[2d] op ... op src[0] per part; with
     * src[j] = rank (r+j)'s block that is exactly the loop below. */
    const void *srcs[16];
    for (int j = 0; j < W; ++j) srcs[j] = by_rank[(r + j) % W] + off_elems * es;
    if (pgk_fold_blocks(out, srcs, W, len, len, im->rings, dt, op, (void *)im->red)) {
      pg_set_error("xgmi: %s", pgk_last_error());
      return -1;
    }
  }
  for (int g = 0; g < im->rings && !one_launch; ++g) {
    size_t po, pl;
    pg_block_part(len, im->rings, g, &po, &pl);
    if (!pl) continue;
    const void *srcs[16];
    const int d = pg_ring_offset(W, im->rings, g);
    for (int j = 0; j < W; ++j) {
      int q = ((r + (j + 1) * d) % W + W) % W;
      srcs[j] = by_rank[q] + (off_elems + po) * es;
      pg_trace(pg, "xgmi fold: part %d source %d = rank %d at %p", g, j, q, srcs[j]);
    }
    /* PG_KERNEL_TIMING=1: the fold's own kernel time (pg_stats.red_kernel_us),
     * as the ring executor stamps its reduce launches */
    void *t0 = NULL, *t1 = NULL;
    if (im->kt_on) {
      if (pg_kt_pair(im, &t0, &t1)) return -1;
      im->stats.red_kernel_bytes += (int64_t)((size_t)(W + 1) * pl * es);
    }
    if (pgk_fold_timed((char *)out + po * es, srcs, W, pl, dt, op, local_sources ? 0u : PGK_FOLD_REMOTE_SOURCES,
                       (void *)im->red, t0, t1)) {
      pg_set_error("xgmi: %s", pgk_last_error());
      return -1;
    }
    im->stats.reduce_launches += 1;
  }
  if (pg_stream_wait(im->red)) return -1;
  pg_kt_collect(im);
  pg_trace(pg, "xgmi fold: done");
  im->stats.kernel_us += us_now() - tk;
  im->stats.reduce_launches += one_launch;
  im->stats.reduce_elems += (int64_t)len * (W - 1);
  im->stats.bytes_recv += (int64_t)(len * es) * (W - 1);
  return 0;
}

static int overlaps(const void *a, size_t na, const void *b, size_t nb) {
  const char *x = (const char *)a, *y = (const char *)b;
  return na && nb && x < y + nb && y < x + na;
}

/* ---- push mode (PG_XGMI_MODE=push) --------------------------------------------
 * The same reduce-scatter with the xGMI traffic as writes instead of reads:
 * every rank writes block q of its input into rank q's X[parity] at piece
 * position r (one pgk_gather launch, all links at once), meets the others at
 * a barrier, and folds its own block from local memory in ring order.  Local
 * HBM traffic grows (W pieces read instead of one); which of the two is
 * faster depends on whether the links move pushed or pulled bytes faster,
 * which is what the link probe measures (pgx_xgmi_link_probe).  The choice
 * is collective: every rank flags whether it can push (device input, 4-byte
 * aligned, output not overlapping the input), and if any cannot, all of them
 * take the read path.  pieces[q] = block `rank` of rank q's contribution. */
static size_t push_stride(int count, int world, size_t es) {
  size_t b = ((size_t)count + (size_t)world - 1) / (size_t)world;
  return ((b ? b : 1) * es + 255) & ~(size_t)255;
}

static int push_inputs(struct pg *pg, const char *in, int count, int dt, int can, const char **pieces,
                       int *pushed) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xgmi_ctx *x = ctx_of(pg);
  const int W = pg->world_size, r = pg->rank, which = (int)(x->gen & 1);
  const size_t es = pg_elem_size(dt), stride = push_stride(count, W, es);
  *pushed = 0;
  double t0 = us_now();
  if (can && pg_wait_producers(im, 1)) return -1;          /* peers read it after the barrier */
  double t1 = us_now();
  im->stats.sync_us += t1 - t0;
  struct xg_desc mine;
  memset(&mine, 0, sizeof(mine));
  mine.ok = can && ((uintptr_t)in & 3) == 0;
  mine.nbytes = (size_t)count * es;
  descs(x)[r] = mine;
  if (barrier(pg)) return -1;
  int all_ok = 1, agree = 1;
  for (int q = 0; q < W; ++q) {
    all_ok &= descs(x)[q].ok;
    agree &= descs(x)[q].nbytes == mine.nbytes;
  }
  im->stats.barrier_us += us_now() - t1;
  if (!agree) {                                  /* as in share_inputs: everybody fails here */
    pg_set_error("xgmi: ranks called with different counts (counts must agree)");
    barrier(pg);
    return -1;
  }
  if (!all_ok) {
    /* everybody takes the read path, whose first step rewrites the descriptor
     * page: meet once more so that no rank does so before all have read it */
    return barrier(pg) ? -1 : 0;
  }
  if (ensure(pg, XG_REG_X, stride * (size_t)W)) return -1;
  void *dst[16];
  const void *src[16];
  size_t nb[16];
  int k = 0;
  for (int q = 0; q < W; ++q) {
    size_t qo, ql;
    pg_block_range(count, W, q, &qo, &ql);
    if (q == r) { pieces[q] = in + qo * es; continue; }
    pieces[q] = slot(x, XG_REG_X, r, which) + (size_t)q * stride;
    if (!ql) continue;
    dst[k] = slot(x, XG_REG_X, q, which) + (size_t)r * stride;
    src[k] = in + qo * es;
    nb[k++] = ql * es;
  }
  double t2 = us_now();
  pg_trace(pg, "xgmi push: %d pieces", k);
  if (k && pgk_gather(dst, src, nb, k, (void *)im->red)) { pg_set_error("xgmi: %s", pgk_last_error()); return -1; }
  if (pg_stream_wait(im->red)) return -1;
  double t3 = us_now();
  im->stats.copy_us += t3 - t2;
  im->stats.bytes_sent += (int64_t)((size_t)count * es);
  if (barrier(pg)) return -1;                                /* every piece has landed */
  im->stats.barrier_us += us_now() - t3;
  *pushed = 1;
  return 0;
}

static int rs_once(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xgmi_ctx *x = ctx_of(pg);
  size_t es = pg_elem_size(dt), bytes = (size_t)count * es, off, len;
  pg_block_range(count, pg->world_size, pg->rank, &off, &len);
  int rd = is_dev(recvbuf), zc = 0, fail = 0, pushed = 0;
  const char *by_rank[16];
  size_t fold_off = off;
  if (x->push && bytes) {
    int can = is_dev(sendbuf) && !overlaps(sendbuf, bytes, recvbuf, len * es);
    if (push_inputs(pg, (const char *)sendbuf, count, dt, can, by_rank, &pushed)) return -1;
    if (pushed) fold_off = 0;                   /* by_rank[q] point at block `rank` itself */
  }
  if (pushed) release_unread_imports(pg, x);
  if (!pushed && share_inputs(pg, sendbuf, bytes, is_dev(sendbuf), overlaps(sendbuf, bytes, recvbuf, len * es),
                              by_rank, &zc, &fail))
    return -1;
  void *out = recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, len * es)) fail = 1;   /* reported by finish() on every rank */
    out = im->dout;
  }
  if (!fail && fold_block(pg, out, by_rank, fold_off, len, dt, op, pushed)) fail = 1;
  int fin = finish(pg, zc, fail);
  if (fin) return fin;
  if (!rd && len && pg_copy_parallel(recvbuf, out, len * es)) return -1;
  return 0;
}

/* Gather block q of every rank (bases by_rank[q], uniform: blocks of `count`
 * at base + 0; else the reduce-scatter partition at base + off(q)) into
 * full + off(q), one launch (pgk_gather). */
static int gather(struct pg *pg, char *full, const char *const *by_rank, int count, int uniform, int dt) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  size_t es = pg_elem_size(dt);
  void *dst[16];
  const void *src[16];
  size_t nb[16];
  int k = 0;
  for (int q = 0; q < pg->world_size; ++q) {
    size_t off, len;
    if (uniform) { off = (size_t)q * (size_t)count; len = (size_t)count; }
    else pg_block_range(count, pg->world_size, q, &off, &len);
    if (!len) continue;
    dst[k] = full + off * es;
    src[k] = by_rank[q] + (uniform ? 0 : off * es);
    nb[k] = len * es;
    ++k;
  }
  double tk = us_now();
  if (pgk_gather(dst, src, nb, k, (void *)im->red)) { pg_set_error("xgmi: %s", pgk_last_error()); return -1; }
  if (pg_stream_wait(im->red)) return -1;
  im->stats.kernel_us += us_now() - tk;
  return 0;
}

static int ag_once(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  size_t es = pg_elem_size(dt), slot_bytes = (size_t)count * es, total = slot_bytes * (size_t)pg->world_size;
  int rd = is_dev(recvbuf), zc, fail;
  const void *mine = sendbuf ? sendbuf : (const char *)recvbuf + (size_t)pg->rank * slot_bytes;
  const char *by_rank[16];
  if (share_inputs(pg, mine, slot_bytes, sendbuf ? is_dev(sendbuf) : rd, overlaps(mine, slot_bytes, recvbuf, total),
                   by_rank, &zc, &fail))
    return -1;
  char *full = (char *)recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, total)) fail = 1;
    full = (char *)im->dout;
  }
  if (!fail && gather(pg, full, by_rank, count, 1, dt)) fail = 1;
  int fin = finish(pg, zc, fail);
  if (fin) return fin;
  if (!rd && total && pg_copy_parallel(recvbuf, full, total)) return -1;
  im->stats.bytes_recv += (int64_t)(total - slot_bytes);
  return 0;
}

static int ar_once(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xgmi_ctx *x = ctx_of(pg);
  size_t es = pg_elem_size(dt), bytes = (size_t)count * es, off, len;
  pg_block_range(count, pg->world_size, pg->rank, &off, &len);
  int rd = is_dev(recvbuf), which = (int)(x->gen & 1), zc = 0, fail = 0, pushed = 0;
  const char *by_rank[16];
  size_t fold_off = off;
  if (x->push && bytes > x->oneshot_max) {      /* same branch on every rank: same count */
    int can = is_dev(sendbuf) && !overlaps(sendbuf, bytes, recvbuf, bytes);
    if (push_inputs(pg, (const char *)sendbuf, count, dt, can, by_rank, &pushed)) return -1;
    if (pushed) fold_off = 0;
  }
  if (pushed) release_unread_imports(pg, x);
  if (!pushed && share_inputs(pg, sendbuf, bytes, is_dev(sendbuf), overlaps(sendbuf, bytes, recvbuf, bytes), by_rank,
                              &zc, &fail))
    return -1;
  char *full = (char *)recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, bytes)) fail = 1;
    full = (char *)im->dout;
  }
  if (bytes <= x->oneshot_max) {
    /* small message: every rank folds the whole vector itself, each block in
     * its ring order -- one launch, no second barrier */
    if (!fail && count) {
      const void *srcs[16];
      for (int q = 0; q < pg->world_size; ++q) srcs[q] = by_rank[q];
      size_t blk = ((size_t)count + (size_t)pg->world_size - 1) / (size_t)pg->world_size;
      double tk = us_now();
      if (pgk_fold_blocks(full, srcs, pg->world_size, (size_t)count, blk, im->rings, dt, op, (void *)im->red) ||
          pg_stream_wait(im->red)) {
        pg_set_error("xgmi: %s", pgk_last_error());
        fail = 1;
      }
      im->stats.kernel_us += us_now() - tk;
    }
  } else {
    /* my block of the result goes to R[which] so that every rank can gather it */
    if (ensure(pg, XG_REG_R, bytes)) return -1;
    if (!fail && fold_block(pg, slot(x, XG_REG_R, pg->rank, which) + off * es, by_rank, fold_off, len, dt, op, 0))
      fail = 1;
    double tb = us_now();
    if (barrier(pg)) return -1;
    im->stats.barrier_us += us_now() - tb;
    const char *res_by_rank[16];
    for (int q = 0; q < pg->world_size; ++q) res_by_rank[q] = slot(x, XG_REG_R, q, which);
    if (!fail && gather(pg, full, res_by_rank, count, 0, dt)) fail = 1;
  }
  int fin = finish(pg, zc, fail);
  if (fin) return fin;
  if (!rd && bytes && pg_copy_parallel(recvbuf, full, bytes)) return -1;
  return 0;
}

/* A call some rank could not zero-copy (a peer's input failed to map: an IPC
 * open that ROCm refused) is redone once on every rank with the slot copy,
 * which needs no mapping of caller memory; every rank learned of it at the
 * same closing barrier, so all of them retry.  The first attempt wrote
 * nothing that the retry does not overwrite (in-place calls never take
 * zero-copy). */
static int xgmi_retry(struct pg *pg, int first) {
  struct xgmi_ctx *x = ctx_of(pg);
  if (first != 1) return first;
  x->force_copy = 1;
  ((struct pg_impl *)pg->impl)->stats.retried = 1;
  ((struct pg_impl *)pg->impl)->calls_redone++;
  pg_trace(pg, "xgmi: a peer's input could not be mapped; redoing the call with the slot copy");
  return 0;
}

int pg_xgmi_reduce_scatter(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  int rc = rs_once(pg, sendbuf, recvbuf, count, dt, op);
  if (rc == 1 && xgmi_retry(pg, rc) == 0) rc = rs_once(pg, sendbuf, recvbuf, count, dt, op);
  ctx_of(pg)->force_copy = 0;
  return rc == 0 ? 0 : -1;
}

int pg_xgmi_all_gather(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt) {
  int rc = ag_once(pg, sendbuf, recvbuf, count, dt);
  if (rc == 1 && xgmi_retry(pg, rc) == 0) rc = ag_once(pg, sendbuf, recvbuf, count, dt);
  ctx_of(pg)->force_copy = 0;
  return rc == 0 ? 0 : -1;
}

int pg_xgmi_all_reduce(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  int rc = ar_once(pg, sendbuf, recvbuf, count, dt, op);
  if (rc == 1 && xgmi_retry(pg, rc) == 0) rc = ar_once(pg, sendbuf, recvbuf, count, dt, op);
  ctx_of(pg)->force_copy = 0;
  return rc == 0 ? 0 : -1;
}

/* ---- link probe ----------------------------------------------------------------
 * Measures what the transport's traffic rides on (the rule followed: "measure
 * the unidirectional per-link rate with a P2P probe before quoting roofline for
 * the ring").  Every rank runs the same four phases, each `reps` copy launches
 * of `bytes` (pgk_gather) timed with HIP events, with barriers in between:
 *   0 read one:  peer (r+1)'s X0  -> my X1              (one link, pulled)
 *   1 write one: my X0            -> peer (r+1)'s X1     (one link, pushed)
 *   2 read all:  bytes/(W-1) from every peer's X0 -> my X1   (all links, pulled)
 *   3 write all: bytes/(W-1) of my X0 -> every peer's X1, at my own offset
 * gbs[phase] = bytes * reps / time on this rank (1e9 B/s).  Collective. */
int pgx_xgmi_link_probe(void *pg_handle, size_t bytes, int reps, double *gbs) {
  struct pg *pg = (struct pg *)pg_handle;
  if (!pg || !pg->impl || pg->transport != PG_TRANSPORT_XGMI || pg->world_size < 2 || !gbs || reps < 1 ||
      bytes < 4096 || (bytes & 4095)) {
    pg_set_error("pgx_xgmi_link_probe: needs an xgmi handle with world >= 2, bytes a multiple of 4 KiB, reps >= 1");
    return -1;
  }
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct xgmi_ctx *x = ctx_of(pg);
  const int W = pg->world_size, r = pg->rank, right = (r + 1) % W;
  if (ensure(pg, XG_REG_X, bytes)) return -1;
  PG_CHECK_HIP(hipMemsetAsync(slot(x, XG_REG_X, r, 0), r + 1, bytes, im->red));
  PG_CHECK_HIP(hipStreamSynchronize(im->red));
  size_t part = (bytes / (size_t)(W - 1)) & ~(size_t)15;
  hipEvent_t e0, e1;
  PG_CHECK_HIP(hipEventCreate(&e0));
  PG_CHECK_HIP(hipEventCreate(&e1));
  /* A rank whose launch or event call fails keeps meeting the others at every
   * phase's barriers (it only skips its launches), and the outcome is agreed at
   * the end: all ranks fail together instead of the healthy ones waiting out
   * the barrier timeout for the one that left. */
  int rc = 0, lost = 0;
  const char *fail_hook = getenv("PG_XGMI_FAIL_PROBE");     /* test hook: this rank's phase 1 fails */
  for (int phase = 0; phase < 4; ++phase) {
    void *dst[16];
    const void *src[16];
    size_t nb[16];
    int k = 0;
    if (phase == 0) { dst[0] = slot(x, XG_REG_X, r, 1); src[0] = slot(x, XG_REG_X, right, 0); nb[0] = bytes; k = 1; }
    if (phase == 1) { dst[0] = slot(x, XG_REG_X, right, 1); src[0] = slot(x, XG_REG_X, r, 0); nb[0] = bytes; k = 1; }
    for (int q = 0; phase >= 2 && q < W; ++q) {
      if (q == r) continue;
      int my_idx = r < q ? r : r - 1;           /* my position among q's peers */
      int q_idx = q < r ? q : q - 1;            /* q's position among mine     */
      if (phase == 2) { dst[k] = slot(x, XG_REG_X, r, 1) + (size_t)q_idx * part; src[k] = slot(x, XG_REG_X, q, 0); }
      else { dst[k] = slot(x, XG_REG_X, q, 1) + (size_t)my_idx * part; src[k] = slot(x, XG_REG_X, r, 0); }
      nb[k++] = part;
    }
    if (barrier(pg)) { lost = 1; break; }
    if (rc == 0 && phase == 1 && fail_hook && *fail_hook && atoi(fail_hook) == r) {
      pg_set_error("xgmi probe: failure injected on rank %d (PG_XGMI_FAIL_PROBE)", r);
      rc = -1;
    }
    if (rc == 0 && pgk_gather(dst, src, nb, k, (void *)im->red)) { pg_set_error("xgmi probe: %s", pgk_last_error()); rc = -1; }
    if (rc == 0 && (hipEventRecord(e0, im->red) != hipSuccess)) rc = -1;
    for (int i = 0; rc == 0 && i < reps; ++i)
      if (pgk_gather(dst, src, nb, k, (void *)im->red)) { pg_set_error("xgmi probe: %s", pgk_last_error()); rc = -1; }
    float ms = 0.f;
    if (rc == 0 && (hipEventRecord(e1, im->red) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                    hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
      rc = -1;
    if (rc) (void)hipStreamSynchronize(im->red);   /* whatever was launched has left the slots */
    size_t moved = phase < 2 ? bytes : part * (size_t)(W - 1);
    gbs[phase] = rc == 0 && ms > 0.f ? (double)moved * reps / (ms * 1e-3) / 1e9 : 0.0;
    if (barrier(pg)) { lost = 1; break; }      /* nobody overwrites a slot a peer still reads */
  }
  if (lost) rc = -1;                           /* a barrier failed: the ranks are no longer in step */
  else if (!all_ranks_ok(pg, rc == 0) && rc == 0) {
    pg_set_error("xgmi probe: a peer's probe failed");
    rc = -1;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (rc && !pg_last_error()[0]) pg_set_error("xgmi probe: HIP event failure");
  return rc;
}
