/*
 * pg.c -- public API of libpg_amd.so (include/pg.h): handle lifecycle,
 * argument validation, host<->HBM staging, and dispatch to
 *   SELF      world_size == 1: the reference's copy fast paths
 *             (src/pg.c:269-272, :302-306, :328-330)
 *   LOOPBACK  the reference's single-process mock schedule
 *             (src/pg.c:264-321), every reduce on the gfx950 kernel
 *   ring      RCCL over xGMI (or in-process virtual ranks): pg_plan.c's
 *             schedule executed by pg_exec.c
 *
 * Validation and return codes follow the reference exactly
 * (src/pg.c:267, :295, :325): NULL handle/buffer, count < 0 or an unknown
 * datatype -> -1.  An operation other than OP_SUM multiplies, as the
 * reference's `(op == OP_SUM) ? add : mul` does (src/pg.c:154,157).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "pg_impl.h"

/* ---- errors ----------------------------------------------------------------- */

static __thread char g_pg_err[512];

void pg_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_pg_err, sizeof(g_pg_err), fmt, ap);
  va_end(ap);
  if (getenv("PG_DEBUG")) fprintf(stderr, "[pg] %s\n", g_pg_err);
}

const char *pg_last_error(void) { return g_pg_err; }

/* PG_TRACE=1: one stderr line per transport phase (rank, monotonic time), to
 * name the phase a stalled multi-process call is in.  PG_TRACE_FILE=prefix
 * instead writes them, fully buffered, to prefix.<pid> (flushed at exit): far
 * less perturbation when chasing a timing-dependent fault. */
static FILE *g_trace = NULL;
static int g_trace_on = -1;

void pg_trace(const struct pg *pg, const char *fmt, ...) {
  if (g_trace_on < 0) {
    const char *f = getenv("PG_TRACE_FILE"), *e = getenv("PG_TRACE");
    g_trace_on = 0;
    if (f && *f) {
      char path[512];
      snprintf(path, sizeof(path), "%s.%d", f, (int)getpid());
      g_trace = fopen(path, "w");
      if (g_trace) { setvbuf(g_trace, NULL, _IOFBF, 1 << 20); g_trace_on = 1; }
    } else if (e && *e == '1') {
      g_trace = stderr;
      g_trace_on = 1;
    }
  }
  if (!g_trace_on) return;
  char msg[320];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(msg, sizeof(msg), fmt, ap);
  va_end(ap);
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  fprintf(g_trace, "[pg r%d %ld.%06ld] %s\n", pg ? pg->rank : -1, (long)ts.tv_sec, ts.tv_nsec / 1000L, msg);
  if (g_trace == stderr) fflush(stderr);
}

/* ---- small helpers ---------------------------------------------------------- */

size_t pg_elem_size(int dt) {                 /* reference src/pg.c:109-115 */
  return dt == DT_INT32 ? 4 : dt == DT_DOUBLE ? 8 : 0;
}

static double now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e6 + (double)ts.tv_nsec * 1e-3;
}

/* Wait for `s` to drain: poll hipStreamQuery for up to PG_SPIN_US (default
 * 200 us) -- a short collective finishes well inside that, without the wake-up
 * latency of a blocking wait -- then fall back to hipStreamSynchronize.  No
 * process-wide scheduling flags are touched. */
int pg_stream_wait(hipStream_t s) {
  static double spin_us = -1.0;
  if (spin_us < 0) {
    const char *e = getenv("PG_SPIN_US");
    spin_us = (e && *e) ? atof(e) : 200.0;
  }
  double t0 = spin_us > 0 ? now_us() : 0;
  while (spin_us > 0) {
    hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) {
      pg_set_error("stream wait: %s", hipGetErrorString(e));
      return -1;
    }
    if (now_us() - t0 > spin_us) break;
    __builtin_ia32_pause();
  }
  PG_CHECK_HIP(hipStreamSynchronize(s));
  return 0;
}

/* Device buffers: the caller's producers are the work it enqueued on the null
 * stream before the call (work on other
 * streams the caller orders before the call itself).  The collective must not
 * read its buffers before that work ends.
 * An idle null stream (the usual case: the caller synchronised, or produced
 * the input by a blocking copy) is a host-side query and costs no GPU round
 * trip.  Otherwise the ring's streams wait for it on the device (host_wait =
 * 0): nothing blocks the host, and the first transfer is queued behind the
 * producer.  A transport whose peers read this rank's buffers once it reaches
 * a host barrier (xgmi) waits on the host instead (host_wait = 1).  Either way
 * it is narrower than a hipDeviceSynchronize(): non-blocking streams of the
 * process that the caller did not order before the call (another thread's
 * work, RCCL's) are not waited for
 * (tests/test_api_gpu.py::test_device_input_behind_slow_producer).
 * PG_PRODUCER_SYNC=device restores the reference's fully synchronous contract
 * (src/pg.c:323-339 is a host call on host memory: whatever produced the
 * buffers has finished when it is entered): every stream of the device is
 * waited for at entry, so inputs written on any stream are safe. */
int pg_wait_producers(struct pg_impl *im, int host_wait) {
  static int skip = -1;                 /* test hook: PG_TEST_SKIP_PRODUCER_WAIT=1 shows the race it prevents */
  static int device_sync = 0;
  if (skip < 0) {
    const char *e = getenv("PG_TEST_SKIP_PRODUCER_WAIT"), *m = getenv("PG_PRODUCER_SYNC");
    if (m && *m && strcmp(m, "device") != 0 && strcmp(m, "null") != 0) {
      pg_set_error("PG_PRODUCER_SYNC=%s: expected null or device", m);
      return -1;
    }
    device_sync = m && strcmp(m, "device") == 0;
    skip = e && *e == '1';
  }
  if (skip) return 0;
  if (device_sync) { PG_CHECK_HIP(hipDeviceSynchronize()); return 0; }
  hipError_t q = hipStreamQuery(NULL);
  if (q == hipSuccess) return 0;
  if (q != hipErrorNotReady) { pg_set_error("null stream query: %s", hipGetErrorString(q)); return -1; }
  if (host_wait) return pg_stream_wait(NULL);
  PG_CHECK_HIP(hipEventRecord(im->entry_ev, NULL));
  PG_CHECK_HIP(hipStreamWaitEvent(im->comm, im->entry_ev, 0));
  PG_CHECK_HIP(hipStreamWaitEvent(im->red, im->entry_ev, 0));
  return 0;
}

int pg_ensure(void **buf, size_t *cap, size_t bytes) {
  if (bytes <= *cap && (*buf || bytes == 0)) return 0;
  if (*buf) { hipFree(*buf); *buf = NULL; *cap = 0; }
  size_t want = (bytes + 0xFFFFF) & ~(size_t)0xFFFFF;     /* 1 MiB granules */
  PG_CHECK_HIP(hipMalloc(buf, want));
  *cap = want;
  return 0;
}

/* HIP device or managed memory?  Anything else is treated as host memory and
 * staged through HBM. */
int pg_is_device_ptr(const void *p) {
  if (!p) return 0;
  hipPointerAttribute_t a;
  memset(&a, 0, sizeof(a));
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.isManaged;
}

int pg_ranges_overlap(const void *a, size_t na, const void *b, size_t nb) {
  const char *x = (const char *)a, *y = (const char *)b;
  return na && nb && x < y + nb && y < x + na;
}

/* Host<->device copies of large buffers, optionally split over
 * PG_COPY_THREADS threads (default 1: measured on MI355X + EPYC 9575F, one
 * hipMemcpy of pageable memory already runs at the PCIe Gen5 x16 limit,
 * ~53 GB/s, and 2/4/8 threads measured 52/51/49 GB/s; tools/copy_threads_probe.py).
 * Kept for hosts whose single-thread staging is slower than the link. */
struct copy_job {
  void *dst;
  const void *src;
  size_t bytes;
  int device;
  hipError_t err;
};

static void *copy_thread(void *arg) {
  struct copy_job *j = (struct copy_job *)arg;
  j->err = hipSetDevice(j->device);
  if (j->err == hipSuccess) j->err = hipMemcpy(j->dst, j->src, j->bytes, hipMemcpyDefault);
  /* a host-to-device hipMemcpy may return once the bytes are staged, before
   * they land; the consumers run on non-blocking streams, so wait for them */
  if (j->err == hipSuccess) j->err = hipStreamSynchronize(NULL);
  return NULL;
}

int pg_copy_parallel(void *dst, const void *src, size_t bytes) {
  static int nthreads = -1;
  if (nthreads < 0) {
    const char *e = getenv("PG_COPY_THREADS");
    nthreads = (e && *e) ? atoi(e) : 1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 16) nthreads = 16;
  }
  if (nthreads == 1 || bytes < (32u << 20)) {
    PG_CHECK_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
    PG_CHECK_HIP(hipStreamSynchronize(NULL));                 /* as in copy_thread */
    return 0;
  }
  int dev = 0;
  PG_CHECK_HIP(hipGetDevice(&dev));
  struct copy_job jobs[16];
  pthread_t tid[16];
  size_t slice = ((bytes / (size_t)nthreads) + 4095) & ~(size_t)4095;
  int n = 0;
  for (size_t off = 0; off < bytes && n < nthreads; off += slice, ++n) {
    jobs[n].dst = (char *)dst + off;
    jobs[n].src = (const char *)src + off;
    jobs[n].bytes = bytes - off < slice ? bytes - off : slice;
    jobs[n].device = dev;
    jobs[n].err = hipSuccess;
  }
  int started = 0;
  for (int i = 1; i < n; ++i, ++started)
    if (pthread_create(&tid[i], NULL, copy_thread, &jobs[i])) break;
  copy_thread(&jobs[0]);
  for (int i = 1; i <= started; ++i) pthread_join(tid[i], NULL);
  for (int i = started + 1; i < n; ++i) copy_thread(&jobs[i]);   /* threads that failed to start */
  for (int i = 0; i < n; ++i)
    if (jobs[i].err != hipSuccess) { pg_set_error("copy: %s", hipGetErrorString(jobs[i].err)); return -1; }
  return 0;
}

static int copy_any(void *dst, const void *src, size_t bytes) {
  if (!bytes || dst == src) return 0;
  int dd = pg_is_device_ptr(dst), sd = pg_is_device_ptr(src);
  if (!dd && !sd) { memmove(dst, src, bytes); return 0; }
  if (dd != sd) return pg_copy_parallel(dst, src, bytes);      /* crosses PCIe */
  /* device to device: hipMemcpy may return before the copy has landed, and
   * the comm / reduce streams are non-blocking (no implicit wait on the null
   * stream), so a send enqueued next could read the old bytes: wait here */
  PG_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, NULL));
  PG_CHECK_HIP(hipStreamSynchronize(NULL));
  return 0;
}

int pg_timed_copy(void *dst, const void *src, size_t bytes, double *acc_us) {
  double t = now_us();
  int rc = copy_any(dst, src, bytes);
  *acc_us += now_us() - t;
  return rc;
}

/* ---- handle ----------------------------------------------------------------- */

int pg_impl_create(struct pg *pg) {
  struct pg_impl *im = (struct pg_impl *)calloc(1, sizeof(*im));
  if (!im) { pg_set_error("out of host memory"); return -1; }
  pg->impl = im;
  im->pg = pg;
  PG_CHECK_HIP(hipSetDevice(pg->device));
  PG_CHECK_HIP(hipStreamCreateWithFlags(&im->comm, hipStreamNonBlocking));
  PG_CHECK_HIP(hipStreamCreateWithFlags(&im->red, hipStreamNonBlocking));
  for (int i = 0; i < PG_RECV_EVENTS; ++i)
    PG_CHECK_HIP(hipEventCreateWithFlags(&im->recv_ev[i], hipEventDisableTiming));
  PG_CHECK_HIP(hipEventCreateWithFlags(&im->join_ev, hipEventDisableTiming));
  PG_CHECK_HIP(hipEventCreateWithFlags(&im->entry_ev, hipEventDisableTiming));
  PG_CHECK_HIP(hipEventCreate(&im->t0));
  PG_CHECK_HIP(hipEventCreate(&im->t1));
  const char *e = getenv("PG_EAGER_ONESHOT");
  im->eager_oneshot = !(e && *e && atoi(e) == 0);
  /* PG_ALGO: ring | direct; unset: direct when every rank is on this node
   * (connect_process_group), the ring for in-process virtual ranks */
  im->algo = PG_ALGO_RING;
  e = getenv("PG_ALGO");
  if (e && *e) {
    if (strcmp(e, "direct") == 0) im->algo = PG_ALGO_DIRECT;
    else if (strcmp(e, "ring") != 0) { pg_set_error("PG_ALGO=%s: expected ring or direct", e); return -1; }
  } else if (pg->hosts && pg_default_transport(pg) == PG_TRANSPORT_XGMI) {
    im->algo = PG_ALGO_DIRECT;                   /* one node, W <= 16: every peer one link away */
  }
  im->red_bytes = PG_DEFAULT_REDUCE_BYTES;
  e = getenv("PG_REDUCE_BYTES");
  if (e && *e) im->red_bytes = (size_t)strtoull(e, NULL, 0);
  im->rings = 2;
  e = getenv("PG_RINGS");
  if (e && *e) {
    im->rings = atoi(e);
    if (im->rings < 1 || im->rings > PG_MAX_RINGS) { pg_set_error("PG_RINGS=%s: expected 1 .. %d", e, PG_MAX_RINGS); return -1; }
  }
  return 0;
}

void pg_impl_destroy(struct pg *pg) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  if (!im) return;
  if (im->comm) hipStreamSynchronize(im->comm);
  if (im->red) hipStreamSynchronize(im->red);
  if (pg->transport == PG_TRANSPORT_XGMI) pg_xport_xgmi_destroy(pg);
  if (im->ops && im->ops->destroy) im->ops->destroy(im);
  pg_boot_close(im->boot_fds, pg->world_size);
  im->boot_fds = NULL;
  for (int i = 0; i < im->n_red_ev; ++i) hipEventDestroy(im->red_ev[i]);
  free(im->red_ev);
  for (int i = 0; i < im->n_round_ev; ++i) hipEventDestroy(im->round_ev[i]);
  free(im->round_ev);
  for (int i = 0; i < PG_RECV_EVENTS; ++i) if (im->recv_ev[i]) hipEventDestroy(im->recv_ev[i]);
  if (im->join_ev) hipEventDestroy(im->join_ev);
  if (im->entry_ev) hipEventDestroy(im->entry_ev);
  for (int i = 0; i < im->n_kt_ev; ++i) hipEventDestroy(im->kt_ev[i]);
  free(im->kt_ev);
  if (im->t0) hipEventDestroy(im->t0);
  if (im->t1) hipEventDestroy(im->t1);
  if (im->comm) hipStreamDestroy(im->comm);
  if (im->red) hipStreamDestroy(im->red);
  free(im->pend);
  free(im->ranges);
  for (int i = 0; i < 2; ++i) if (im->stage[i]) hipFree(im->stage[i]);
  if (im->dsrc) hipFree(im->dsrc);
  if (im->dout) hipFree(im->dout);
  if (im->ebuf) hipFree(im->ebuf);
  free(im->steps);
  free(im);
  pg->impl = NULL;
}

static void pg_defaults(struct pg *pg) {
  pg->chunk_bytes = PG_DEFAULT_CHUNK_BYTES;
  pg->eager_max = PG_DEFAULT_EAGER_MAX;
  pg->inflight = PG_DEFAULT_INFLIGHT;
  pg->port = PG_DEFAULT_PORT;
  pg_apply_env(pg);                 /* env after defaults: env wins */
}

/* Without PG_TRANSPORT: the xgmi transport when every rank is on this node
 * (every entry of the server list names the same host) and W <= 16 -- it is
 * the one exercised with real processes (tests/test_xgmi_gpu.py) and it pulls
 * over all of a GPU's links at once -- else the RCCL ring, which also crosses
 * nodes.  Both give the same bits (every transport folds in the ring's order). */
int pg_default_transport(const struct pg *pg) {
  if (pg->world_size > 16) return PG_TRANSPORT_RCCL;
  for (int i = 1; i < pg->world_size; ++i)
    if (strcmp(pg->hosts[i], pg->hosts[0]) != 0) return PG_TRANSPORT_RCCL;
  return PG_TRANSPORT_XGMI;
}

int connect_process_group(const char *serverlist, void **out_handle) {
  if (!serverlist || !out_handle) { pg_set_error("connect_process_group: NULL argument"); return -1; }
  struct pg *pg = (struct pg *)calloc(1, sizeof(*pg));
  if (!pg) return -1;
  if (pg_parse_hosts(serverlist, &pg->hosts, &pg->world_size)) goto fail;
  if (pg_discover_rank(pg->hosts, pg->world_size, &pg->rank)) goto fail;
  pg_defaults(pg);
  if (pg_discover_device(pg->rank, &pg->device)) goto fail;

  const char *tr = getenv("PG_TRANSPORT");
  if (pg->world_size == 1) pg->transport = PG_TRANSPORT_SELF;
  else if (tr && strcmp(tr, "loopback") == 0) pg->transport = PG_TRANSPORT_LOOPBACK;
  else if (tr && strcmp(tr, "xgmi") == 0) pg->transport = PG_TRANSPORT_XGMI;
  else if (tr && strcmp(tr, "rccl") == 0) pg->transport = PG_TRANSPORT_RCCL;
  else if (!tr || !*tr) pg->transport = pg_default_transport(pg);
  else { pg_set_error("PG_TRANSPORT=%s: expected rccl, xgmi or loopback", tr); goto fail; }

  if (pg_impl_create(pg)) goto fail;
  if (pg->transport == PG_TRANSPORT_RCCL && pg_xport_rccl_init(pg)) goto fail;
  if (pg->transport == PG_TRANSPORT_XGMI) {
    int rc = pg_xport_xgmi_init(pg);
    if (rc == 1 && (!tr || !*tr)) {
      /* xgmi was this library's choice, not the caller's, and the ranks cannot
       * map each other's memory (every rank learned that together): take the
       * RCCL transport over the same bootstrap star instead */
      pg_trace(pg, "xgmi unavailable (%s): falling back to the rccl transport", pg_last_error());
      pg_xport_xgmi_destroy(pg);
      pg->transport = PG_TRANSPORT_RCCL;
      if (pg_xport_rccl_init(pg)) goto fail;
    } else if (rc) {
      goto fail;
    }
  }
  *out_handle = pg;
  return 0;
fail:
  fprintf(stderr, "Process group connection failed during setup: %s\n", pg_last_error());
  pg_close(pg);
  return -1;
}

int pg_connect_local(int rank, int world, int transport, void **out_handle) {
  if (!out_handle || world < 1 || rank < 0 || rank >= world) { pg_set_error("pg_connect_local: bad arguments"); return -1; }
  if (transport != PG_TRANSPORT_LOOPBACK && transport != PG_TRANSPORT_SELF) {
    pg_set_error("pg_connect_local: transport must be LOOPBACK or SELF");
    return -1;
  }
  if (transport == PG_TRANSPORT_SELF && world != 1) { pg_set_error("pg_connect_local: SELF needs world 1"); return -1; }
  struct pg *pg = (struct pg *)calloc(1, sizeof(*pg));
  if (!pg) return -1;
  pg->rank = rank;
  pg->world_size = world;
  pg_defaults(pg);
  if (hipGetDevice(&pg->device) != hipSuccess) { pg_set_error("no HIP device"); free(pg); return -1; }
  pg->transport = world == 1 ? PG_TRANSPORT_SELF : transport;
  if (pg_impl_create(pg)) { pg_close(pg); return -1; }
  *out_handle = pg;
  return 0;
}

int pg_close(void *pg_handle) {
  struct pg *pg = (struct pg *)pg_handle;
  if (!pg) return 0;
  pg_impl_destroy(pg);
  if (g_trace && g_trace != stderr) fflush(g_trace);   /* a host that ends with _exit() keeps its trace */
  if (pg->hosts) {
    for (int i = 0; i < pg->world_size; ++i) free(pg->hosts[i]);
    free(pg->hosts);
  }
  free(pg);
  return 0;
}

int pg_get_stats(void *pg_handle, struct pg_stats *out) {
  struct pg *pg = (struct pg *)pg_handle;
  if (!pg || !pg->impl || !out) return -1;
  const struct pg_impl *im = (const struct pg_impl *)pg->impl;
  *out = im->stats;
  out->calls_redone = im->calls_redone;
  out->transport = pg->transport;
  out->algo_direct = im->algo == PG_ALGO_DIRECT;
  if (pg->transport == PG_TRANSPORT_XGMI) {
    int push = 0;
    double rd = 0, wr = 0;
    if (pgx_xgmi_mode(pg, &push, &rd, &wr) == 0) {
      out->xgmi_push = push;
      out->xgmi_mode_auto = rd > 0 || wr > 0;
      out->probe_read_gbs = rd;
      out->probe_write_gbs = wr;
    }
  }
  return 0;
}

/* PG_KERNEL_TIMING=1: every reduce launch of the ring executor carries its own
 * kernel timestamps (pgk_reduce_ranges start/stop events); the call's summed
 * kernel time lands in pg_stats.red_kernel_us.  Stamping costs a few us per
 * launch, so it is for measuring calls, not for timed ones. */
static void stats_begin(struct pg_impl *im) {
  memset(&im->stats, 0, sizeof(im->stats));
  const char *e = getenv("PG_KERNEL_TIMING");
  im->kt_on = e && *e == '1';
  im->kt_used = 0;
}

/* After the streams drained: sum the stamped launches of this call. */
void pg_kt_collect(struct pg_impl *im) {
  for (int u = 0; u < im->kt_used; ++u) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, im->kt_ev[2 * u], im->kt_ev[2 * u + 1]) == hipSuccess)
      im->stats.red_kernel_us += (double)ms * 1e3;
  }
  im->kt_used = 0;
}

static int sync_ring(struct pg_impl *im, int timed) {
  if (pg_stream_wait(im->comm) || pg_stream_wait(im->red)) return -1;
  if (timed) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, im->t0, im->t1) == hipSuccess) im->stats.ring_us += (double)ms * 1e3;
  }
  pg_kt_collect(im);
  return 0;
}

static int plan_into(struct pg_impl *im, int is_rs, int count, int dt, int alias, int uniform) {
  struct pg *pg = im->pg;
  int n = is_rs ? pg_plan_reduce_scatter(pg->rank, pg->world_size, count, dt, pg->chunk_bytes,
                                         pg->eager_max, pg->inflight, im->rings, alias, NULL, 0)
                : pg_plan_all_gather(pg->rank, pg->world_size, count, dt, uniform, im->rings, NULL, 0);
  if (n < 0) { pg_set_error("plan: bad arguments, or chunk_bytes too small for this count"); return -1; }
  if (n > im->steps_cap) {
    struct pg_step *s = (struct pg_step *)realloc(im->steps, sizeof(*s) * (size_t)n);
    if (!s) { pg_set_error("plan: out of host memory"); return -1; }
    im->steps = s;
    im->steps_cap = n;
  }
  if (is_rs)
    pg_plan_reduce_scatter(pg->rank, pg->world_size, count, dt, pg->chunk_bytes, pg->eager_max,
                           pg->inflight, im->rings, alias, im->steps, im->steps_cap);
  else
    pg_plan_all_gather(pg->rank, pg->world_size, count, dt, uniform, im->rings, im->steps, im->steps_cap);
  return n;
}

static int ensure_stage(struct pg_impl *im, int count, int dt) {
  size_t blk = ((size_t)count + (size_t)im->pg->world_size - 1) / (size_t)im->pg->world_size;
  size_t R = (size_t)im->rings, part = (blk + R - 1) / R;        /* ring g stages at g*part (pg_plan.c) */
  size_t bytes = R * part * pg_elem_size(dt);
  size_t cap1 = im->stage_cap;
  if (pg_ensure(&im->stage[0], &im->stage_cap, bytes)) return -1;
  return pg_ensure(&im->stage[1], &cap1, bytes);
}

/* ---- host-staging pipeline ----------------------------------------------------
 * Host buffers are moved block by block between the ring rounds instead of
 * whole up front: before round k the host uploads the source blocks that
 * round first reads (round 0 sends block r-1 and every round k reduces into
 * block r-2-k), while the GPU is still moving round k-1; an all-gather's
 * arrived block is downloaded while the next round is on the wire.  Plain
 * (pageable) hipMemcpy is synchronous for the host thread but runs beside the
 * non-blocking comm/reduce streams. */
struct stage_ctx {
  const char *host_src;   /* upload source (host), NULL: nothing to upload      */
  char *dev_src;          /* device image of the source                        */
  char *host_dst;         /* download target (host), NULL: nothing to download */
  char *dev_dst;          /* device image of the result                        */
  int count, dt, uniform; /* block geometry (uniform: AG blocks of `count`)     */
  unsigned char *up;      /* uploaded flags per block                          */
  int next_dl;            /* first all-gather round whose block is not downloaded */
  double *h2d_us, *d2h_us;
};

static void stage_block(const struct stage_ctx *c, int world, int b, size_t *off, size_t *len) {
  if (c->uniform) { *off = (size_t)b * (size_t)c->count; *len = (size_t)c->count; }
  else pg_block_range(c->count, world, b, off, len);
}

static int upload_block(struct pg *pg, struct stage_ctx *c, int b) {
  b = ((b % pg->world_size) + pg->world_size) % pg->world_size;
  if (!c->host_src || c->up[b]) return 0;
  size_t es = pg_elem_size(c->dt), off, len;
  stage_block(c, pg->world_size, b, &off, &len);
  c->up[b] = 1;
  return len ? pg_timed_copy(c->dev_src + off * es, c->host_src + off * es, len * es, c->h2d_us) : 0;
}

/* reduce-scatter rounds: ring g of step d reads source blocks r-d (k = 0,
 * sent) and r-(2+k)d in round k (d = +1: r-1 and r-2-k) */
static int rs_upload_hook(struct pg_impl *im, void *ctx, int k) {
  struct pg *pg = im->pg;
  struct stage_ctx *c = (struct stage_ctx *)ctx;
  if (k >= pg->world_size - 1) return 0;
  for (int g = 0; g < im->rings; ++g) {
    const int d = -pg_ring_offset(pg->world_size, im->rings, g);   /* step of the block walk */
    if (k == 0 && upload_block(pg, c, pg->rank + d)) return -1;
    if (upload_block(pg, c, pg->rank + d * (2 + k))) return -1;
    if (k == 0 && upload_block(pg, c, pg->rank + d * 3)) return -1;   /* one block of lead */
  }
  return 0;
}

/* all-gather rounds: ring g of step d receives block r-(j+1)d in round j, so
 * block b is complete after the latest of those rounds over the rings
 * (d = +1: (r-1-b) mod W; d = -1: (b-r-1) mod W).  Before round k starts, every
 * round < k has been enqueued; wait for the last recorded one (stream order
 * covers the earlier ones) and download the blocks completed in rounds
 * next_dl .. k-1.  Called with k = world-1 after the last round.  Empty
 * blocks have nothing to download. */
static int ag_download_hook(struct pg_impl *im, void *ctx, int k) {
  struct pg *pg = im->pg;
  struct stage_ctx *c = (struct stage_ctx *)ctx;
  const int W = pg->world_size, r = pg->rank;
  if (!c->host_dst || c->next_dl >= k) return 0;
  if (im->last_round_rec >= 0) PG_CHECK_HIP(hipEventSynchronize(im->round_ev[im->last_round_rec]));
  size_t es = pg_elem_size(c->dt);
  for (int b = 0; b < W; ++b) {
    if (b == r) continue;
    int done = 0;
    for (int g = 0; g < im->rings; ++g) {
      const int d = pg_ring_offset(W, im->rings, g);
      for (int j = 0; j + 1 < W; ++j)
        if ((((r - (j + 1) * d) % W) + W) % W == b) { if (j > done) done = j; break; }
    }
    if (done < c->next_dl || done >= k) continue;
    size_t off, len;
    stage_block(c, W, b, &off, &len);
    if (len && pg_timed_copy(c->host_dst + off * es, c->dev_dst + off * es, len * es, c->d2h_us)) return -1;
  }
  c->next_dl = k;
  return 0;
}

/* ---- reduce-scatter ---------------------------------------------------------- */

static int ring_reduce_scatter(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  size_t es = pg_elem_size(dt), boff, blen;
  pg_block_range(count, pg->world_size, pg->rank, &boff, &blen);
  int sd = pg_is_device_ptr(sendbuf), rd = pg_is_device_ptr(recvbuf);
  if ((sd || rd) && pg_wait_producers(im, 0)) return -1;

  void *src = sendbuf;
  unsigned char up[64];
  struct stage_ctx sc;
  memset(&sc, 0, sizeof(sc));
  int lazy = !sd && pg->world_size <= 64;
  if (!sd) {
    if (pg_ensure(&im->dsrc, &im->dsrc_cap, (size_t)count * es)) return -1;
    src = im->dsrc;
    if (lazy) {                   /* blocks go up between rounds (rs_upload_hook) */
      memset(up, 0, sizeof(up));
      sc.host_src = (const char *)sendbuf;
      sc.dev_src = (char *)src;
      sc.count = count;
      sc.dt = dt;
      sc.up = up;
      sc.h2d_us = &im->stats.h2d_us;
      sc.d2h_us = &im->stats.d2h_us;
    } else if (pg_timed_copy(im->dsrc, sendbuf, (size_t)count * es, &im->stats.h2d_us)) {
      return -1;
    }
  }
  void *out = recvbuf;
  int post_copy = 0;
  if (!rd || pg_ranges_overlap(recvbuf, blen * es, src, (size_t)count * es)) {
    if (pg_ensure(&im->dout, &im->dout_cap, blen * es)) return -1;
    out = im->dout;
    post_copy = 1;
  }
  if (ensure_stage(im, count, dt)) return -1;
  int n = plan_into(im, 1, count, dt, 0, 0);
  if (n < 0) return -1;
  void *bufs[5] = {NULL, src, out, im->stage[0], im->stage[1]};
  PG_CHECK_HIP(hipEventRecord(im->t0, im->comm));
  if (pg_exec_plan(im, im->steps, n, bufs, dt, op, lazy ? rs_upload_hook : NULL, &sc)) return -1;
  PG_CHECK_HIP(hipEventRecord(im->t1, im->comm));
  if (sync_ring(im, 1)) return -1;
  if (post_copy && pg_timed_copy(recvbuf, out, blen * es, &im->stats.d2h_us)) return -1;
  return 0;
}

/* The reference's mock (src/pg.c:264-291) on the GPU: recvbuf is indexed as a
 * full count-element buffer and the partition unit is chunk_bytes. */
static int loopback_reduce_scatter(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  size_t es = pg_elem_size(dt), bytes = (size_t)count * es;
  size_t ce = pg->chunk_bytes / es ? pg->chunk_bytes / es : 1;      /* src/pg.c:118-123 */
  int W = pg->world_size, r = pg->rank;
  /* refuse the shapes where the reference reads past sendbuf (src/pg.c:282-287
   * use recv_len on the send side): on a GPU that read could fault */
  for (int k = 0; k + 1 < W; ++k) {
    size_t s_idx = (size_t)(((r - k) % W + W) % W), r_idx = (size_t)(((r - k - 1) % W + W) % W);
    size_t so = s_idx * ce, ro = r_idx * ce;
    size_t rl = ro < (size_t)count ? (((ro + ce) < (size_t)count ? ro + ce : (size_t)count) - ro) : 0;
    if (rl && so + rl > (size_t)count) {
      pg_set_error("loopback reduce_scatter: the reference reads past sendbuf for this shape "
                   "(count=%d chunk_elems=%zu rank=%d world=%d)", count, ce, r, W);
      return -1;
    }
  }
  int sd = pg_is_device_ptr(sendbuf), rd = pg_is_device_ptr(recvbuf);
  if ((sd || rd) && pg_wait_producers(im, 0)) return -1;
  char *s, *d;
  if (sendbuf == recvbuf) {
    if (rd) s = d = (char *)recvbuf;
    else {
      if (pg_ensure(&im->dout, &im->dout_cap, bytes) || pg_timed_copy(im->dout, recvbuf, bytes, &im->stats.h2d_us)) return -1;
      s = d = (char *)im->dout;
    }
  } else {
    if (sd) s = (char *)sendbuf;
    else {
      if (pg_ensure(&im->dsrc, &im->dsrc_cap, bytes) || pg_timed_copy(im->dsrc, sendbuf, bytes, &im->stats.h2d_us)) return -1;
      s = (char *)im->dsrc;
    }
    if (rd) d = (char *)recvbuf;
    else {
      if (pg_ensure(&im->dout, &im->dout_cap, bytes) || pg_timed_copy(im->dout, recvbuf, bytes, &im->stats.h2d_us)) return -1;
      d = (char *)im->dout;
    }
  }
  PG_CHECK_HIP(hipEventRecord(im->t0, im->red));
  for (int k = 0; k + 1 < W; ++k) {                       /* src/pg.c:277-289 */
    size_t s_idx = (size_t)(((r - k) % W + W) % W), r_idx = (size_t)(((r - k - 1) % W + W) % W);
    size_t so = s_idx * ce, ro = r_idx * ce;
    if (ro >= (size_t)count) continue;                     /* recv_len == 0 */
    size_t rend = ro + ce < (size_t)count ? ro + ce : (size_t)count;
    /* lengths are whole elements, so the mock's tail memcpy (:174-177) never runs */
    if (pgk_reduce(d + ro * es, s + so * es, rend - ro, dt, op, (void *)im->red)) {
      pg_set_error("%s", pgk_last_error());
      return -1;
    }
    im->stats.reduce_launches++;
    im->stats.reduce_elems += (int64_t)(rend - ro);
  }
  PG_CHECK_HIP(hipEventRecord(im->t1, im->red));
  PG_CHECK_HIP(hipStreamSynchronize(im->red));
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, im->t0, im->t1) == hipSuccess) im->stats.ring_us = (double)ms * 1e3;
  if (!rd && pg_timed_copy(recvbuf, d, bytes, &im->stats.d2h_us)) return -1;
  return 0;
}

int pg_reduce_scatter(void *sendbuf, void *recvbuf, int count, DATATYPE datatype,
                      OPERATION op, void *pg_handle) {
  struct pg *pg = (struct pg *)pg_handle;
  if (!pg || !sendbuf || !recvbuf || count < 0 || pg_elem_size(datatype) == 0) {
    pg_set_error("pg_reduce_scatter: invalid argument");
    return -1;                                               /* src/pg.c:267 */
  }
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  if (!im) { pg_set_error("pg_reduce_scatter: closed handle"); return -1; }
  int kop = op == OP_SUM ? PGK_OP_SUM : PGK_OP_PROD;
  double t = now_us();
  stats_begin(im);
  int rc;
  if (pg->world_size == 1)                                  /* src/pg.c:269-272 */
    rc = copy_any(recvbuf, sendbuf, (size_t)count * pg_elem_size(datatype));
  else if (pg->transport == PG_TRANSPORT_LOOPBACK)
    rc = loopback_reduce_scatter(pg, sendbuf, recvbuf, count, datatype, kop);
  else if (pg->transport == PG_TRANSPORT_XGMI)
    rc = pg_xgmi_reduce_scatter(pg, sendbuf, recvbuf, count, datatype, kop);
  else if (pg_eager_applies(pg, count, datatype))
    rc = pg_eager_reduce_scatter(pg, sendbuf, recvbuf, count, datatype, kop);
  else if (pg_direct_applies(pg, count) && (rc = pg_direct_prepare(pg, count, datatype)) != 0)
    rc = rc < 0 ? -1 : pg_direct_reduce_scatter(pg, sendbuf, recvbuf, count, datatype, kop);
  else
    rc = ring_reduce_scatter(pg, sendbuf, recvbuf, count, datatype, kop);
  im->stats.wall_us = now_us() - t;
  return rc;
}

/* ---- all-gather ---------------------------------------------------------------- */

static int ring_all_gather(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  size_t slot = (size_t)count * pg_elem_size(dt), total = slot * (size_t)pg->world_size;
  int rd = pg_is_device_ptr(recvbuf), sd = sendbuf && pg_is_device_ptr(sendbuf);
  if ((rd || sd) && pg_wait_producers(im, 0)) return -1;
  char *full = (char *)recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, total)) return -1;
    full = (char *)im->dout;
  }
  char *own = full + (size_t)pg->rank * slot;
  if (sendbuf) {
    if ((char *)sendbuf != own && pg_timed_copy(own, sendbuf, slot, sd ? &im->stats.ring_us : &im->stats.h2d_us)) return -1;
  } else if (!rd) {
    if (pg_timed_copy(own, (char *)recvbuf + (size_t)pg->rank * slot, slot, &im->stats.h2d_us)) return -1;
  }
  int n = plan_into(im, 0, count, dt, 0, 1);
  if (n < 0) return -1;
  void *bufs[5] = {NULL, NULL, full, NULL, NULL};
  struct stage_ctx sc;
  memset(&sc, 0, sizeof(sc));
  sc.host_dst = rd ? NULL : (char *)recvbuf;
  sc.dev_dst = full;
  sc.count = count;
  sc.dt = dt;
  sc.uniform = 1;
  sc.d2h_us = &im->stats.d2h_us;
  PG_CHECK_HIP(hipEventRecord(im->t0, im->comm));
  if (pg_exec_plan(im, im->steps, n, bufs, dt, PGK_OP_SUM, rd ? NULL : ag_download_hook, &sc)) return -1;
  PG_CHECK_HIP(hipEventRecord(im->t1, im->comm));
  if (sync_ring(im, 1)) return -1;
  /* the hook downloaded every received block as its round completed; this
   * rank's own block is still only on the device */
  if (!rd && pg_timed_copy((char *)recvbuf + (size_t)pg->rank * slot, own, slot, &im->stats.d2h_us)) return -1;
  return 0;
}

/* The reference's mock all-gather (src/pg.c:293-321): it SUMS slot (r-k) into
 * slot (r-k-1) instead of copying (:317).  Reproduced for parity only. */
static int loopback_all_gather(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  int W = pg->world_size, r = pg->rank;
  size_t slot = (size_t)count * pg_elem_size(dt), total = slot * (size_t)W;
  int rd = pg_is_device_ptr(recvbuf), sd = sendbuf && pg_is_device_ptr(sendbuf);
  if ((rd || sd) && pg_wait_producers(im, 0)) return -1;
  char *full = (char *)recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, total) || pg_timed_copy(im->dout, recvbuf, total, &im->stats.h2d_us)) return -1;
    full = (char *)im->dout;
  }
  if (sendbuf && pg_timed_copy(full + (size_t)r * slot, sendbuf, slot, &im->stats.h2d_us)) return -1;
  for (int k = 0; k + 1 < W; ++k) {
    int s = ((r - k) % W + W) % W, d = ((r - k - 1) % W + W) % W;
    if (pgk_reduce(full + (size_t)d * slot, full + (size_t)s * slot, (size_t)count, dt, PGK_OP_SUM,
                   (void *)im->red)) {
      pg_set_error("%s", pgk_last_error());
      return -1;
    }
    im->stats.reduce_launches++;
  }
  PG_CHECK_HIP(hipStreamSynchronize(im->red));
  if (!rd && pg_timed_copy(recvbuf, full, total, &im->stats.d2h_us)) return -1;
  return 0;
}

int pg_all_gather(void *sendbuf, void *recvbuf, int count, DATATYPE datatype, void *pg_handle) {
  struct pg *pg = (struct pg *)pg_handle;
  if (!pg || !recvbuf || count < 0 || pg_elem_size(datatype) == 0) {
    pg_set_error("pg_all_gather: invalid argument");
    return -1;                                               /* src/pg.c:295 */
  }
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  if (!im) { pg_set_error("pg_all_gather: closed handle"); return -1; }
  double t = now_us();
  stats_begin(im);
  int rc;
  if (pg->world_size == 1)                                  /* src/pg.c:302-306 */
    rc = sendbuf ? copy_any(recvbuf, sendbuf, (size_t)count * pg_elem_size(datatype)) : 0;
  else if (pg->transport == PG_TRANSPORT_LOOPBACK)
    rc = loopback_all_gather(pg, sendbuf, recvbuf, count, datatype);
  else if (pg->transport == PG_TRANSPORT_XGMI)
    rc = pg_xgmi_all_gather(pg, sendbuf, recvbuf, count, datatype);
  else if (pg_eager_applies(pg, count, datatype))
    rc = pg_eager_all_gather(pg, sendbuf, recvbuf, count, datatype);
  else if (pg_direct_applies(pg, count))
    rc = pg_direct_all_gather(pg, sendbuf, recvbuf, count, datatype);
  else
    rc = ring_all_gather(pg, sendbuf, recvbuf, count, datatype);
  im->stats.wall_us = now_us() - t;
  return rc;
}

/* ---- all-reduce ------------------------------------------------------------------ */

/* Reduce-scatter in place on the working copy, then all-gather it: the
 * reference's composition (src/pg.c:323-339) on one full-size buffer, without
 * its out-of-bounds all-gather sizing (:303, :313-317). */
static int ring_all_reduce(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  size_t es = pg_elem_size(dt), bytes = (size_t)count * es, boff, blen;
  pg_block_range(count, pg->world_size, pg->rank, &boff, &blen);
  int rd = pg_is_device_ptr(recvbuf), sd = pg_is_device_ptr(sendbuf);
  if ((rd || sd) && pg_wait_producers(im, 0)) return -1;
  char *work = (char *)recvbuf;
  if (!rd) {
    if (pg_ensure(&im->dout, &im->dout_cap, bytes)) return -1;
    work = (char *)im->dout;
  }
  /* the input reaches `work` either by a device copy, or -- from host memory
   * -- block by block between the reduce-scatter rounds */
  const void *host_in = NULL;
  if (sendbuf != recvbuf) {
    if (sd) { if (pg_timed_copy(work, sendbuf, bytes, &im->stats.ring_us)) return -1; }
    else host_in = sendbuf;
  } else if (!rd) {
    host_in = recvbuf;
  }
  if (host_in && pg->world_size > 64) {
    if (pg_timed_copy(work, host_in, bytes, &im->stats.h2d_us)) return -1;
    host_in = NULL;
  }
  if (ensure_stage(im, count, dt)) return -1;
  unsigned char up[64];
  memset(up, 0, sizeof(up));
  struct stage_ctx sc;
  memset(&sc, 0, sizeof(sc));
  sc.host_src = (const char *)host_in;
  sc.dev_src = work;
  sc.host_dst = rd ? NULL : (char *)recvbuf;
  sc.dev_dst = work;
  sc.count = count;
  sc.dt = dt;
  sc.up = up;
  sc.h2d_us = &im->stats.h2d_us;
  sc.d2h_us = &im->stats.d2h_us;
  PG_CHECK_HIP(hipEventRecord(im->t0, im->comm));
  int n = plan_into(im, 1, count, dt, 1, 0);
  if (n < 0) return -1;
  void *rs_bufs[5] = {NULL, work, work + boff * es, im->stage[0], im->stage[1]};
  if (pg_exec_plan(im, im->steps, n, rs_bufs, dt, op, host_in ? rs_upload_hook : NULL, &sc)) return -1;
  /* the in-place fold of the last round reads block `rank` itself */
  if (host_in && upload_block(pg, &sc, pg->rank)) return -1;
  n = plan_into(im, 0, count, dt, 0, 0);
  if (n < 0) return -1;
  void *ag_bufs[5] = {NULL, NULL, work, NULL, NULL};
  if (pg_exec_plan(im, im->steps, n, ag_bufs, dt, op, rd ? NULL : ag_download_hook, &sc)) return -1;
  PG_CHECK_HIP(hipEventRecord(im->t1, im->comm));
  if (sync_ring(im, 1)) return -1;
  /* received blocks were downloaded round by round; this rank's own block
   * (reduced here) is still only on the device */
  if (!rd && blen && pg_timed_copy((char *)recvbuf + boff * es, work + boff * es, blen * es, &im->stats.d2h_us))
    return -1;
  return 0;
}

int pg_all_reduce(void *sendbuf, void *recvbuf, int count, DATATYPE datatype, OPERATION op,
                  void *pg_handle) {
  struct pg *pg = (struct pg *)pg_handle;
  if (!pg || !sendbuf || !recvbuf || count < 0) {
    pg_set_error("pg_all_reduce: invalid argument");
    return -1;                                               /* src/pg.c:325 */
  }
  if (pg_elem_size(datatype) == 0) {                         /* via RS, src/pg.c:333 */
    pg_set_error("pg_all_reduce: unknown datatype %d", (int)datatype);
    return -1;
  }
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  if (!im) { pg_set_error("pg_all_reduce: closed handle"); return -1; }
  int kop = op == OP_SUM ? PGK_OP_SUM : PGK_OP_PROD;
  double t = now_us();
  stats_begin(im);
  int rc;
  if (pg->world_size == 1)                                  /* src/pg.c:328-330 */
    rc = sendbuf != recvbuf ? copy_any(recvbuf, sendbuf, (size_t)count * pg_elem_size(datatype)) : 0;
  else if (pg->transport == PG_TRANSPORT_LOOPBACK) {
    pg_set_error("pg_all_reduce: the reference's world_size > 1 all-reduce writes past a "
                 "count-element recvbuf (src/pg.c:303,313-317); no defined result to reproduce");
    rc = -1;
  } else if (pg->transport == PG_TRANSPORT_XGMI)
    rc = pg_xgmi_all_reduce(pg, sendbuf, recvbuf, count, datatype, kop);
  else if (pg_eager_applies(pg, count, datatype))
    rc = pg_eager_all_reduce(pg, sendbuf, recvbuf, count, datatype, kop);
  else if (pg_direct_applies(pg, count) && (rc = pg_direct_prepare(pg, count, datatype)) != 0)
    rc = rc < 0 ? -1 : pg_direct_all_reduce(pg, sendbuf, recvbuf, count, datatype, kop);
  else
    rc = ring_all_reduce(pg, sendbuf, recvbuf, count, datatype, kop);
  im->stats.wall_us = now_us() - t;
  return rc;
}
