/*
 * pg_host.c -- the chunk reduce with both operands in host memory
 * (pgx_reduce_host, include/pg_ext.h): the PCIe-inclusive form of the hot path
 * that is reported beside the device-resident rate.  Pinned, mapped
 * operands are reduced in place by one kernel over PCIe; pageable ones flow
 * through HBM slots.
 */
#include <pthread.h>
#include <stdio.h>
#include <string.h>

#include "pg_impl.h"

/* ---- the chunk reduce with host operands (PCIe-inclusive path) ---------------
 *
 * dst and src live in host memory.  The buffers are cut into pieces that flow
 * through HP_SLOTS device slots so that the two PCIe directions work at once:
 * the calling thread uploads piece k (dst and src, H2D) and launches its
 * reduce while a helper thread downloads piece k-1 or k-2 (D2H).  Host-to-
 * device carries 2 bytes and device-to-host 1 byte per payload byte, so with
 * both directions busy the call is bound by the upload alone instead of by
 * the sum of all three copies.
 *   upload  (caller):  [H2D d_k, s_k] -> ev_up -> reduce on s_red -> ev_red[slot]
 *   download (helper): wait ev_red[slot] -> D2H d_k -> synchronize -> downloaded = k+1
 * A slot is refilled only after its previous piece has been downloaded. */
#define HP_SLOTS 3
#define HP_PIECE_DEFAULT (16u << 20)   /* tools/host_pipe_probe.py: 16 MiB 60.6 GB/s, 32 MiB 58.0, 4 MiB 51.0, 256 MiB 46.4 */

struct hp_ctx {
  pthread_mutex_t mu;
  pthread_cond_t cv;
  size_t launched, downloaded, npieces, n, pe, es;
  int failed, device;
  char err[256];
  char *hdst;
  void *dd[HP_SLOTS];
  hipStream_t s_down;
  hipEvent_t ev_red[HP_SLOTS];
};

static void hp_fail(struct hp_ctx *c, const char *what, hipError_t e) {
  pthread_mutex_lock(&c->mu);
  if (!c->failed) snprintf(c->err, sizeof(c->err), "pgx_reduce_host: %s: %s", what, hipGetErrorString(e));
  c->failed = 1;
  pthread_cond_broadcast(&c->cv);
  pthread_mutex_unlock(&c->mu);
}

static void *hp_downloader(void *arg) {
  struct hp_ctx *c = (struct hp_ctx *)arg;
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) { hp_fail(c, "hipSetDevice", e); return NULL; }
  for (size_t k = 0; k < c->npieces; ++k) {
    pthread_mutex_lock(&c->mu);
    while (c->launched <= k && !c->failed) pthread_cond_wait(&c->cv, &c->mu);
    int failed = c->failed;
    pthread_mutex_unlock(&c->mu);
    if (failed) return NULL;
    int slot = (int)(k % HP_SLOTS);
    size_t off = k * c->pe, m = c->n - off < c->pe ? c->n - off : c->pe;
    if ((e = hipStreamWaitEvent(c->s_down, c->ev_red[slot], 0)) != hipSuccess ||
        (e = hipMemcpyAsync(c->hdst + off * c->es, c->dd[slot], m * c->es, hipMemcpyDeviceToHost, c->s_down)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(c->s_down)) != hipSuccess) {
      hp_fail(c, "download", e);
      return NULL;
    }
    pthread_mutex_lock(&c->mu);
    c->downloaded = k + 1;
    pthread_cond_broadcast(&c->cv);
    pthread_mutex_unlock(&c->mu);
  }
  return NULL;
}

/* The device address of [p, p+bytes) when it lies inside one pinned, mapped
 * host allocation (hipHostMalloc, hipHostRegister), else NULL.  Only such
 * memory may be touched by a kernel: pageable memory would fault (no XNACK). */
static void *mapped_host(const void *p, size_t bytes) {
  hipPointerAttribute_t a;
  memset(&a, 0, sizeof(a));
  void *d = NULL, *start = NULL;
  size_t size = 0;
  if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost ||
      hipHostGetDevicePointer(&d, (void *)p, 0) != hipSuccess || !d ||
      hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) != hipSuccess ||
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return NULL;
  }
  const char *lo = (const char *)start, *q = (const char *)p;
  if (!lo || q < lo || bytes > size || (size_t)(q - lo) > size - bytes) return NULL;
  return d;
}

/* Both operands pinned and mapped: one reduce launch on their device
 * addresses.  The kernel reads dst and src across PCIe and writes dst back
 * itself, so both link directions carry data at once; the staged pipeline's
 * SDMA copies run one direction at a time (tools/lab/host_direct_probe.py,
 * 256 MiB double sum: 10.1 ms direct vs 13.4 ms staged). */
static int reduce_host_direct(void *ddst, const void *dsrc, size_t n, int datatype, int op) {
  if (pgk_reduce(ddst, dsrc, n, datatype, op, NULL)) {
    pg_set_error("pgx_reduce_host: %s", pgk_last_error());
    return -1;
  }
  hipError_t e = hipStreamSynchronize(NULL);
  if (e != hipSuccess) { pg_set_error("pgx_reduce_host: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgx_reduce_host(void *dst, const void *src, size_t n, int datatype, int op, size_t chunk_bytes) {
  size_t es = pg_elem_size(datatype);
  if (!es || (op != PGK_OP_SUM && op != PGK_OP_PROD)) { pg_set_error("pgx_reduce_host: bad datatype/op"); return -1; }
  if (!n) return 0;
  if (!dst || !src) { pg_set_error("pgx_reduce_host: NULL buffer"); return -1; }
  void *ddst = mapped_host(dst, n * es), *dsrc = mapped_host(src, n * es);
  if (ddst && dsrc) return reduce_host_direct(ddst, dsrc, n, datatype, op);
  size_t piece = chunk_bytes >= (1u << 20) ? chunk_bytes : HP_PIECE_DEFAULT;
  struct hp_ctx c;
  memset(&c, 0, sizeof(c));
  pthread_mutex_init(&c.mu, NULL);
  pthread_cond_init(&c.cv, NULL);
  c.es = es;
  c.n = n;
  c.pe = piece / es ? piece / es : 1;
  if (c.pe > n) c.pe = n;
  c.npieces = (n + c.pe - 1) / c.pe;
  c.hdst = (char *)dst;
  hipStream_t s_up = NULL, s_red = NULL;
  void *ds[HP_SLOTS] = {0};
  hipEvent_t ev_up[HP_SLOTS] = {0};
  pthread_t tid;
  int started = 0, rc = -1;
  hipError_t e = hipGetDevice(&c.device);
  const int nslots = c.npieces < HP_SLOTS ? (int)c.npieces : HP_SLOTS;
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s_up, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s_red, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c.s_down, hipStreamNonBlocking);
  for (int i = 0; i < nslots && e == hipSuccess; ++i) {
    if ((e = hipMalloc(&c.dd[i], c.pe * es)) != hipSuccess || (e = hipMalloc(&ds[i], c.pe * es)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ev_up[i], hipEventDisableTiming)) != hipSuccess)
      break;
    e = hipEventCreateWithFlags(&c.ev_red[i], hipEventDisableTiming);
  }
  if (e != hipSuccess) { pg_set_error("pgx_reduce_host: setup: %s", hipGetErrorString(e)); goto out; }
  if (pthread_create(&tid, NULL, hp_downloader, &c)) { pg_set_error("pgx_reduce_host: pthread_create"); goto out; }
  started = 1;
  for (size_t k = 0; k < c.npieces; ++k) {
    int slot = (int)(k % HP_SLOTS);
    pthread_mutex_lock(&c.mu);
    while (k >= HP_SLOTS && c.downloaded < k - HP_SLOTS + 1 && !c.failed) pthread_cond_wait(&c.cv, &c.mu);
    int failed = c.failed;
    pthread_mutex_unlock(&c.mu);
    if (failed) break;
    size_t off = k * c.pe, m = n - off < c.pe ? n - off : c.pe;
    if ((e = hipMemcpyAsync(c.dd[slot], (char *)dst + off * es, m * es, hipMemcpyHostToDevice, s_up)) != hipSuccess ||
        (e = hipMemcpyAsync(ds[slot], (const char *)src + off * es, m * es, hipMemcpyHostToDevice, s_up)) !=
            hipSuccess ||
        (e = hipEventRecord(ev_up[slot], s_up)) != hipSuccess ||
        (e = hipStreamWaitEvent(s_red, ev_up[slot], 0)) != hipSuccess) {
      hp_fail(&c, "upload", e);
      break;
    }
    if (pgk_reduce(c.dd[slot], ds[slot], m, datatype, op, (void *)s_red)) {
      hp_fail(&c, pgk_last_error(), hipErrorLaunchFailure);
      break;
    }
    if ((e = hipEventRecord(c.ev_red[slot], s_red)) != hipSuccess) { hp_fail(&c, "record", e); break; }
    pthread_mutex_lock(&c.mu);
    c.launched = k + 1;
    pthread_cond_broadcast(&c.cv);
    pthread_mutex_unlock(&c.mu);
  }
out:
  if (started) pthread_join(tid, NULL);
  if (started && !c.failed && c.downloaded == c.npieces) rc = 0;
  else if (c.failed) pg_set_error("%s", c.err);
  if (s_up) { hipStreamSynchronize(s_up); hipStreamDestroy(s_up); }
  if (s_red) { hipStreamSynchronize(s_red); hipStreamDestroy(s_red); }
  if (c.s_down) { hipStreamSynchronize(c.s_down); hipStreamDestroy(c.s_down); }
  for (int i = 0; i < HP_SLOTS; ++i) {
    if (c.dd[i]) hipFree(c.dd[i]);
    if (ds[i]) hipFree(ds[i]);
    if (ev_up[i]) hipEventDestroy(ev_up[i]);
    if (c.ev_red[i]) hipEventDestroy(c.ev_red[i]);
  }
  pthread_cond_destroy(&c.cv);
  pthread_mutex_destroy(&c.mu);
  return rc;
}
