/*
 * pg_xport_threads.c -- W virtual ranks inside one process, one GPU.
 *
 * RCCL refuses two ranks on one device unless each rank claims its own host
 * (NCCL_HOSTID, tests/test_rccl_gpu.py), and then its hops ride sockets.  This
 * transport runs up to 64 ranks in ONE process instead: it keeps everything of
 * the real path -- plan,
 * executor, streams, events, staging, the gfx950 reduce kernel, the public
 * pg_* entry points -- and replaces only the hop: a send is published in a
 * per-edge FIFO and the receiving rank copies it device-to-device on its own
 * comm stream.  It plays the role the reference's pg_sendrecv_mock played
 * (src/pg.c:161-179) -- a transport that needs no network -- but it moves the
 * data between distinct ranks instead of reducing a rank's own buffers.
 *
 * Each group is synchronous on the host (sender's data ready -> publish ->
 * receiver copies -> ack), which is slow and obviously ordered; it exists to
 * prove results, not to be timed.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pg_impl.h"

struct sim_msg {
  const void *buf;
  size_t bytes;
  struct sim_msg *next;
};

struct sim_chan {              /* edge src -> dst: chan[src * world + dst] */
  struct sim_msg *head, *tail;
  long pushed, acked;
};

struct sim_hub {
  int world;
  int abort;
  pthread_mutex_t mu;
  pthread_cond_t cv;
  struct sim_chan *chan;
};

struct sim_io { void *buf; size_t bytes; int peer; };

struct sim_rank {
  struct sim_hub *hub;
  struct sim_io *sends, *recvs;
  int n_send, n_recv, cap_send, cap_recv;
};

static int hub_wait(struct sim_hub *h) {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  ts.tv_sec += 120;
  int e = pthread_cond_timedwait(&h->cv, &h->mu, &ts);
  if (e == ETIMEDOUT) { h->abort = 1; pthread_cond_broadcast(&h->cv); return -1; }
  return h->abort ? -1 : 0;
}

static int th_group_start(struct pg_impl *im) {
  struct sim_rank *sr = (struct sim_rank *)im->xctx;
  sr->n_send = sr->n_recv = 0;
  return 0;
}

static int push_io(struct sim_io **arr, int *n, int *cap, void *buf, size_t bytes, int peer) {
  if (*n == *cap) {
    int c = *cap ? *cap * 2 : 16;
    struct sim_io *a = (struct sim_io *)realloc(*arr, sizeof(**arr) * (size_t)c);
    if (!a) return -1;
    *arr = a;
    *cap = c;
  }
  (*arr)[*n].buf = buf;
  (*arr)[*n].bytes = bytes;
  (*arr)[*n].peer = peer;
  ++*n;
  return 0;
}

static int th_send(struct pg_impl *im, const void *buf, size_t bytes, int peer, hipStream_t s) {
  (void)s;
  struct sim_rank *sr = (struct sim_rank *)im->xctx;
  if (push_io(&sr->sends, &sr->n_send, &sr->cap_send, (void *)buf, bytes, peer)) { pg_set_error("sim: oom"); return -1; }
  return 0;
}

static int th_recv(struct pg_impl *im, void *buf, size_t bytes, int peer, hipStream_t s) {
  (void)s;
  struct sim_rank *sr = (struct sim_rank *)im->xctx;
  if (push_io(&sr->recvs, &sr->n_recv, &sr->cap_recv, buf, bytes, peer)) { pg_set_error("sim: oom"); return -1; }
  return 0;
}

static int th_group_end(struct pg_impl *im, hipStream_t s) {
  struct sim_rank *sr = (struct sim_rank *)im->xctx;
  struct sim_hub *h = sr->hub;
  const int r = im->pg->rank, W = h->world;
  /* everything enqueued before the group (incl. waits on reduces) is done */
  PG_CHECK_HIP(hipStreamSynchronize(s));

  pthread_mutex_lock(&h->mu);
  for (int i = 0; i < sr->n_send; ++i) {
    struct sim_msg *m = (struct sim_msg *)calloc(1, sizeof(*m));
    if (!m) { h->abort = 1; pthread_cond_broadcast(&h->cv); pthread_mutex_unlock(&h->mu); pg_set_error("sim: oom"); return -1; }
    m->buf = sr->sends[i].buf;
    m->bytes = sr->sends[i].bytes;
    struct sim_chan *c = &h->chan[r * W + sr->sends[i].peer];
    if (c->tail) c->tail->next = m; else c->head = m;
    c->tail = m;
    c->pushed++;
  }
  pthread_cond_broadcast(&h->cv);
  pthread_mutex_unlock(&h->mu);

  for (int i = 0; i < sr->n_recv; ++i) {
    const int from = sr->recvs[i].peer;
    pthread_mutex_lock(&h->mu);
    struct sim_chan *c = &h->chan[from * W + r];
    while (!c->head) {
      if (hub_wait(h)) { pthread_mutex_unlock(&h->mu); pg_set_error("sim: rank %d timed out waiting for rank %d", r, from); return -1; }
    }
    struct sim_msg *m = c->head;
    c->head = m->next;
    if (!c->head) c->tail = NULL;
    pthread_mutex_unlock(&h->mu);
    if (m->bytes != sr->recvs[i].bytes) {
      pg_set_error("sim: rank %d expected %zu bytes from rank %d, got %zu", r, sr->recvs[i].bytes, from, m->bytes);
      free(m);
      pthread_mutex_lock(&h->mu); h->abort = 1; pthread_cond_broadcast(&h->cv); pthread_mutex_unlock(&h->mu);
      return -1;
    }
    hipError_t e = hipMemcpyAsync(sr->recvs[i].buf, m->buf, m->bytes, hipMemcpyDefault, s);
    free(m);
    if (e != hipSuccess) { pg_set_error("sim: copy: %s", hipGetErrorString(e)); return -1; }
  }
  PG_CHECK_HIP(hipStreamSynchronize(s));

  pthread_mutex_lock(&h->mu);
  for (int i = 0; i < sr->n_recv; ++i) h->chan[sr->recvs[i].peer * W + r].acked += 1;
  pthread_cond_broadcast(&h->cv);
  for (int i = 0; i < sr->n_send; ++i) {
    struct sim_chan *c = &h->chan[r * W + sr->sends[i].peer];
    while (c->acked < c->pushed) {
      if (hub_wait(h)) { pthread_mutex_unlock(&h->mu); pg_set_error("sim: rank %d: sends never consumed", r); return -1; }
    }
  }
  pthread_mutex_unlock(&h->mu);
  return 0;
}

static void th_destroy(struct pg_impl *im) {
  struct sim_rank *sr = (struct sim_rank *)im->xctx;
  if (sr) { free(sr->sends); free(sr->recvs); free(sr); }
  im->xctx = NULL;
}

static const struct pg_xport_ops threads_ops = {
  "threads", th_group_start, th_send, th_recv, th_group_end, th_destroy,
};

int pg_xport_threads_attach(struct pg *pg, void *hub) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  struct sim_rank *sr = (struct sim_rank *)calloc(1, sizeof(*sr));
  if (!sr) return -1;
  sr->hub = (struct sim_hub *)hub;
  im->xctx = sr;
  im->ops = &threads_ops;
  return 0;
}

/* ---- pgx_sim_run ------------------------------------------------------------ */

struct sim_job {
  struct pg *pg;
  int device, coll, count, dt, op, rc;
  void *send, *recv;
  char err[256];
};

static void *sim_thread(void *arg) {
  struct sim_job *j = (struct sim_job *)arg;
  j->rc = -1;
  if (hipSetDevice(j->device) != hipSuccess) { snprintf(j->err, sizeof(j->err), "sim: hipSetDevice"); return NULL; }
  if (j->coll == PG_COLL_REDUCE_SCATTER)
    j->rc = pg_reduce_scatter(j->send, j->recv, j->count, (DATATYPE)j->dt, (OPERATION)j->op, j->pg);
  else if (j->coll == PG_COLL_ALL_GATHER)
    j->rc = pg_all_gather(j->send, j->recv, j->count, (DATATYPE)j->dt, j->pg);
  else
    j->rc = pg_all_reduce(j->send, j->recv, j->count, (DATATYPE)j->dt, (OPERATION)j->op, j->pg);
  if (j->rc) {
    snprintf(j->err, sizeof(j->err), "%s", pg_last_error());
    struct sim_rank *sr = (struct sim_rank *)((struct pg_impl *)j->pg->impl)->xctx;
    pthread_mutex_lock(&sr->hub->mu);
    sr->hub->abort = 1;
    pthread_cond_broadcast(&sr->hub->cv);
    pthread_mutex_unlock(&sr->hub->mu);
  }
  return NULL;
}

int pgx_sim_run(int world, int coll, void *const *sendbufs, void *const *recvbufs,
                int count, int datatype, int op, size_t chunk_bytes,
                size_t eager_max, int inflight, int rings) {
  if (world < 1 || world > 64 || !recvbufs || coll < 0 || coll > 2 || rings < 0 || rings > PG_MAX_RINGS) {
    pg_set_error("pgx_sim_run: bad arguments");
    return -1;
  }
  int dev = 0;
  PG_CHECK_HIP(hipGetDevice(&dev));
  struct sim_hub hub;
  memset(&hub, 0, sizeof(hub));
  hub.world = world;
  pthread_mutex_init(&hub.mu, NULL);
  pthread_cond_init(&hub.cv, NULL);
  hub.chan = (struct sim_chan *)calloc((size_t)world * (size_t)world, sizeof(struct sim_chan));
  struct sim_job *jobs = (struct sim_job *)calloc((size_t)world, sizeof(struct sim_job));
  pthread_t *tid = (pthread_t *)calloc((size_t)world, sizeof(pthread_t));
  int rc = -1, started = 0;
  if (!hub.chan || !jobs || !tid) { pg_set_error("pgx_sim_run: oom"); goto out; }

  for (int r = 0; r < world; ++r) {
    struct pg *pg = (struct pg *)calloc(1, sizeof(struct pg));
    if (!pg) { pg_set_error("pgx_sim_run: oom"); goto out; }
    pg->rank = r;
    pg->world_size = world;
    pg->chunk_bytes = chunk_bytes ? chunk_bytes : PG_DEFAULT_CHUNK_BYTES;
    pg->eager_max = eager_max;
    pg->inflight = inflight > 0 ? inflight : PG_DEFAULT_INFLIGHT;
    pg->port = PG_DEFAULT_PORT;
    pg->device = dev;
    pg->transport = world == 1 ? PG_TRANSPORT_SELF : PG_TRANSPORT_THREADS;
    jobs[r].pg = pg;
    if (pg_impl_create(pg) || pg_xport_threads_attach(pg, &hub)) goto out;
    if (rings) ((struct pg_impl *)pg->impl)->rings = rings;    /* 0: PG_RINGS / default */
    jobs[r].device = dev; jobs[r].coll = coll; jobs[r].count = count;
    jobs[r].dt = datatype; jobs[r].op = op;
    jobs[r].send = sendbufs ? sendbufs[r] : NULL;
    jobs[r].recv = recvbufs[r];
  }
  for (int r = 0; r < world; ++r, ++started)
    if (pthread_create(&tid[r], NULL, sim_thread, &jobs[r])) { pg_set_error("pgx_sim_run: pthread_create"); break; }
  for (int r = 0; r < started; ++r) pthread_join(tid[r], NULL);
  if (started == world) {
    rc = 0;
    for (int r = 0; r < world; ++r)
      if (jobs[r].rc) { pg_set_error("rank %d: %s", r, jobs[r].err); rc = -1; break; }
  }
out:
  for (int r = 0; jobs && r < world; ++r) if (jobs[r].pg) pg_close(jobs[r].pg);
  if (hub.chan) {
    for (int r = 0; r < world * world; ++r) {
      struct sim_msg *m = hub.chan[r].head;
      while (m) { struct sim_msg *n = m->next; free(m); m = n; }
    }
  }
  free(hub.chan); free(jobs); free(tid);
  pthread_mutex_destroy(&hub.mu);
  pthread_cond_destroy(&hub.cv);
  return rc;
}
