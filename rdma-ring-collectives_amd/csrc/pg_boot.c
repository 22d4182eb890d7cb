/*
 * pg_boot.c -- server list, rank/device discovery, tuning env, and the TCP
 * relay that hands rank 0's RCCL unique id to every other rank.
 *
 * Reference counterparts: parse_server_list (src/pg.c:64-102), rank by
 * gethostname (src/pg.c:188-200), pg_init_env (src/pg.c:40-58) and the TCP
 * ring bootstrap (src/pg_net.c:721-783) that exchanged queue-pair info.  On
 * one 8-GPU node the only thing to bootstrap is a 128-byte ncclUniqueId, so
 * the relay is a star on hosts[0]:port, with the reference's retry/backoff
 * discipline (src/pg_net.c:298-436) and timeout env names.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include "pg_impl.h"

int pg_parse_hosts(const char *list, char ***hosts_out, int *n_out) {
  int n = 0, cap = 8;
  char **hosts = (char **)malloc(sizeof(char *) * (size_t)cap);
  if (!hosts) return -1;
  const char *p = list;
  for (;;) {
    while (*p && isspace((unsigned char)*p)) ++p;
    if (!*p) break;
    const char *q = p;
    while (*q && !isspace((unsigned char)*q)) ++q;
    if (n == cap) {
      cap *= 2;
      char **h2 = (char **)realloc(hosts, sizeof(char *) * (size_t)cap);
      if (!h2) goto fail;
      hosts = h2;
    }
    hosts[n] = strndup(p, (size_t)(q - p));
    if (!hosts[n]) goto fail;
    ++n;
    p = q;
  }
  if (n == 0) { pg_set_error("connect_process_group: empty server list"); goto fail; }
  *hosts_out = hosts;
  *n_out = n;
  return 0;
fail:
  for (int i = 0; i < n; ++i) free(hosts[i]);
  free(hosts);
  return -1;
}

static int env_int(const char *name, int *out) {
  const char *s = getenv(name);
  if (!s || !*s) return 0;
  char *end = NULL;
  long v = strtol(s, &end, 0);
  if (end == s) return 0;
  *out = (int)v;
  return 1;
}

int pg_discover_rank(char **hosts, int n, int *rank_out) {
  int r;
  if (env_int("PG_RANK", &r) || env_int("RANK", &r)) {
    if (r < 0 || r >= n) {
      pg_set_error("rank %d from PG_RANK/RANK outside server list of %d", r, n);
      return -1;
    }
    *rank_out = r;
    return 0;
  }
  char self[256];
  if (gethostname(self, sizeof(self)) != 0) {
    pg_set_error("gethostname: %s", strerror(errno));
    return -1;
  }
  self[sizeof(self) - 1] = 0;
  for (int i = 0; i < n; ++i)
    if (strcmp(hosts[i], self) == 0) { *rank_out = i; return 0; }
  pg_set_error("Hostname '%s' not found in server list (set PG_RANK)", self);
  return -1;
}

int pg_discover_device(int rank, int *device_out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    pg_set_error("no HIP device visible");
    return -1;
  }
  int d;
  if (env_int("PG_DEVICE", &d) || env_int("LOCAL_RANK", &d)) {
    if (d < 0 || d >= ndev) { pg_set_error("device %d out of range (%d devices)", d, ndev); return -1; }
  } else {
    d = rank % ndev;
  }
  *device_out = d;
  return 0;
}

void pg_apply_env(struct pg *pg) {
  const char *s;
  if ((s = getenv("PG_CHUNK_BYTES")) && *s) {
    unsigned long long v = strtoull(s, NULL, 0);
    if (v) pg->chunk_bytes = (size_t)v;
  }
  if ((s = getenv("PG_EAGER_MAX")) && *s) pg->eager_max = (size_t)strtoull(s, NULL, 0);
  int v;
  if (env_int("PG_INFLIGHT", &v) && v > 0) pg->inflight = v;
  if (env_int("PG_PORT", &v) && v > 0 && v < 65536) pg->port = v;
}

static long now_ms(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (long)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

static int io_full(int fd, void *buf, size_t n, int writing) {
  char *p = (char *)buf;
  while (n) {
    ssize_t k = writing ? send(fd, p, n, MSG_NOSIGNAL) : recv(fd, p, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    p += k;
    n -= (size_t)k;
  }
  return 0;
}

/* ---- the bootstrap star ---------------------------------------------------------
 * Rank 0 listens on PG_PORT and keeps one TCP connection per peer for the
 * handle's lifetime; the others keep one connection to rank 0.  On it run the
 * few host-side collectives the library needs (unique-id broadcast, IPC handle
 * all-gather, barriers).  Retry/backoff and the 0xA5 ready token follow the
 * reference's bootstrap (src/pg_net.c:298-436, :699-710). */

/* Established star connections: no Nagle delay, and every send/recv bounded by
 * PG_BARRIER_TIMEOUT_MS (default 300 s), so a dead peer turns an all-gather or
 * barrier into an error instead of a hang. */
static void tune_socket(int fd) {
  int one = 1, timeout_ms = 300000;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  env_int("PG_BARRIER_TIMEOUT_MS", &timeout_ms);
  if (timeout_ms > 0) {
    struct timeval tv = {timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  }
}

int pg_boot_open(struct pg *pg, int **fds_out) {
  int timeout_ms = PG_DEFAULT_CONNECT_TIMEOUT_MS, backoff_ms = PG_DEFAULT_BACKOFF_MS;
  env_int("PG_CONNECT_TIMEOUT_MS", &timeout_ms);
  env_int("PG_BACKOFF_MS", &backoff_ms);
  int W = pg->world_size;
  int *fds = (int *)malloc(sizeof(int) * (size_t)W);
  if (!fds) return -1;
  for (int i = 0; i < W; ++i) fds[i] = -1;
  char port[16];
  snprintf(port, sizeof(port), "%d", pg->port);

  if (pg->rank == 0) {
    int ls = socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) { pg_set_error("socket: %s", strerror(errno)); free(fds); return -1; }
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    struct sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    a.sin_port = htons((uint16_t)pg->port);
    if (bind(ls, (struct sockaddr *)&a, sizeof(a)) || listen(ls, W)) {
      pg_set_error("bootstrap listen on port %d: %s", pg->port, strerror(errno));
      close(ls);
      free(fds);
      return -1;
    }
    long deadline = now_ms() + timeout_ms;
    int joined = 0;
    while (joined < W - 1) {
      struct pollfd pfd = {ls, POLLIN, 0};
      long left = deadline - now_ms();
      if (left <= 0) {
        pg_set_error("bootstrap: %d of %d ranks never connected to port %d", W - 1 - joined, W - 1, pg->port);
        close(ls);
        pg_boot_close(fds, W);
        return -1;
      }
      int pr = poll(&pfd, 1, (int)left);
      if (pr <= 0) continue;
      int c = accept(ls, NULL, NULL);
      if (c < 0) continue;
      int32_t peer = -1;
      uint8_t ack = 0xA5;
      if (io_full(c, &peer, sizeof(peer), 0) == 0 && peer > 0 && peer < W && fds[peer] < 0 &&
          io_full(c, &ack, 1, 1) == 0) {
        tune_socket(c);
        fds[peer] = c;
        ++joined;
      } else {
        close(c);
      }
    }
    close(ls);
    *fds_out = fds;
    return 0;
  }

  struct addrinfo hints, *res = NULL;
  memset(&hints, 0, sizeof(hints));
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  int gai = getaddrinfo(pg->hosts[0], port, &hints, &res);
  if (gai != 0 || !res) {
    pg_set_error("bootstrap: resolve %s: %s", pg->hosts[0], gai_strerror(gai));
    free(fds);
    return -1;
  }
  long deadline = now_ms() + timeout_ms;
  while (now_ms() < deadline) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) break;
    if (connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
      int32_t me = pg->rank;
      uint8_t ack = 0;
      if (io_full(fd, &me, sizeof(me), 1) == 0 && io_full(fd, &ack, 1, 0) == 0 && ack == 0xA5) {
        tune_socket(fd);
        fds[0] = fd;
        break;
      }
    }
    close(fd);
    struct timespec ts = {backoff_ms / 1000, (long)(backoff_ms % 1000) * 1000000L};
    nanosleep(&ts, NULL);
  }
  freeaddrinfo(res);
  if (fds[0] < 0) {
    pg_set_error("bootstrap: could not reach rank 0 at %s:%s within %d ms", pg->hosts[0], port, timeout_ms);
    free(fds);
    return -1;
  }
  *fds_out = fds;
  return 0;
}

void pg_boot_close(int *fds, int n) {
  if (!fds) return;
  for (int i = 0; i < n; ++i) if (fds[i] >= 0) close(fds[i]);
  free(fds);
}

/* all[q*bytes ..] = rank q's `mine`, on every rank. */
int pg_boot_allgather(struct pg *pg, const int *fds, const void *mine, void *all, size_t bytes) {
  int W = pg->world_size;
  if (W == 1) { memcpy(all, mine, bytes); return 0; }
  if (pg->rank == 0) {
    memcpy(all, mine, bytes);
    for (int q = 1; q < W; ++q)
      if (io_full(fds[q], (char *)all + (size_t)q * bytes, bytes, 0)) {
        pg_set_error("bootstrap allgather: lost rank %d", q);
        return -1;
      }
    for (int q = 1; q < W; ++q)
      if (io_full(fds[q], all, bytes * (size_t)W, 1)) {
        pg_set_error("bootstrap allgather: lost rank %d", q);
        return -1;
      }
    return 0;
  }
  if (io_full(fds[0], (void *)mine, bytes, 1) || io_full(fds[0], all, bytes * (size_t)W, 0)) {
    pg_set_error("bootstrap allgather: lost rank 0");
    return -1;
  }
  return 0;
}

int pg_boot_barrier(struct pg *pg, const int *fds) {
  uint8_t me = 0xA5, all[256];
  uint8_t *buf = pg->world_size <= 256 ? all : (uint8_t *)malloc((size_t)pg->world_size);
  if (!buf) return -1;
  int rc = pg_boot_allgather(pg, fds, &me, buf, 1);
  if (buf != all) free(buf);
  return rc;
}

/* ---- node-local barrier over POSIX shared memory --------------------------------
 * For transports whose ranks are by construction on one node (xgmi needs HIP
 * IPC), a barrier on a shared page costs a few microseconds instead of two TCP
 * hops through rank 0 with their scheduling jitter.  Sense-reversing counter;
 * every wait is bounded (PG_BARRIER_TIMEOUT_MS, default 300 s) so a dead peer
 * turns into an error, never a hang. */
#include <fcntl.h>
#include <sched.h>
#include <stdatomic.h>
#include <sys/mman.h>
#include <sys/stat.h>

struct pg_shm_bar {
  _Atomic unsigned count;
  _Atomic unsigned gen;
};

int pg_shm_open(struct pg *pg, const int *fds, void **bar_out) {
  char name[64], all[64 * 64];
  memset(name, 0, sizeof(name));
  if (pg->world_size > 64) return -1;
  if (pg->rank == 0) {
    snprintf(name, sizeof(name), "/pgamd.%d.%d.%ld", (int)getpid(), pg->port, (long)now_ms());
    int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, 4096)) {
      if (fd >= 0) close(fd);
      name[0] = 0;                              /* tell the others: no shm barrier */
    } else {
      close(fd);
    }
  }
  if (pg_boot_allgather(pg, fds, name, all, sizeof(name))) return -1;
  memcpy(name, all, sizeof(name));             /* rank 0's name */
  void *p = NULL;
  int ok = 0;
  if (name[0]) {
    int fd = shm_open(name, O_RDWR, 0600);
    if (fd >= 0) {
      p = mmap(NULL, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      close(fd);
      if (p == MAP_FAILED) p = NULL;
    }
    ok = p != NULL;
  }
  /* everyone mapped (or gave up) before rank 0 unlinks the name */
  char okc = (char)ok, oks[64];
  int rc = pg_boot_allgather(pg, fds, &okc, oks, 1);
  if (pg->rank == 0 && name[0]) shm_unlink(name);
  if (rc) { if (p) munmap(p, 4096); return -1; }
  for (int q = 0; q < pg->world_size; ++q)
    if (!oks[q]) { if (p) munmap(p, 4096); *bar_out = NULL; return 0; }   /* fall back to TCP */
  *bar_out = p;
  return 0;
}

void pg_shm_close(void *bar) {
  if (bar) munmap(bar, 4096);
}

int pg_shm_barrier(struct pg *pg, void *barp) {
  struct pg_shm_bar *b = (struct pg_shm_bar *)barp;
  int timeout_ms = 300000;
  env_int("PG_BARRIER_TIMEOUT_MS", &timeout_ms);
  unsigned g = atomic_load_explicit(&b->gen, memory_order_acquire);
  if (atomic_fetch_add_explicit(&b->count, 1, memory_order_acq_rel) == (unsigned)pg->world_size - 1) {
    atomic_store_explicit(&b->count, 0, memory_order_relaxed);
    atomic_store_explicit(&b->gen, g + 1, memory_order_release);
    return 0;
  }
  long deadline = 0;
  for (unsigned long spin = 0;; ++spin) {
    if (atomic_load_explicit(&b->gen, memory_order_acquire) != g) return 0;
    if (spin < 4096) { __builtin_ia32_pause(); continue; }
    if (!deadline) deadline = now_ms() + timeout_ms;
    if ((spin & 255) == 0 && now_ms() > deadline) {
      pg_set_error("barrier: peers did not arrive within %d ms", timeout_ms);
      return -1;
    }
    sched_yield();
  }
}

/* Test hook (include/pg_ext.h): the bootstrap star without any GPU. */
int pgx_boot_selftest(const char *serverlist, int rank, int port, int value, int *out) {
  if (!serverlist || !out) { pg_set_error("pgx_boot_selftest: NULL argument"); return -1; }
  struct pg pg;
  memset(&pg, 0, sizeof(pg));
  if (pg_parse_hosts(serverlist, &pg.hosts, &pg.world_size)) return -1;
  int rc = -1, *fds = NULL;
  if (rank < 0 || rank >= pg.world_size) { pg_set_error("pgx_boot_selftest: bad rank"); goto out; }
  pg.rank = rank;
  pg.port = port;
  if (pg_boot_open(&pg, &fds)) goto out;
  if (pg_boot_allgather(&pg, fds, &value, out, sizeof(int)) == 0 && pg_boot_barrier(&pg, fds) == 0) {
    void *bar = NULL;                            /* and the node-local shm barrier */
    if (pg_shm_open(&pg, fds, &bar) == 0 && bar) {
      rc = 0;
      for (int i = 0; i < 1000 && rc == 0; ++i) rc = pg_shm_barrier(&pg, bar);
      pg_shm_close(bar);
    }
  }
out:
  pg_boot_close(fds, pg.world_size);
  for (int i = 0; i < pg.world_size; ++i) free(pg.hosts[i]);
  free(pg.hosts);
  return rc;
}

