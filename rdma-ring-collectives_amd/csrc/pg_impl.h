/*
 * pg_impl.h -- internals of libpg_amd.so (not installed).
 *
 * Layering (mirrors the reference's split into collectives / group lifecycle / bootstrap,
 * src/pg.c:264-339 / :185-262 / src/pg_net.c):
 *   pg.c          public API, validation, host<->HBM staging, loopback mock
 *   pg_plan.c     ring schedule as data (pure C, no HIP)
 *   pg_exec.c     executes a plan: transport groups on the comm stream,
 *                 pgk_reduce on the reduce stream, events in between
 *   pg_xport_*.c  the hop: RCCL P2P over xGMI, or in-process virtual ranks
 *   pg_boot.c     server list, rank/device discovery, TCP unique-id relay
 */
#ifndef PG_IMPL_H
#define PG_IMPL_H

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include "pg.h"
#include "pg_ext.h"
#include "pgk.h"

/* Defaults.  The reference's 4 KiB chunk (src/constants.h:82) was sized for an
 * RDMA MTU; a GPU ring segment below ~1 MiB is launch-bound, so the segment
 * default is 4 MiB here.  eager_max and inflight keep the reference values
 * (src/constants.h:75,89).  Env overrides win (the reference applied them
 * only to zero fields after setting defaults, so they never took effect:
 * src/pg.c:203-209 vs :42-50). */
#define PG_DEFAULT_CHUNK_BYTES   (4u << 20)
#define PG_DEFAULT_EAGER_MAX     4096u
#define PG_DEFAULT_INFLIGHT      4
/* The link segment (chunk_bytes x inflight per transport group) and the reduce
 * launch are separate knobs: arrived segments of a round are reduced together
 * once this many bytes per operand are pending.  A 32 MiB launch (the default
 * group, two rings) runs at 71-73% of the HBM peak, a 128 MiB one at 80-82%
 * (kernel-stamped, MI355X). */
#define PG_DEFAULT_REDUCE_BYTES  (128u << 20)
#define PG_DEFAULT_PORT          18515
#define PG_DEFAULT_CONNECT_TIMEOUT_MS 60000
#define PG_DEFAULT_BACKOFF_MS    100

#define PG_RECV_EVENTS 8

struct pg_impl;

/* The hop.  A group holds the sends and receives of one batch (clockwise:
 * to the right neighbour / from the left one; counter-clockwise: the
 * opposite); all are enqueued on `stream`.  Same per-peer ordering rules as
 * ncclSend/ncclRecv. */
struct pg_xport_ops {
  const char *name;
  int (*group_start)(struct pg_impl *im);
  int (*send)(struct pg_impl *im, const void *buf, size_t bytes, int peer, hipStream_t s);
  int (*recv)(struct pg_impl *im, void *buf, size_t bytes, int peer, hipStream_t s);
  int (*group_end)(struct pg_impl *im, hipStream_t s);
  void (*destroy)(struct pg_impl *im);
};

struct pg_impl {
  struct pg *pg;
  const struct pg_xport_ops *ops;
  void *xctx;                 /* ncclComm_t, or the virtual-rank context      */

  hipStream_t comm, red;      /* transfers / reductions                       */
  size_t red_bytes;           /* PG_REDUCE_BYTES: arrived segments are reduced once this many
                                 bytes per operand are pending (or the round ends); 0 = per batch */
  int *pend; int pend_cap;    /* plan steps whose reduce is pending            */
  struct pg_red_range *ranges; int ranges_cap;   /* what the next reduce launch covers */
  hipEvent_t *red_ev;         /* per segment: its reduce finished             */
  int n_red_ev;
  hipEvent_t recv_ev[PG_RECV_EVENTS]; /* per batch: its receives landed       */
  hipEvent_t join_ev, t0, t1;
  hipEvent_t entry_ev;        /* the caller's null-stream work at entry (pg_wait_producers) */
  hipEvent_t *kt_ev;          /* PG_KERNEL_TIMING=1: start/stop pairs of this call's reduce launches */
  int n_kt_ev, kt_used, kt_on;
  hipEvent_t *round_ev;       /* per ring round: recorded behind its transfers */
  int n_round_ev;
  int last_round_rec;         /* round whose round_ev was recorded last, -1: none */

  /* HBM working memory, grown on demand and kept (288 GB per GPU). */
  void *stage[2];  size_t stage_cap;
  void *dsrc;      size_t dsrc_cap;   /* device copy of a host sendbuf        */
  void *dout;      size_t dout_cap;   /* device result / full buffer          */
  void *ebuf;      size_t ebuf_cap;   /* eager one-shot gather area (pg_eager.c) */
  int eager_oneshot;          /* PG_EAGER_ONESHOT, default 1                  */
  int rings;                  /* PG_RINGS: 1 .. 4, default 2, pg_ext.h         */
  int algo;                   /* PG_ALGO: PG_ALGO_RING / PG_ALGO_DIRECT (P2P transports) */

  struct pg_step *steps; int steps_cap;
  int *boot_fds;              /* bootstrap star (pg_boot.c), world_size slots */
  struct pg_stats stats;
  int64_t calls_redone;       /* cumulative: xgmi calls redone with the slot copy */
};

/* pg.c */
void pg_set_error(const char *fmt, ...);
void pg_trace(const struct pg *pg, const char *fmt, ...);
int pg_ensure(void **buf, size_t *cap, size_t bytes);   /* hipMalloc-grow */
int pg_stream_wait(hipStream_t s);                        /* bounded spin, then block */
int pg_wait_producers(struct pg_impl *im, int host_wait); /* caller's pending null-stream work */
int pg_copy_parallel(void *dst, const void *src, size_t bytes);  /* host<->device, threaded */
int pg_impl_create(struct pg *pg);                        /* streams/events */
void pg_impl_destroy(struct pg *pg);
size_t pg_elem_size(int dt);
int pg_is_device_ptr(const void *p);                      /* HIP device/managed memory? */
int pg_ranges_overlap(const void *a, size_t na, const void *b, size_t nb);
int pg_timed_copy(void *dst, const void *src, size_t bytes, double *acc_us);  /* any direction */
int pg_default_transport(const struct pg *pg);            /* no PG_TRANSPORT: xgmi on one node, else rccl */

/* pg_direct.c: one-hop exchanges over every link, fold in ring order (P2P transports) */
#define PG_ALGO_RING   0
#define PG_ALGO_DIRECT 1
int pg_direct_applies(const struct pg *pg, int count);
int pg_direct_prepare(struct pg *pg, int count, int dt);  /* 1 go, 0 every rank takes the ring, -1 failed */
int pg_direct_reduce_scatter(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op);
int pg_direct_all_gather(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt);
int pg_direct_all_reduce(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op);

/* pg_eager.c: one group + one launch for messages <= eager_max (P2P transports) */
int pg_eager_applies(const struct pg *pg, int count, int dt);
int pg_eager_reduce_scatter(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op);
int pg_eager_all_gather(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt);
int pg_eager_all_reduce(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op);

/* pg_exec.c: run `n` steps; bufs[] indexed by PG_BUF_*.  If `hook` is set it
 * is called on the host before the first batch of each round k (and once with
 * k = rounds after the last), after round_ev[k-1] -- recorded on the comm
 * stream behind round k-1's transfers -- exists: the host-staging pipeline
 * uploads/downloads blocks there while the GPU runs the ring. */
typedef int (*pg_round_hook)(struct pg_impl *im, void *ctx, int round);
int pg_kt_pair(struct pg_impl *im, void **t0, void **t1);   /* PG_KERNEL_TIMING: next stamp pair */
void pg_kt_collect(struct pg_impl *im);                     /* sum them once the streams drained */
int pg_exec_plan(struct pg_impl *im, const struct pg_step *st, int n,
                 void *const bufs[5], int dt, int op, pg_round_hook hook, void *hook_ctx);

/* pg_xport_rccl.c */
int pg_xport_rccl_init(struct pg *pg);
/* pg_xport_xgmi.c: direct peer reads over xGMI (IPC-mapped exchange buffers) */
int pg_xport_xgmi_init(struct pg *pg);
void pg_xport_xgmi_destroy(struct pg *pg);
int pg_xgmi_reduce_scatter(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op);
int pg_xgmi_all_gather(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt);
int pg_xgmi_all_reduce(struct pg *pg, void *sendbuf, void *recvbuf, int count, int dt, int op);
/* pg_xport_threads.c */
int pg_xport_threads_attach(struct pg *pg, void *hub);

/* pg_boot.c */
int pg_parse_hosts(const char *list, char ***hosts_out, int *n_out);
int pg_discover_rank(char **hosts, int n, int *rank_out);
int pg_discover_device(int rank, int *device_out);
void pg_apply_env(struct pg *pg);
int pg_boot_open(struct pg *pg, int **fds_out);
void pg_boot_close(int *fds, int n);
int pg_boot_allgather(struct pg *pg, const int *fds, const void *mine, void *all, size_t bytes);
int pg_boot_barrier(struct pg *pg, const int *fds);
int pg_shm_open(struct pg *pg, const int *fds, void **bar_out);   /* NULL bar: fall back to TCP */
void pg_shm_close(void *bar);
int pg_shm_barrier(struct pg *pg, void *bar);

#define PG_CHECK_HIP(expr)                                                          \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) {                                                         \
      pg_set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
      return -1;                                                                    \
    }                                                                               \
  } while (0)

#endif /* PG_IMPL_H */
