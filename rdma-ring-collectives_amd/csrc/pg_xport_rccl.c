/*
 * pg_xport_rccl.c -- the ring hop over RCCL point-to-point (xGMI on one node).
 *
 * Replaces the reference's transport layer: RC queue pairs to the left and
 * right neighbour (src/pg.c:225-232, src/RDMA_api.c:93-309) bootstrapped over
 * TCP (src/pg_net.c), whose data path the reference never wired up
 * (pg_sendrecv_mock, src/pg.c:161-179).  One group = the sends to the right
 * neighbour and the receives from the left neighbour of one batch, fused in
 * ncclGroupStart/End so both directions progress together.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include "pg_impl.h"

#define PG_CHECK_NCCL(expr)                                                             \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess) {                                                            \
      pg_set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, ncclGetErrorString(r_));  \
      return -1;                                                                        \
    }                                                                                   \
  } while (0)

static int rccl_group_start(struct pg_impl *im) {
  (void)im;
  PG_CHECK_NCCL(ncclGroupStart());
  return 0;
}

/* A send or receive that fails inside a group returns -1 to the executor,
 * which then skips group_end; the group is closed here instead, so the
 * thread's RCCL group depth is back to zero for the caller's next call. */
#define PG_CHECK_NCCL_IN_GROUP(expr)                                                    \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess) {                                                            \
      pg_set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, ncclGetErrorString(r_));  \
      (void)ncclGroupEnd();                                                             \
      return -1;                                                                        \
    }                                                                                   \
  } while (0)

static int rccl_send(struct pg_impl *im, const void *buf, size_t bytes, int peer, hipStream_t s) {
  PG_CHECK_NCCL_IN_GROUP(ncclSend(buf, bytes, ncclUint8, peer, (ncclComm_t)im->xctx, s));
  return 0;
}

static int rccl_recv(struct pg_impl *im, void *buf, size_t bytes, int peer, hipStream_t s) {
  PG_CHECK_NCCL_IN_GROUP(ncclRecv(buf, bytes, ncclUint8, peer, (ncclComm_t)im->xctx, s));
  return 0;
}

static int rccl_group_end(struct pg_impl *im, hipStream_t s) {
  (void)im; (void)s;
  PG_CHECK_NCCL(ncclGroupEnd());
  return 0;
}

static void rccl_destroy(struct pg_impl *im) {
  if (im->xctx) ncclCommDestroy((ncclComm_t)im->xctx);
  im->xctx = NULL;
}

static const struct pg_xport_ops rccl_ops = {
  "rccl", rccl_group_start, rccl_send, rccl_recv, rccl_group_end, rccl_destroy,
};

int pg_xport_rccl_init(struct pg *pg) {
  struct pg_impl *im = (struct pg_impl *)pg->impl;
  ncclUniqueId id;
  memset(&id, 0, sizeof(id));
  if (pg->rank == 0) PG_CHECK_NCCL(ncclGetUniqueId(&id));
  if (!im->boot_fds && pg_boot_open(pg, &im->boot_fds)) return -1;
  ncclUniqueId *all = (ncclUniqueId *)malloc(sizeof(ncclUniqueId) * (size_t)pg->world_size);
  if (!all) { pg_set_error("out of host memory"); return -1; }
  if (pg_boot_allgather(pg, im->boot_fds, &id, all, sizeof(id))) { free(all); return -1; }
  id = all[0];                                   /* rank 0's id, relayed */
  free(all);
  ncclComm_t comm = NULL;
  PG_CHECK_NCCL(ncclCommInitRank(&comm, pg->world_size, id, pg->rank));
  im->xctx = comm;
  im->ops = &rccl_ops;
  return 0;
}
