/*
 * include/pg.h -- public C API of the MI355X ring-collective library
 * (libpg_amd.so).  Source-compatible drop-in for the reference's
 * include/pg.h (gevahaviv1/RDMA-Ring-Collectives): same five entry points with
 * the same signatures, the same enum names and values, and a public struct pg
 * whose leading tuning fields keep the reference's names and types so an
 * existing harness can still read rank/world_size and set chunk_bytes /
 * eager_max / inflight directly (reference pg.h:40-46).
 *
 * What changed underneath:
 *   - one process per GPU; the ring hop is RCCL point-to-point over xGMI
 *     instead of RC queue pairs (reference src/RDMA_api.c, src/pg_net.c);
 *   - every arriving segment is reduced by a hand-written gfx950 HIP kernel
 *     (include/pgk.h) instead of the scalar loop at reference src/pg.c:151-159;
 *   - buffers may be host memory (staged through HBM) or HIP device memory
 *     (used in place, "device-resident").
 * Calls are synchronous: buffers are reusable when a call returns.
 * Every function returns 0 on success and -1 on failure (reference pg.h:97,121).
 */
#ifndef PG_H
#define PG_H

#ifndef PG_API
#define PG_API __attribute__((visibility("default")))
#endif

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Process-group handle.  Allocated by connect_process_group(), released by
 * pg_close().  Callers treat it as opaque except for the leading fields. */
struct pg {
  /* -- same names/types/order as reference include/pg.h:42-46 -- */
  int      rank;         /* this process's rank, 0 .. world_size-1            */
  int      world_size;   /* number of ranks (= number of hosts in the list)   */
  size_t   chunk_bytes;  /* ring pipelining segment (bytes); PG_CHUNK_BYTES   */
  size_t   eager_max;    /* blocks <= this go unsegmented; PG_EAGER_MAX       */
  int      inflight;     /* segments per transport group; PG_INFLIGHT         */

  /* -- bootstrap (reference pg.h:49-50) -- */
  char   **hosts;        /* parsed server list, world_size entries            */
  int      port;         /* TCP port of the bootstrap listener; PG_PORT       */

  /* -- MI355X build -- */
  int      device;       /* HIP device ordinal used by this rank              */
  int      transport;    /* PG_TRANSPORT_* (include/pg_ext.h)                 */
  void    *impl;         /* streams, events, HBM staging, communicator        */
};

/* Element datatypes (reference pg.h:78-81). */
typedef enum {
  DT_INT32,   /* 32-bit signed integer, wraps on overflow */
  DT_DOUBLE   /* IEEE-754 binary64 */
} DATATYPE;

/* Reduction operations (reference pg.h:84-87). */
typedef enum {
  OP_SUM,
  OP_PROD
} OPERATION;

/* Join the ring named by a whitespace-separated server list.  Rank: PG_RANK
 * (or RANK) if set, else the position of gethostname() in the list (reference
 * behaviour).  Device: PG_DEVICE, else LOCAL_RANK, else rank % device count.
 * On success *out_handle receives a struct pg*.                 (ref pg.h:99) */
PG_API int connect_process_group(const char *serverlist, void **out_handle);

/* Release everything the handle owns.  NULL-safe; always returns 0. (ref :107) */
PG_API int pg_close(void *pg_handle);

/* recvbuf[0..count) = reduction over all ranks of sendbuf[0..count).
 * In place iff sendbuf == recvbuf.                                 (ref :123) */
PG_API int pg_all_reduce(void *sendbuf, void *recvbuf, int count, DATATYPE datatype,
                  OPERATION op, void *pg_handle);

/* Reduce sendbuf[0..count) over all ranks and leave block `rank` of the result
 * in recvbuf[0 .. block_len).  Blocks: ceil(count/world_size) elements each,
 * the last ones clamped to count (include/pg_ext.h: pg_block_range).
 * world_size == 1 copies count elements, as the reference does.    (ref :140) */
PG_API int pg_reduce_scatter(void *sendbuf, void *recvbuf, int count,
                      DATATYPE datatype, OPERATION op, void *pg_handle);

/* recvbuf[q*count .. (q+1)*count) = sendbuf of rank q, on every rank.
 * sendbuf may be NULL when this rank's slot of recvbuf already holds its
 * contribution.                                                    (ref :156) */
PG_API int pg_all_gather(void *sendbuf, void *recvbuf, int count, DATATYPE datatype,
                  void *pg_handle);

#ifdef __cplusplus
}
#endif
#endif /* PG_H */
