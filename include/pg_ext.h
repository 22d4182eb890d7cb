/*
 * include/pg_ext.h -- extensions of libpg_amd.so beyond the reference surface.
 *
 * None of these are needed by a caller of the reference API (include/pg.h).
 * They expose (a) the ring schedule as data, so the host logic can be tested
 * without a GPU, (b) transports for single-process operation, and
 * (c) per-call measurements for the benchmark.
 */
#ifndef PG_EXT_H
#define PG_EXT_H

#ifndef PG_API
#define PG_API __attribute__((visibility("default")))
#endif

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* struct pg.transport values.  Selected with PG_TRANSPORT=rccl|xgmi|loopback;
 * unset: XGMI when every server-list entry names the same host and W <= 16,
 * else RCCL. */
#define PG_TRANSPORT_RCCL     0  /* one process per GPU, RCCL P2P ring (xGMI on a node) */
#define PG_TRANSPORT_LOOPBACK 1  /* one process, the reference's single-process mock
                                    schedule (src/pg.c:161-179, :264-321) run on the
                                    GPU kernel: results equal the reference's own   */
#define PG_TRANSPORT_THREADS  2  /* W virtual ranks in one process (one thread each)
                                    sharing one GPU; the hop is a device copy.  Used
                                    by pgx_sim_run() to exercise the ring executor   */
#define PG_TRANSPORT_SELF     3  /* world_size == 1 */
#define PG_TRANSPORT_XGMI     4  /* one process per GPU; each rank reads block r of every
                                    peer's contribution directly over xGMI (HIP IPC) and
                                    folds them in ring order with one kernel: all links
                                    busy at once, results identical to the ring        */

/* Ring block partition used by pg_reduce_scatter / pg_all_reduce: block b of
 * count elements = [b*B, min((b+1)*B, count)) with B = ceil(count/world), the
 * reference's chunk_offsets() clamping (src/pg.c:126-138).  Elements. */
PG_API int pg_block_range(int count, int world, int block, size_t *off, size_t *len);

/* Rings.  Every block is split into `rings` parts, part g =
 * [ceil(g*len/R), ceil((g+1)*len/R)) (part 0 the largest), and part g travels
 * its own ring of step d = pg_ring_offset(world, rings, g): send to rank+d,
 * receive from rank-d, folded
 *     x[b+d] op x[b+2d] op ... op x[b+(W-1)d] op x[b]      (indices mod W)
 * Steps: +1, -1 (rings = 2, the default: both directions of each ring link
 * carry data), then +3, -3 (rings = 3, 4: rings over further xGMI links) when
 * coprime with the world size and new mod world; when those run out the list
 * repeats.  rings = 1: one part, the whole block, clockwise.  Every transport
 * (ring, eager one-shot, xgmi) folds each part in its ring's order, so all of
 * them give identical bits for a given `rings` (PG_RINGS).  Elements. */
#define PG_MAX_RINGS 4
PG_API int pg_block_part(size_t len, int rings, int part, size_t *off, size_t *plen);
PG_API int pg_ring_offset(int world, int rings, int part);

/* Buffer roles named by plan steps. */
#define PG_BUF_NONE   0
#define PG_BUF_SRC    1   /* this rank's input (count elements)               */
#define PG_BUF_OUT    2   /* RS: this rank's result block; AG: the full buffer */
#define PG_BUF_STAGE0 3   /* HBM staging, one block                            */
#define PG_BUF_STAGE1 4   /* HBM staging, one block                            */

/* One ring step: in one transport group, send `send_bytes` to rank
 * (rank + send_peer) and receive `recv_bytes` from rank (rank + recv_peer),
 * mod world (d / -d of the step's ring: the clockwise ring sends right and
 * receives from the left, the counter-clockwise ring the opposite); then (on the reduce stream,
 * after the receive) red_dst[i] = red_dst[i] op red_src[i] for i < red_elems,
 * or, with red_rev, red_dst[i] = red_src[i] op red_dst[i]: the arrival is
 * always the left operand (the ring order), which matters for the NaN payload
 * a sum or product of two NaNs returns.  Offsets/lengths in bytes except
 * red_elems. */
struct pg_step {
  int32_t round;       /* ring round k, 0 .. world-2                          */
  int32_t batch;       /* steps with equal batch share one transport group    */
  int32_t seg;         /* segment index within the round (event slot)         */
  int32_t send_wait;   /* 1: the sent segment is the previous round's reduce
                          output for `seg`; wait for it before sending        */
  int32_t send_buf, recv_buf, red_dst_buf, red_src_buf;
  int32_t send_peer, recv_peer; /* rank offsets of the peers: d and -d       */
  int64_t send_off, send_bytes;
  int64_t recv_off, recv_bytes;
  int64_t red_dst_off, red_src_off, red_elems;
  int32_t red_rev;     /* 1: red_dst = red_src op red_dst (in-place last round) */
  int32_t red_fold;    /* direct plans: 1 = fold block `rank`'s W copies, see below */
};

/* Reduce-scatter plan for one rank.  Clockwise ring: round k sends block
 * (rank-1-k) and receives block (rank-2-k) mod world -- the reference's
 * rs_send/recv_chunk_index (src/pg.c:141-148) evaluated at rank-1, so that
 * rank r finishes with block r.  Ring g of step d: round k sends block
 * (rank-(k+1)d) and receives block (rank-(k+2)d), its part g only (d = -1,
 * the counter-clockwise ring: blocks rank+1+k and rank+2+k).
 * Segments: chunk_elems_from_bytes(chunk_bytes) (src/pg.c:118-123) elements;
 * parts <= eager_max bytes are one segment; each batch carries `inflight`
 * segment indices of every ring (ring 0's steps first).  Ring g stages its
 * parts at element g*ceil(B/R) of the staging blocks (B = ceil(count/world);
 * staging blocks hold R*ceil(B/R) elements).
 * out_aliases_src: OUT is block `rank` of SRC (in-place all-reduce).  Returns
 * the number of steps written (or needed, when steps == NULL), -1 on bad
 * arguments or a chunk_bytes so small that the plan would exceed 2^28 steps. */
PG_API int pg_plan_reduce_scatter(int rank, int world, int count, int datatype,
                           size_t chunk_bytes, size_t eager_max, int inflight, int rings,
                           int out_aliases_src, struct pg_step *steps, int max_steps);

/* All-gather plan: round k sends block (rank-k) and receives block
 * (rank-k-1) of OUT (src/pg.c:309-318 indices), whole parts, no reduce; part
 * g of each block rides ring g of step d (round k sends block rank-k*d to
 * rank+d and receives block rank-(k+1)*d from rank-d).
 * uniform = 1: blocks of `count` elements (pg_all_gather);
 * uniform = 0: the reduce-scatter partition of `count` (pg_all_reduce). */
PG_API int pg_plan_all_gather(int rank, int world, int count, int datatype, int uniform, int rings,
                       struct pg_step *steps, int max_steps);

/* Direct-exchange plan (PG_ALGO=direct) for one rank's reduce-scatter.
 * Transfer steps (red_elems == 0): send `send_bytes` of SRC at send_off to
 * rank+send_peer and receive `recv_bytes` from rank+recv_peer into STAGE0 at
 * recv_off (STAGE0 = W slots of B = ceil(count/world) elements; slot q holds
 * rank q's copy of block `rank`).  Fold steps (red_fold == 1, after the
 * transfers of their batch): OUT[red_dst_off ..] (red_elems elements, offsets
 * in bytes within block `rank`) = x[rank+d] op x[rank+2d] op ... op x[rank]
 * with d = pg_ring_offset(world, rings, seg), x[q] = slot q of STAGE0 at
 * red_src_off, x[rank] = SRC at (block offset + red_src_off).  Batches carry
 * `inflight` segments of chunk_bytes; every rank's groups pair up. */
PG_API int pg_plan_direct_reduce_scatter(int rank, int world, int count, int datatype, size_t chunk_bytes,
                                         int inflight, int rings, struct pg_step *steps, int max_steps);

/* The reduce launches of a set of ring steps.  The executor does not reduce a
 * transport group's arrived segments at once: steps wait until PG_REDUCE_BYTES
 * per operand are pending (or the round ends) and are then reduced together.
 * This lists what that one launch covers: idx[0..n) are indices into st[] of
 * steps with red_elems > 0; they are sorted in place by (buffers, direction,
 * destination offset), and every run of steps contiguous in both operands
 * becomes one range (the segments of one ring over consecutive groups are
 * neighbours in the same block, so usually one range per ring).  elem_size: 4
 * or 8.  Returns the number of ranges written to out[0..max_out), or -1 when
 * max_out is too small or an argument is bad. */
struct pg_red_range {
  int32_t dst_buf, src_buf;   /* PG_BUF_*                                        */
  int32_t rev, pad;           /* rev: dst = src op dst (pg_step.red_rev)         */
  int64_t dst_off, src_off;   /* bytes                                           */
  int64_t elems;
};
PG_API int pg_plan_coalesce(const struct pg_step *st, int *idx, int n, size_t elem_size,
                            struct pg_red_range *out, int max_out);

/* Open a handle without a server list: transport LOOPBACK (reference mock
 * semantics for a given rank/world) or SELF (world must be 1).  The device is
 * the current HIP device. */
PG_API int pg_connect_local(int rank, int world, int transport, void **out_handle);

/* Run one collective over `world` virtual ranks in this process (transport
 * THREADS): rank r uses sendbufs[r] / recvbufs[r] (HIP device or host
 * memory).  coll: 0 reduce-scatter, 1 all-gather, 2 all-reduce.  rings:
 * 1 .. PG_MAX_RINGS, 0 = PG_RINGS / the default.  The schedule is the W-1
 * round ring unless PG_ALGO=direct.
 *
 * PG_ALGO (point-to-point transports: rccl, threads): "ring" = the W-1 round
 * ring (pg_plan.c / pg_exec.c); "direct" = block q sent straight to rank q
 * over its own link, block r folded from all W copies in ring order
 * (pg_direct.c), same bits.  Unset: direct when every server-list entry names
 * the same host and W <= 16, else ring. */
#define PG_COLL_REDUCE_SCATTER 0
#define PG_COLL_ALL_GATHER     1
#define PG_COLL_ALL_REDUCE     2
PG_API int pgx_sim_run(int world, int coll, void *const *sendbufs, void *const *recvbufs,
                int count, int datatype, int op, size_t chunk_bytes,
                size_t eager_max, int inflight, int rings);

/* The hot path with both operands in host memory: dst[i] = dst[i] op src[i]
 * (op: OP_SUM / OP_PROD).  Both operands pinned and mapped (hipHostMalloc,
 * hipHostRegister): one reduce kernel works on them in place across PCIe,
 * reading and writing at once.  Otherwise staged through HBM in chunk_bytes
 * pieces (0 = 16 MiB) that flow through 3 device slots: uploads (dst, src)
 * and the reduce run on the calling thread while a helper thread downloads
 * finished pieces.  Synchronous.  This call is what the PCIe-inclusive rate
 * of the hot path is measured on. */
PG_API int pgx_reduce_host(void *dst, const void *src, size_t n, int datatype, int op, size_t chunk_bytes);

/* Measurements of the last collective on this handle. */
struct pg_stats {
  double wall_us;        /* host wall time of the call                      */
  double h2d_us, d2h_us; /* host-staging copies (0 when device-resident)    */
  double ring_us;        /* device part: first transfer to last reduce      */
  int64_t reduce_launches;
  int64_t reduce_elems;  /* elements reduced by this rank                   */
  int64_t bytes_sent, bytes_recv;
  /* host-side phase times of the last call (xgmi transport) */
  double sync_us;        /* waiting for the caller's pending GPU work       */
  double copy_us;        /* input -> exchange slot (H2D or D2D), synced     */
  double barrier_us;     /* meeting the other ranks                         */
  double kernel_us;      /* fold / gather launch + completion               */
  int32_t zero_copy;     /* xgmi: 1 = peers read this call's inputs in place */
  int32_t retried;       /* xgmi: 1 = redone with the slot copy (a peer input failed to map) */
  int64_t calls_redone;  /* xgmi: calls redone that way on this handle so far (cumulative) */
  double red_kernel_us;  /* P2P transports: summed kernel time of the reduce launches,
                            when PG_KERNEL_TIMING=1 stamps each launch (else 0) */
  int64_t red_kernel_bytes; /* algorithmic HBM bytes of those launches: 3*n*es per
                            ring reduce, (W+1)*n*es per direct fold            */
  /* which data path this handle runs (constant over the handle's life), so that a
     record of a run shows it: */
  int32_t transport;     /* PG_TRANSPORT_* actually in use (RCCL after an xgmi fallback) */
  int32_t algo_direct;   /* P2P transports: 1 = direct exchange, 0 = W-1 round ring */
  int32_t xgmi_push;     /* xgmi: 1 = push mode, 0 = read mode                   */
  int32_t xgmi_mode_auto;/* xgmi: 1 = the mode was chosen by the connect-time probe */
  double probe_read_gbs, probe_write_gbs;  /* that probe's medians over ranks (0 when forced) */
};
PG_API int pg_get_stats(void *pg_handle, struct pg_stats *out);

/* The TCP bootstrap star on its own (no GPU): join the ranks of `serverlist`
 * through hosts[0]:port, all-gather one int per rank into out[world], meet at
 * a barrier, disconnect.  Exercises the rank-0 relay that carries the RCCL
 * unique id and the xgmi IPC handles. */
PG_API int pgx_boot_selftest(const char *serverlist, int rank, int port, int value, int *out);

/* xgmi transport only, collective: the copy rates this node's links give
 * (pgk_gather launches, HIP events, `reps` launches of `bytes` per phase).
 * gbs[0] read one link (peer rank+1 -> me), gbs[1] write one link (me -> rank+1),
 * gbs[2] read from all peers at once, gbs[3] write to all peers at once;
 * 1e9 bytes/s moved by this rank.  bytes: a multiple of 4 KiB. */
PG_API int pgx_xgmi_link_probe(void *pg_handle, size_t bytes, int reps, double *gbs);

/* xgmi transport: the reduce-scatter mode in use (*push: 1 = each rank writes
 * every peer's block to it, 0 = each rank reads its block from every peer).
 * PG_XGMI_MODE=auto (the default) chose it at connect time with the link
 * probe above (32 MiB, all links at once): push when pushed bytes moved >= 15%
 * faster than pulled ones; *read_gbs / *write_gbs are that probe's medians over
 * ranks (0 when the mode was forced with PG_XGMI_MODE=read|push). */
PG_API int pgx_xgmi_mode(void *pg_handle, int *push, double *read_gbs, double *write_gbs);

/* Last error message of the calling thread ("" if none). */
PG_API const char *pg_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PG_EXT_H */
