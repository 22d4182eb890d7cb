/*
 * include/pgk.h -- thin C-ABI from the host schedule to the MI355X (gfx950)
 * reduction kernels.  Plain pointers and sizes only; no HIP or torch types.
 *
 * This is the inner boundary of the drop-in: the reference's
 *   static void reduce_inplace(void *dst, const void *src, size_t n,
 *                              DATATYPE dt, OPERATION op)        (src/pg.c:151-159)
 * called once per arriving segment by pg_sendrecv_mock (src/pg.c:166-179, call
 * at :172) becomes pgk_reduce(), called once per arriving segment by the ring
 * executor in libpg_amd.so.
 *
 * All device pointers are HIP device (or managed) allocations on the current
 * device.  `stream` is a hipStream_t passed as void* (NULL = the null stream).
 * Calls are asynchronous on `stream`, allocate nothing and are safe to capture
 * into a hipGraph.  Return 0 on success, -1 on failure (message via
 * pgk_last_error()).
 */
#ifndef PGK_H
#define PGK_H

#ifndef PG_API
#define PG_API __attribute__((visibility("default")))
#endif

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same values as DATATYPE / OPERATION in include/pg.h (reference pg.h:78-87). */
#define PGK_DT_INT32  0
#define PGK_DT_DOUBLE 1
#define PGK_OP_SUM    0
#define PGK_OP_PROD   1

/* dst[i] = dst[i] op src[i] for i < n.  Replaces reduce_inplace
 * (reference src/pg.c:151-159): int32 wraps (two's complement), double is one
 * IEEE-754 add or multiply per element (round-to-nearest, denormals kept), so
 * results are bit-identical to the reference loop for every non-NaN result.
 * dst == src is allowed; dst and src overlapping at different addresses is
 * refused (-1): the reference loop's element-by-element order is not what a
 * parallel launch would compute there.
 * n == 0 is a no-op returning 0.  dt/op outside the values above -> -1.
 * Above 512 MiB per operand the call is several back-to-back launches on
 * `stream` (each at most 512 MiB), which measure faster than one. */
PG_API int pgk_reduce(void *dst, const void *src, size_t n, int dt, int op, void *stream);

/* out[i] = a[i] op b[i] (out may equal a or b; any other overlap of out with
 * an operand is refused).  Same numerics as pgk_reduce;
 * used where the ring must not modify the caller's send buffer. */
PG_API int pgk_reduce_out(void *out, const void *a, const void *b, size_t n, int dt, int op,
                   void *stream);

/* Up to 8 independent ranges in one launch: outs[j][i] = as[j][i] op bs[j][i]
 * for i < ns[j] (out may equal a or b within a range; ranges must not overlap
 * each other).  Same numerics as pgk_reduce.  The ring executor reduces every
 * ring's arrived segments with one call.  start_event/stop_event
 * (hipEvent_t as void*, may be NULL) receive the kernel's own begin/end
 * timestamps as in pgk_reduce_timed; ranges that cannot share one launch
 * (not 16-byte congruent) are launched one by one, stamped first-to-last. */
PG_API int pgk_reduce_ranges(void *const *outs, const void *const *as, const void *const *bs, const size_t *ns,
                             int k, int dt, int op, void *stream, void *start_event, void *stop_event);

/* out[i] = ((srcs[0][i] op srcs[1][i]) op srcs[2][i]) ... op srcs[nsrc-1][i],
 * folded left to right (1 <= nsrc <= 16).  Sources may be peer GPUs' memory
 * mapped through HIP IPC (read over xGMI; a caller whose sources are mostly
 * remote says so through pgk_fold_timed below).  With srcs in ring order this
 * is bit-identical to the W-1 ring steps of reduce_inplace it fuses. */
PG_API int pgk_reduce_multi(void *out, const void *const *srcs, int nsrc, size_t n, int dt, int op,
                     void *stream);
/* The same launch with the kernel's own begin/end timestamps recorded into two
 * HIP events (as pgk_reduce_timed; NULL events = untimed).
 * From 5 to 8 sources and 32 MiB per source both calls take the burst form:
 * launches of at most 64 MiB per source in which every wave folds all its
 * tiles before it stores any (the chip reads, then writes), 80-84% of the HBM
 * peak against 73-75% for one tile per wave; the events then stamp the first
 * launch's begin and the last one's end.  out may be one of the sources. */
PG_API int pgk_reduce_multi_timed(void *out, const void *const *srcs, int nsrc, size_t n, int dt, int op,
                                  void *stream, void *start_event, void *stop_event);
/* pgk_reduce_multi_timed with what the caller knows about the launch:
 *   PGK_FOLD_REMOTE_SOURCES  the sources are mostly peers' memory read over
 *       xGMI: the links bound the rate, and the burst form (tuned on local HBM)
 *       is not used;
 *   PGK_FOLD_SHARED_GPU  other kernels (a transport's sends and receives) are
 *       resident while the fold runs: the burst form is cut into 32 MiB
 *       launches that use half of every CU's registers (79% of the peak, and
 *       the same beside other kernels), where the 64 MiB launches of a fold
 *       that has the GPU to itself (82-84%) fall to 69% beside eight foreign
 *       workgroups.
 * Same bits in every form.  Unknown flags -> -1. */
#define PGK_FOLD_REMOTE_SOURCES 1u
#define PGK_FOLD_SHARED_GPU 2u
PG_API int pgk_fold_timed(void *out, const void *const *srcs, int nsrc, size_t n, int dt, int op, unsigned flags,
                          void *stream, void *start_event, void *stop_event);

/* How pgk_fold_timed would cut a fold of n elements per source (operands
 * 16-byte aligned) with these flags: returns the number of burst launches and
 * fills the first max_launches entries of launch_bytes (bytes per source) and
 * launch_tiles (tiles per wave); *plain_bytes = what is folded one tile per
 * wave (everything, when the burst form does not apply).  Host arithmetic
 * only: for tests and benches. */
PG_API int pgk_fold_geometry(size_t n, int dt, int nsrc, unsigned flags, size_t *launch_bytes, int *launch_tiles,
                             int max_launches, size_t *plain_bytes);

/* One-shot all-reduce fold: element i lies in ring block b = i / block_elems
 * and out[i] = srcs[(b+1)%k][i] op srcs[(b+2)%k][i] op ... op srcs[b][i]
 * (k = nsrc; requires ceil(n / block_elems) <= k): block b folded in exactly
 * the order the ring reduce-scatter uses for it.  rings = R (1 .. 4): part g
 * of each block ([ceil(g*len_b/R), ceil((g+1)*len_b/R)), include/pg_ext.h) is
 * folded srcs[(b+d)%k] op srcs[(b+2d)%k] op ... op srcs[b] with d the step of
 * ring g (+1, -1, +3, -3 as pg_ring_offset gives them for world = k). */
PG_API int pgk_fold_blocks(void *out, const void *const *srcs, int nsrc, size_t n, size_t block_elems,
                           int rings, int dt, int op, void *stream);

/* Copy k <= 16 byte ranges srcs[j] -> dsts[j] (bytes[j] each, 4-byte aligned,
 * sources may be peer memory) in one launch. */
PG_API int pgk_gather(void *const *dsts, const void *const *srcs, const size_t *bytes, int k, void *stream);

/* No counterpart in the reference.  For callers that cannot allocate device
 * memory: code under HIP graph capture, tight serving loops, harnesses that
 * forbid hipMalloc.  It is the all-reduce of pgx_sim_run(coll =
 * PG_COLL_ALL_REDUCE) (include/pg_ext.h) over `world` (1 .. 16) device buffers
 * of the calling process on the current device, with that call's exchange
 * area (which pgx_sim_run allocates) replaced by a fixed device array inside
 * the library:
 *     recvbufs[r][0..count) = the ring all-reduce of sendbufs[0..world)[0..count)
 * for every r, block b = [b*B, min((b+1)*B, count)), B = ceil(count/world),
 * part g of `rings` folded in its ring's order (pgk_fold_blocks), so the bits
 * equal pgx_sim_run's and pg_all_reduce's.  sendbufs[r] == recvbufs[r] (in
 * place) is allowed; other overlaps are not.  Two launches on `stream`
 * (inputs -> exchange slots, fold -> every output), asynchronous; it calls no
 * hipMalloc / hipFree or other allocating routine.
 * Limit: world * round_up(count * elem_size, 256) <= PGK_STAGED_MAX_BYTES,
 * else -1 with a message.  Every GPU the library is used on holds that many
 * bytes from the library's load to the end of the process.
 * The array's address is resolved once per device by the first call made with
 * that device current (a count == 0 call does only that; make it outside any
 * stream capture).  All calls on one GPU share the one array: calls that
 * overlap in time on the same GPU (different streams or threads) race. */
#define PGK_STAGED_MAX_BYTES (16u << 20)
PG_API int pgk_all_reduce_staged(void *const *sendbufs, void *const *recvbufs, int world, size_t count,
                                 int rings, int dt, int op, void *stream);

/* Device helpers for hosts that do not link HIP themselves (ctypes, cgo ...). */
PG_API int pgk_device_count(int *count);
PG_API int pgk_set_device(int device);
PG_API int pgk_synchronize(void);

/* Launch tuning, process-wide.  blocks_per_cu: grid cap = CUs x blocks_per_cu
 * (0 = uncapped one-shot grid, <0 = keep).  nontemporal: 1 = nt loads/stores,
 * 0 = default cache policy, <0 = keep.  Defaults are the measured best
 * on MI355X. */
PG_API int pgk_tune(int blocks_per_cu, int nontemporal);

/* burst: 1 = pgk_reduce_multi may take its burst form (default), 0 = never,
 * <0 = keep.  Process-wide; results are bit-identical either way. */
PG_API int pgk_tune_fold(int burst);

/* Vector-kernel shape: threads per block x 16-byte vectors per operand each
 * thread keeps in flight.  Instantiated: 256x2, 256x4, 256x8, 512x2, 1024x1;
 * 0x0 (the default) picks by operand size (512x2 below 128 MiB, else 1024x1). */
PG_API int pgk_tune_shape(int block, int unroll);

/* pgk_reduce, with the kernel's own begin/end timestamps recorded into two
 * HIP events (hipEvent_t as void*, from pgk_event_create) through
 * hipExtLaunchKernelGGL: their elapsed time is the kernel's execution, without
 * the dispatch overhead of separate event markers.  Used by bench.py. */
PG_API int pgk_reduce_timed(void *dst, const void *src, size_t n, int dt, int op, void *stream,
                     void *start_event, void *stop_event);
PG_API int pgk_event_create(void **event);
PG_API int pgk_event_destroy(void *event);
PG_API int pgk_event_elapsed_ms(void *start_event, void *stop_event, float *ms);

/* Grid the next pgk_reduce of n elements of dt would launch (for bench/tests).
 * A call above 512 MiB per operand is cut into equal launches of at most
 * 512 MiB (pgk_reduce.hip, kSplitBytes); this reports the first of them. */
PG_API int pgk_launch_geometry(size_t n, int dt, unsigned *grid, unsigned *block);

/* Last error message of the calling thread ("" if none). */
PG_API const char *pgk_last_error(void);

/* Build identification, e.g. "pgk gfx950 hip-7.2". */
PG_API const char *pgk_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PGK_H */
