/*
 * oracle/ref_driver.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Appended after the reference's extracted path lines (see ref_prelude.h).
 * Exposes the reference's static helpers and its collectives, driven with a
 * hand-filled struct pg {rank, world_size, chunk_bytes} (no connect_process_group,
 * which needs libibverbs), under ref_* names for ctypes.
 */
#include <time.h>

size_t ref_elem_size(int dt) { return elem_size((DATATYPE)dt); }
size_t ref_chunk_elems_from_bytes(size_t cb, int dt) { return chunk_elems_from_bytes(cb, (DATATYPE)dt); }
void ref_chunk_offsets(size_t count, size_t ce, int dt, size_t idx, size_t *off, size_t *len) {
    chunk_offsets(count, ce, (DATATYPE)dt, idx, off, len);
}
int ref_rs_send_chunk_index(int round, int rank, int world) { return rs_send_chunk_index(round, rank, world); }
int ref_rs_recv_chunk_index(int round, int rank, int world) { return rs_recv_chunk_index(round, rank, world); }
void ref_reduce_inplace(void *dst, const void *src, size_t n, int dt, int op) {
    reduce_inplace(dst, src, n, (DATATYPE)dt, (OPERATION)op);
}

static void ref_fill_pg(struct pg *pg, int rank, int world, size_t chunk_bytes) {
    memset(pg, 0, sizeof(*pg));
    pg->rank = rank;
    pg->world_size = world;
    pg->chunk_bytes = chunk_bytes;
}
int ref_reduce_scatter(int rank, int world, size_t chunk_bytes, void *s, void *r,
                       int count, int dt, int op) {
    struct pg pg; ref_fill_pg(&pg, rank, world, chunk_bytes);
    return pg_reduce_scatter(s, r, count, (DATATYPE)dt, (OPERATION)op, &pg);
}
int ref_all_gather(int rank, int world, void *s, void *r, int count, int dt) {
    struct pg pg; ref_fill_pg(&pg, rank, world, 4096);
    return pg_all_gather(s, r, count, (DATATYPE)dt, &pg);
}
int ref_all_reduce(int rank, int world, size_t chunk_bytes, void *s, void *r,
                   int count, int dt, int op) {
    struct pg pg; ref_fill_pg(&pg, rank, world, chunk_bytes);
    return pg_all_reduce(s, r, count, (DATATYPE)dt, (OPERATION)op, &pg);
}
/* CPU baseline: the reference's own reduce loop, `reps` times, seconds. */
double ref_time_reduce(void *dst, const void *src, size_t n, int dt, int op, int reps) {
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < reps; ++i) reduce_inplace(dst, src, n, (DATATYPE)dt, (OPERATION)op);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
