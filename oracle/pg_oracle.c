/*
 * oracle/pg_oracle.c -- TEST INFRASTRUCTURE ONLY (see pg_oracle.h).
 *
 * A plain-C restatement of the reference's collective path
 * (/root/reference/src/pg.c:104-179 helpers + reduce loop, :264-339 collectives)
 * plus a single-process simulator of the real W-rank ring that the MI355X
 * library executes.  Pinned against tests/golden/ (generated from the compiled
 * reference) and against oracle/_ref/libpgref.so when it is built.
 *
 * Nothing in the product library links or calls this file.
 */
#define _POSIX_C_SOURCE 199309L
#include "pg_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---- helpers: reference src/pg.c:109-148 --------------------------------- */

size_t orc_elem_size(int dt) {                       /* src/pg.c:109-115 */
    if (dt == ORC_DT_INT32) return 4;
    if (dt == ORC_DT_DOUBLE) return 8;
    return 0;
}

size_t orc_chunk_elems_from_bytes(size_t chunk_bytes, int dt) {   /* :118-123 */
    size_t es = orc_elem_size(dt);
    if (es == 0) return 0;
    size_t e = chunk_bytes / es;
    return e ? e : 1;                                /* at least one element */
}

void orc_chunk_offsets(size_t count, size_t chunk_elems, int dt, size_t idx,
                       size_t *off, size_t *len) {   /* :126-138 */
    size_t es = orc_elem_size(dt);
    size_t first = idx * chunk_elems;
    if (first >= count) { *off = 0; *len = 0; return; }
    size_t last = first + chunk_elems;               /* clamp to count */
    if (last > count) last = count;
    *off = first * es;
    *len = (last - first) * es;
}

int orc_rs_send_chunk_index(int round, int rank, int world) {  /* :141-143 */
    return ((rank - round) % world + world) % world;
}

int orc_rs_recv_chunk_index(int round, int rank, int world) {  /* :146-148 */
    return ((rank - round - 1) % world + world) % world;
}

/* ---- the hot loop: src/pg.c:151-159 ---------------------------------------
 * int32 arithmetic is done on uint32_t: the reference relies on signed
 * overflow wrapping (C UB, but gcc emits add/imul which wrap); unsigned
 * arithmetic gives the same bits without UB.  double: one IEEE op/element.
 * The loop keeps the reference's shape (op tested per element, scalar, -O2)
 * so that, timed as the CPU baseline, it runs like the reference loop. */
void orc_reduce_inplace(void *dst, const void *src, size_t n, int dt, int op) {
    if (dt == ORC_DT_INT32) {
        uint32_t *d = (uint32_t *)dst;
        const uint32_t *s = (const uint32_t *)src;
        for (size_t i = 0; i < n; ++i) d[i] = (op == ORC_OP_SUM) ? d[i] + s[i] : d[i] * s[i];
    } else if (dt == ORC_DT_DOUBLE) {
        double *d = (double *)dst;
        const double *s = (const double *)src;
        for (size_t i = 0; i < n; ++i) d[i] = (op == ORC_OP_SUM) ? d[i] + s[i] : d[i] * s[i];
    }
}

/* src/pg.c:166-179: n whole elements reduced, `bytes % es` tail copied. */
static void orc_sendrecv_mock(void *sendbuf, void *recvbuf, size_t bytes, int dt, int op) {
    size_t es = orc_elem_size(dt);
    size_t n = es ? bytes / es : 0;
    if (n) orc_reduce_inplace(recvbuf, sendbuf, n, dt, op);
    size_t tail = es ? bytes % es : 0;
    if (tail) memcpy((char *)recvbuf + n * es, (char *)sendbuf + n * es, tail);
}

/* ---- reference mock collectives, one rank ---------------------------------- */

int orc_mock_reduce_scatter(int rank, int world, size_t chunk_bytes, void *sendbuf,
                            void *recvbuf, int count, int dt, int op) {  /* :264-291 */
    if (!sendbuf || !recvbuf || count < 0 || orc_elem_size(dt) == 0) return -1;
    size_t es = orc_elem_size(dt);
    if (world == 1) { memcpy(recvbuf, sendbuf, (size_t)count * es); return 0; }
    size_t ce = orc_chunk_elems_from_bytes(chunk_bytes, dt);
    for (int k = 0; k + 1 < world; ++k) {
        size_t so, sl, ro, rl;
        orc_chunk_offsets((size_t)count, ce, dt, (size_t)orc_rs_send_chunk_index(k, rank, world), &so, &sl);
        orc_chunk_offsets((size_t)count, ce, dt, (size_t)orc_rs_recv_chunk_index(k, rank, world), &ro, &rl);
        (void)sl;  /* the reference uses recv_len for both sides (:287) */
        if (rl) orc_sendrecv_mock((char *)sendbuf + so, (char *)recvbuf + ro, rl, dt, op);
    }
    return 0;
}

int orc_mock_all_gather(int rank, int world, void *sendbuf, void *recvbuf,
                        int count, int dt) {                             /* :293-321 */
    if (!recvbuf || count < 0 || orc_elem_size(dt) == 0) return -1;
    size_t slot = (size_t)count * orc_elem_size(dt);
    if (sendbuf) memcpy((char *)recvbuf + (size_t)rank * slot, sendbuf, slot);
    if (world == 1) return 0;
    for (int k = 0; k + 1 < world; ++k) {
        int s = ((rank - k) % world + world) % world;
        int r = ((rank - k - 1) % world + world) % world;
        /* the mock reduces with OP_SUM rather than copying (:317) */
        orc_sendrecv_mock((char *)recvbuf + (size_t)s * slot,
                          (char *)recvbuf + (size_t)r * slot, slot, dt, ORC_OP_SUM);
    }
    return 0;
}

int orc_mock_all_reduce(int rank, int world, size_t chunk_bytes, void *sendbuf,
                        void *recvbuf, int count, int dt, int op) {      /* :323-339 */
    if (!sendbuf || !recvbuf || count < 0) return -1;
    if (sendbuf != recvbuf) memcpy(recvbuf, sendbuf, (size_t)count * orc_elem_size(dt));
    if (orc_mock_reduce_scatter(rank, world, chunk_bytes, recvbuf, recvbuf, count, dt, op)) return -1;
    /* For world > 1 the reference's all-gather step writes past a count-element
     * buffer (:303, :313-317); that shape has no defined answer to restate. */
    if (world > 1) return -2;
    return orc_mock_all_gather(rank, world, recvbuf, recvbuf, count, dt);
}

/* ---- real-ring semantics --------------------------------------------------- */

void orc_ring_block(size_t count, int world, int b, size_t *off_elems, size_t *len_elems) {
    /* the reference's chunk_offsets() clamping (src/pg.c:126-138), in
     * elements, with the ring block ceil(count/W) as the chunk */
    size_t be = (count + (size_t)world - 1) / (size_t)world;
    if (be == 0) be = 1;
    size_t first = (size_t)b * be;
    if (first >= count) { *off_elems = 0; *len_elems = 0; return; }
    size_t last = first + be;
    if (last > count) last = count;
    *off_elems = first;
    *len_elems = last - first;
}

/* Step of ring g of `rings` over `world` ranks (include/pg_ext.h "Rings"):
 * +1, -1, then +3, -3, +5, ... kept when coprime with world and not yet used
 * mod world; when they run out the list repeats.  Ring 0 (+1) is the
 * reference's ring (README.md:68-71, rs_{send,recv}_chunk_index at
 * src/pg.c:141-148); the further rings are this build's extension (rings over
 * further xGMI links), restated here independently of the library's code. */
int orc_ring_step(int world, int rings, int g) {
    int offs[4] = {1, -1}, m = 2;
    for (int c = 3; m < 4 && c < 2 * world; c += 2) {
        for (int sgn = 1; sgn >= -1 && m < 4; sgn -= 2) {
            int d = sgn * c, rd = ((d % world) + world) % world, a = rd, b = world;
            while (b) { int t = a % b; a = b; b = t; }          /* a = gcd(rd, world) */
            if (rd == 0 || a != 1) continue;
            int dup = 0;
            for (int i = 0; i < m; ++i) dup |= ((offs[i] % world) + world) % world == rd;
            if (!dup) offs[m++] = d;
        }
    }
    (void)rings;
    return offs[g % m];
}

int orc_ring_reduce_scatter(int world, void *const *sends, void *const *outs,
                            int count, int dt, int op, int rings) {
    size_t es = orc_elem_size(dt);
    if (world < 1 || count < 0 || es == 0 || rings < 1 || rings > 4) return -1;
    for (int b = 0; b < world; ++b) {
        size_t off, len;
        orc_ring_block((size_t)count, world, b, &off, &len);
        if (!len) continue;
        /* part g = [ceil(g*len/R), ceil((g+1)*len/R)) rides the ring of step d:
         * acc = x[b+d]; acc = acc op x[b+j*d], j = 2 .. W  (x[b+W*d] = x[b]).
         * One ring: the whole block, d = +1; two: d = +1 then -1. */
        for (int g = 0; g < rings; ++g) {
            size_t po = ((size_t)g * len + (size_t)rings - 1) / (size_t)rings;
            size_t pe = ((size_t)(g + 1) * len + (size_t)rings - 1) / (size_t)rings;
            size_t pl = pe - po;
            if (!pl) continue;
            char *acc = (char *)outs[b] + po * es;
            int step = ((orc_ring_step(world, rings, g) % world) + world) % world;
            memcpy(acc, (const char *)sends[(b + step) % world] + (off + po) * es, pl * es);
            for (int j = 2; j <= world; ++j)
                orc_reduce_inplace(acc, (const char *)sends[(b + j * step) % world] + (off + po) * es, pl, dt, op);
        }
    }
    return 0;
}

int orc_ring_all_gather(int world, void *const *sends, void *const *recvs,
                        int count, int dt) {
    size_t es = orc_elem_size(dt);
    if (world < 1 || count < 0 || es == 0) return -1;
    size_t slot = (size_t)count * es;
    for (int r = 0; r < world; ++r)
        for (int q = 0; q < world; ++q)
            memcpy((char *)recvs[r] + (size_t)q * slot, sends[q], slot);
    return 0;
}

int orc_ring_all_reduce(int world, void *const *sends, void *const *recvs,
                        int count, int dt, int op, int rings) {
    size_t es = orc_elem_size(dt);
    if (world < 1 || count < 0 || es == 0) return -1;
    size_t total = (size_t)count * es;
    char *full = (char *)malloc(total ? total : 1);
    void **outs = (void **)malloc(sizeof(void *) * (size_t)world);
    if (!full || !outs) { free(full); free(outs); return -1; }
    for (int b = 0; b < world; ++b) {
        size_t off, len;
        orc_ring_block((size_t)count, world, b, &off, &len);
        outs[b] = full + off * es;
    }
    int rc = orc_ring_reduce_scatter(world, sends, outs, count, dt, op, rings);
    for (int r = 0; rc == 0 && r < world; ++r) memcpy(recvs[r], full, total);
    free(outs); free(full);
    return rc;
}

/* ---- synthetic inputs ------------------------------------------------------ */

uint64_t orc_splitmix64(uint64_t *state) {
    uint64_t z = (*state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_fill(void *buf, size_t n, int dt, int op, uint64_t seed) {
    uint64_t st = seed;
    if (dt == ORC_DT_INT32) {
        uint32_t *p = (uint32_t *)buf;
        for (size_t i = 0; i < n; ++i) p[i] = (uint32_t)(orc_splitmix64(&st) >> 32);
    } else {
        double *p = (double *)buf;
        const double u = 1.0 / 9007199254740992.0;     /* 2^-53 */
        for (size_t i = 0; i < n; ++i) {
            double x = (double)(orc_splitmix64(&st) >> 11) * u * 2.0 - 1.0;  /* U[-1,1) */
            p[i] = (op == ORC_OP_SUM) ? x : 1.0 + x * (1.0 / 1024.0);
        }
    }
}

double orc_time_reduce(void *dst, const void *src, size_t n, int dt, int op, int reps) {
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < reps; ++i) orc_reduce_inplace(dst, src, n, dt, op);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
