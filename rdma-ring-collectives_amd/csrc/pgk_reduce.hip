// pgk_reduce.hip -- CDNA4 (gfx950) element-wise reduction kernels + C-ABI.
//
// Replaces the reference's scalar hot loop reduce_inplace (src/pg.c:151-159):
//     d[i] = (op == OP_SUM) ? d[i] + s[i] : d[i] * s[i]     for int32 / double
//
// The op is HBM-bound (1 arithmetic op per 12 B (int32) or 24 B (double) of
// traffic), so there is no MFMA and no LDS: every lane streams 16-byte vectors
// (global_load_dwordx4 / global_store_dwordx4), each wave moves 1 KiB per
// instruction per operand, and each thread keeps kUnroll independent vector
// pairs in flight to cover HBM latency.  The op and dtype are template
// parameters, so the per-element `op` test of the reference disappears.
//
// Numerics (bit-exact vs the reference loop):
//   int32  -> uint32 add / mul_lo (two's-complement wrap, what gcc emits)
//   double -> one v_add_f64 / v_mul_f64 per element, RNE, denormals preserved
//             (built without -ffast-math / denormal flushing); no FMA is
//             possible because each element sees exactly one operation.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>

#include "pgk.h"

namespace {

// Vector kernel shape (threads per block kBlock, 16-B vectors per operand per
// thread per iteration kUnroll) is a template; pgk_tune_shape picks one of the
// instantiated pairs at run time.  Every pair moves 16 KiB per operand per
// block iteration except 256x8 (32 KiB).
constexpr int kScalarBlock = 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <typename T> struct VecOf;
template <> struct VecOf<uint32_t> { using type = u32x4; static constexpr int width = 4; };
template <> struct VecOf<double> { using type = f64x2; static constexpr int width = 2; };

template <int OP, typename X>
__device__ __forceinline__ X apply(X a, X b) {
  if constexpr (OP == PGK_OP_SUM) return a + b;
  else return a * b;
}

template <bool NT, typename X>
__device__ __forceinline__ X ld(const X* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NT, typename X>
__device__ __forceinline__ void st(X* p, X v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// out = a op b over [head elements | nvec 16-B vectors | tail elements].
// The vector region starts at element `head` and is 16-B aligned in all three
// pointers; head/tail (< one vector each) are done by the first threads of
// block 0.  Grid-strided so the host can cap the grid.  `bid` / `nblocks` are
// this block's index and the block count of the range it works on (the whole
// grid for k_reduce_vec, one range's share for k_reduce_ranges).
template <typename T, int OP, bool NT, int kBlock, int kUnroll>
__device__ __forceinline__ void reduce_vec_body(T* __restrict__ out, const T* __restrict__ a,
                                                const T* __restrict__ b, unsigned head, size_t nvec,
                                                unsigned tail, unsigned bid, unsigned nblocks) {
  using V = typename VecOf<T>::type;
  constexpr int W = VecOf<T>::width;
  if (bid == 0 && threadIdx.x < head + tail) {
    size_t e = threadIdx.x < head ? threadIdx.x
                                  : head + nvec * W + (threadIdx.x - head);
    out[e] = apply<OP>(a[e], b[e]);
  }
  V* __restrict__ vo = reinterpret_cast<V*>(out + head);
  const V* __restrict__ va = reinterpret_cast<const V*>(a + head);
  const V* __restrict__ vb = reinterpret_cast<const V*>(b + head);
  const size_t tile = (size_t)kBlock * kUnroll;
  const size_t stride = (size_t)nblocks * tile;
  size_t i = (size_t)bid * tile + threadIdx.x;
  // full tiles: no bounds checks, kUnroll independent loads per operand
  for (; i + (kUnroll - 1) * kBlock < nvec; i += stride) {
    V x[kUnroll], y[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) x[u] = ld<NT>(va + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) y[u] = ld<NT>(vb + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) st<NT>(vo + i + u * kBlock, apply<OP>(x[u], y[u]));
  }
  // the one partial tile (at most one per grid)
  if (i < nvec) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      size_t j = i + u * kBlock;
      if (j < nvec) st<NT>(vo + j, apply<OP>(ld<NT>(va + j), ld<NT>(vb + j)));
    }
  }
}

template <typename T, int OP, bool NT, int kBlock, int kUnroll>
__global__ __launch_bounds__(kBlock) void k_reduce_vec(T* __restrict__ out,
                                                       const T* __restrict__ a,
                                                       const T* __restrict__ b,
                                                       unsigned head, size_t nvec,
                                                       unsigned tail) {
  reduce_vec_body<T, OP, NT, kBlock, kUnroll>(out, a, b, head, nvec, tail, blockIdx.x, gridDim.x);
}

// Several independent ranges in one launch: range j covers blocks
// [first[j], first[j+1]) of the grid and computes out[j] = a[j] op b[j] with
// the same body as k_reduce_vec.  One launch instead of one per range: the
// ring executor reduces every ring's arrived segments at once (they lie in
// different blocks of the buffers), so the launch ramp and tail are paid once
// per launch, not once per ring.
constexpr int kMaxRanges = 8;
template <typename T>
struct RangeList {
  T* out[kMaxRanges];
  const T* a[kMaxRanges];
  const T* b[kMaxRanges];
  size_t nvec[kMaxRanges];
  unsigned head[kMaxRanges];
  unsigned tail[kMaxRanges];
  unsigned first[kMaxRanges + 1];
  int k;
};

template <typename T, int OP, bool NT, int kBlock, int kUnroll>
__global__ __launch_bounds__(kBlock) void k_reduce_ranges(RangeList<T> rl) {
  int r = 0;
  while (r + 1 < rl.k && blockIdx.x >= rl.first[r + 1]) ++r;
  reduce_vec_body<T, OP, NT, kBlock, kUnroll>(rl.out[r], rl.a[r], rl.b[r], rl.head[r], rl.nvec[r], rl.tail[r],
                                               blockIdx.x - rl.first[r], rl.first[r + 1] - rl.first[r]);
}

// Fallback when the three pointers are not mutually 16-B congruent (e.g. a
// segment starting at an odd element of an int32 buffer): element-wise, still
// coalesced (lane i touches element i).
template <typename T, int OP>
__global__ __launch_bounds__(kScalarBlock) void k_reduce_scalar(T* __restrict__ out,
                                                                const T* __restrict__ a,
                                                                const T* __restrict__ b,
                                                                size_t n) {
  const size_t stride = (size_t)gridDim.x * kScalarBlock;
  for (size_t i = (size_t)blockIdx.x * kScalarBlock + threadIdx.x; i < n; i += stride)
    out[i] = apply<OP>(a[i], b[i]);
}

// Multi-source fold: out[i] = ((s0[i] op s1[i]) op s2[i]) ... op s[k-1][i], left
// to right, each source a different rank's buffer (IPC-mapped peer memory over
// xGMI, or local).  One element sees exactly the operation sequence the ring
// would apply, so the result is bit-identical to a W-step ring reduction in
// the same order.  Sources are passed by value in the kernel arguments.
constexpr int kMaxSrc = 16;
constexpr int kMultiBlock = 256;
// The vector fold streams k sources + 1 output.  Block shapes of 256, 512 and
// 1024 threads measure within run-to-run noise of each other (5.6-6.3 TB/s of
// 9 x 64 MiB .. 9 x 1 GiB at k = 8, profiles/r01_lab3_fold.txt); 512 is the middle.
constexpr int kMultiVecBlock = 512;
template <typename T>
struct SrcList {
  const T* p[kMaxSrc];
};

template <typename T, int OP, int NS>
__global__ __launch_bounds__(kMultiVecBlock) void k_reduce_multi_vec(T* __restrict__ out, SrcList<T> src,
                                                                  int nsrc, unsigned head, size_t nvec,
                                                                  unsigned tail) {
  using V = typename VecOf<T>::type;
  constexpr int W = VecOf<T>::width;
  const int k = NS ? NS : nsrc;
  if (blockIdx.x == 0 && threadIdx.x < head + tail) {
    size_t e = threadIdx.x < head ? threadIdx.x : head + nvec * W + (threadIdx.x - head);
    T acc = src.p[0][e];
    for (int j = 1; j < k; ++j) acc = apply<OP>(acc, src.p[j][e]);
    out[e] = acc;
  }
  const size_t stride = (size_t)gridDim.x * kMultiVecBlock;
  size_t i = (size_t)blockIdx.x * kMultiVecBlock + threadIdx.x;
  if constexpr (NS > 0) {
    const V* vs[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) vs[j] = reinterpret_cast<const V*>(src.p[j] + head);
    V* vo = reinterpret_cast<V*>(out + head);
    // one vector per thread: the grid covers nvec except past 2^32 work-items
    for (; i < nvec; i += stride) {
      V x[NS];
#pragma unroll
      for (int j = 0; j < NS; ++j) x[j] = ld<true>(vs[j] + i);
      V acc = x[0];
#pragma unroll
      for (int j = 1; j < NS; ++j) acc = apply<OP>(acc, x[j]);
      st<true>(vo + i, acc);
    }
    return;
  }
  for (; i < nvec; i += stride) {          // nsrc > 8: sources in a runtime loop
    V acc = ld<true>(reinterpret_cast<const V*>(src.p[0] + head) + i);
    for (int j = 1; j < k; ++j) acc = apply<OP>(acc, ld<true>(reinterpret_cast<const V*>(src.p[j] + head) + i));
    st<true>(reinterpret_cast<V*>(out + head) + i, acc);
  }
}

// The same fold with its stores gathered into one burst per launch.  HBM
// serves a thin stream of writes spread through many read streams badly: the
// fold above, one tile per wave and a store right behind its loads, streams
// at 73-75% of the peak from five sources up, where its reads alone reach 85-88%
// (tools/lab/run_mix_lab.py: the same bytes written cost 0.17 us per MiB as a
// dense stream and 0.46 us per MiB spread through eight read streams).  Here
// every wave folds U tiles into registers, reads only, and stores its U results
// at the end; the grid is one-shot and every workgroup is resident at once, so
// the chip reads for most of the launch and then writes.  What a launch may
// hold is what the resident waves' registers hold, and the form only works
// with a whole number of workgroups per CU, all of them resident from the
// start (a launch of 576 or 640 workgroups runs at 64-76%; workgroups that
// must wait for a free CU run as a second round behind the first):
//   512 workgroups x 32 tiles (64 MiB per source; two per CU at ~220 VGPRs, a
//       CU's whole register file): 82-84% on a GPU the fold has to itself,
//       69% as soon as eight workgroups of another kernel are resident;
//   768 x 16 (48 MiB; three per CU at ~124 VGPRs): 80-81%;
//   512 x 16 (32 MiB; two per CU, half the register file): 79%, and the same
//       beside 128 resident workgroups of 256 lanes x 128 VGPRs; it also fits
//       beside waves of 256 VGPRs, which RCCL's kernels are
// (tools/lab/burst_occupied_probe2.py).  So a fold that has the GPU to itself
// is cut into 64 MiB launches and a last one of 32 .. 64 MiB at 16 tiles per
// wave (up to four workgroups per CU; between whole numbers per CU it runs at
// 76-78%, still above one tile per wave), and one that runs beside
// communication kernels (PGK_FOLD_SHARED_GPU) into 32 MiB ones.  It does not pay below five sources
// or 32 MiB per source.
// A lane reads its elements of every source before it writes them, so out may
// be one of the sources, as in the kernel above.
constexpr int kBurstBlock = 256;
constexpr int kBurstBlocks = 512;                  // workgroups per launch: two per CU
constexpr size_t kBurstMinBytes = 32u << 20;       // per source, whole call
constexpr size_t kBurstVecs32 = (size_t)kBurstBlocks * kBurstBlock * 32;       // 64 MiB per source
constexpr size_t kBurstVecs16 = (size_t)kBurstBlocks * kBurstBlock * 16;       // 32 MiB

template <typename T, int OP, int NS, int U>
__global__ __launch_bounds__(kBurstBlock) void k_reduce_multi_burst(T* __restrict__ out, SrcList<T> src,
                                                                    unsigned head, size_t v0, size_t v1,
                                                                    unsigned edge_head, unsigned edge_tail,
                                                                    size_t tail_e) {
  using V = typename VecOf<T>::type;
  // the call's unaligned edge elements, on its first launch only
  if (blockIdx.x == 0 && threadIdx.x < edge_head + edge_tail) {
    const size_t e = threadIdx.x < edge_head ? threadIdx.x : tail_e + (threadIdx.x - edge_head);
    T acc = src.p[0][e];
#pragma unroll
    for (int j = 1; j < NS; ++j) acc = apply<OP>(acc, src.p[j][e]);
    out[e] = acc;
  }
  const V* vs[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) vs[j] = reinterpret_cast<const V*>(src.p[j] + head);
  V* vo = reinterpret_cast<V*>(out + head);
  const size_t base = v0 + (size_t)blockIdx.x * (kBurstBlock * U) + threadIdx.x;
  V r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + (size_t)u * kBurstBlock;
    if (i < v1) {
      V x[NS];
#pragma unroll
      for (int j = 0; j < NS; ++j) x[j] = ld<true>(vs[j] + i);
      V acc = x[0];
#pragma unroll
      for (int j = 1; j < NS; ++j) acc = apply<OP>(acc, x[j]);
      r[u] = acc;
    }
  }
  asm volatile("" ::: "memory");         // no store is scheduled among the loads
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + (size_t)u * kBurstBlock;
    if (i < v1) st<true>(vo + i, r[u]);
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(kMultiBlock) void k_reduce_multi_scalar(T* __restrict__ out, SrcList<T> src,
                                                                     int nsrc, size_t n) {
  const size_t stride = (size_t)gridDim.x * kMultiBlock;
  for (size_t i = (size_t)blockIdx.x * kMultiBlock + threadIdx.x; i < n; i += stride) {
    T acc = src.p[0][i];
    for (int j = 1; j < nsrc; ++j) acc = apply<OP>(acc, src.p[j][i]);
    out[i] = acc;
  }
}

// One-shot all-reduce fold: element i belongs to ring block b = i / block_elems
// and is folded in that block's ring order -- the order the reduce-scatter
// uses for it -- so every rank computing the whole vector this way gets the
// all-reduce result bit for bit.  Block b (length len) is cut into `rings`
// parts, part g = [ceil(g*len/R), ceil((g+1)*len/R)), and part g travels the
// ring of step d_g (include/pg_ext.h): src[(b+d)%k] op src[(b+2d)%k] ... op
// src[b].  steps[g] = d_g mod k.  Used for small messages, where one launch
// beats reduce-scatter + gather.
constexpr int kMaxRings = 4;
struct RingSteps {
  int d[kMaxRings];
};

template <typename T, int OP>
__global__ __launch_bounds__(kMultiBlock) void k_fold_blocks(T* __restrict__ out, SrcList<T> src, int k,
                                                             size_t n, size_t block_elems, int rings,
                                                             RingSteps steps) {
  const size_t stride = (size_t)gridDim.x * kMultiBlock;
  for (size_t i = (size_t)blockIdx.x * kMultiBlock + threadIdx.x; i < n; i += stride) {
    const int b = (int)(i / block_elems);
    const size_t b0 = (size_t)b * block_elems;
    const size_t len = n - b0 < block_elems ? n - b0 : block_elems;
    const int g = (int)((i - b0) * (size_t)rings / len);     // ceil(g*len/R) <= p  <=>  g <= p*R/len
    const int step = steps.d[g];
    int q = b + step >= k ? b + step - k : b + step;
    T acc = src.p[q][i];
    for (int j = 1; j < k; ++j) {
      q = q + step >= k ? q + step - k : q + step;
      acc = apply<OP>(acc, src.p[q][i]);
    }
    out[i] = acc;
  }
}

// k_fold_blocks with the result stored to `nout` buffers at once (every rank
// of an all-reduce receives the same vector): the fold is computed once per
// element and written nout times.
template <typename T>
struct OutList {
  T* p[kMaxSrc];
};

template <typename T, int OP>
__global__ __launch_bounds__(kMultiBlock) void k_fold_blocks_bcast(OutList<T> out, int nout, SrcList<T> src, int k,
                                                                   size_t n, size_t block_elems, int rings,
                                                                   RingSteps steps) {
  const size_t stride = (size_t)gridDim.x * kMultiBlock;
  for (size_t i = (size_t)blockIdx.x * kMultiBlock + threadIdx.x; i < n; i += stride) {
    const int b = (int)(i / block_elems);
    const size_t b0 = (size_t)b * block_elems;
    const size_t len = n - b0 < block_elems ? n - b0 : block_elems;
    const int g = (int)((i - b0) * (size_t)rings / len);
    const int step = steps.d[g];
    int q = b + step >= k ? b + step - k : b + step;
    T acc = src.p[q][i];
    for (int j = 1; j < k; ++j) {
      q = q + step >= k ? q + step - k : q + step;
      acc = apply<OP>(acc, src.p[q][i]);
    }
    for (int j = 0; j < nout; ++j) out.p[j][i] = acc;
  }
}

// Gather: copy up to 16 byte ranges (one per source rank, possibly peer
// memory over xGMI) in one launch; blockIdx.y picks the range.  16-byte
// vectors when a range is 16-B aligned at both ends, else 4-byte words.
struct CopyList {
  const char* src[kMaxSrc];
  char* dst[kMaxSrc];
  size_t bytes[kMaxSrc];
};

__global__ __launch_bounds__(kMultiBlock) void k_gather(CopyList cl) {
  const int r = blockIdx.y;
  const char* s = cl.src[r];
  char* d = cl.dst[r];
  const size_t nb = cl.bytes[r];
  const size_t stride = (size_t)gridDim.x * kMultiBlock;
  size_t t = (size_t)blockIdx.x * kMultiBlock + threadIdx.x;
  if ((((uintptr_t)s | (uintptr_t)d | nb) & 15) == 0) {
    const u32x4* vs = reinterpret_cast<const u32x4*>(s);
    u32x4* vd = reinterpret_cast<u32x4*>(d);
    for (size_t i = t; i < nb / 16; i += stride) st<true>(vd + i, ld<true>(vs + i));
  } else {
    const uint32_t* ws = reinterpret_cast<const uint32_t*>(s);
    uint32_t* wd = reinterpret_cast<uint32_t*>(d);
    for (size_t i = t; i < nb / 4; i += stride) wd[i] = ws[i];
  }
}

// ---- host side ---------------------------------------------------------------

thread_local char g_err[256] = "";

void set_err(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Tuning (process-wide).  The defaults are the measured best on MI355X (the figures are beside each knob).
int g_blocks_per_cu = 0;   // one-shot grid: 6403 vs 6200 GB/s capped at 8/CU (sweep r01)
int g_nontemporal = 1;
int g_fold_burst = 1;          // pgk_tune_fold
// Vector shape: 0x0 = by size (shape_for); else forced by pgk_tune_shape.
int g_block = 0;
int g_unroll = 0;

// Measured on MI355X (profiles/r01_sweep_kernel_shapes.csv, kernel-stamped,
// f64 sum, nt): 512x2 leads below 128 MiB per operand (64 MiB: 31.1 us vs
// 31.8 us for 1024x1), 1024x1 from 256 MiB up (256 MiB: 121.7 us vs 124.5 us
// for 512x2; 1 GiB: 495 us vs 515 us).  From 128 MiB to below 256 MiB 256x4
// leads 1024x1 by 1.3% on two boxes (128 MiB: 63.2 vs 64.1 us,
// profiles/r01_lab2.txt, profiles/r01_lab4_policy.txt).
void shape_for(size_t bytes_per_operand, int* block, int* unroll) {
  if (g_block) { *block = g_block; *unroll = g_unroll; return; }
  if (bytes_per_operand < (128u << 20)) { *block = 512; *unroll = 2; }
  else if (bytes_per_operand < (256u << 20)) { *block = 256; *unroll = 4; }
  else { *block = 1024; *unroll = 1; }
}

constexpr int kMaxDevices = 64;
int g_cu_count[kMaxDevices];  // 0 = not queried yet

int cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
  if (g_cu_count[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_cu_count[dev] = n;
  }
  return g_cu_count[dev];
}

// The AQL dispatch packet holds the grid size in WORK-ITEMS as 32 bits, so
// gridDim.x * blockDim.x must stay below 2^32; the kernels grid-stride over
// whatever a capped grid does not cover (> 64 GiB per operand on the vector
// path, > 4 Gi elements on the scalar one).
unsigned grid_cap(unsigned block) { return (unsigned)(0xFFFFFFFFull / block); }

unsigned grid_for(size_t blocks, unsigned block) {
  size_t g = blocks ? blocks : 1;
  if (g_blocks_per_cu > 0) {
    size_t cap = (size_t)cu_count() * (size_t)g_blocks_per_cu;
    if (g > cap) g = cap;
  }
  if (g > grid_cap(block)) g = grid_cap(block);
  return (unsigned)g;
}

struct Plan {
  bool vec;
  unsigned head, tail;
  size_t nvec;
  unsigned grid;
  int block, unroll;   // vector path shape
};

Plan plan_for(const void* out, const void* a, const void* b, size_t n, size_t es) {
  Plan p{};
  const size_t W = 16 / es;
  uintptr_t mo = (uintptr_t)out & 15, ma = (uintptr_t)a & 15, mb = (uintptr_t)b & 15;
  if (mo == ma && mo == mb && (mo % es) == 0) {
    size_t head = mo ? (16 - mo) / es : 0;
    if (head > n) head = n;
    size_t rest = n - head;
    p.vec = true;
    p.head = (unsigned)head;
    p.nvec = rest / W;
    p.tail = (unsigned)(rest % W);
    shape_for(n * es, &p.block, &p.unroll);
    size_t tile = (size_t)p.block * (size_t)p.unroll;
    size_t tiles = (p.nvec + tile - 1) / tile;
    p.grid = grid_for(tiles, (unsigned)p.block);
  } else {
    p.vec = false;
    p.grid = grid_for((n + kScalarBlock - 1) / kScalarBlock, kScalarBlock);
  }
  return p;
}

// Every launch goes through hipExtLaunchKernelGGL so that a caller can ask for
// the kernel's own begin/end timestamps (start/stop events; nullptr = none).
struct Timing {
  hipEvent_t start, stop;
};

template <typename T, int OP, bool NT, int B, int U>
void launch_shape(const Plan& p, T* out, const T* a, const T* b, hipStream_t s, Timing tm) {
  hipExtLaunchKernelGGL((k_reduce_vec<T, OP, NT, B, U>), dim3(p.grid), dim3(B), 0, s, tm.start, tm.stop, 0,
                        out, a, b, p.head, p.nvec, p.tail);
}

template <typename T, int OP, bool NT>
void launch_vec(const Plan& p, T* out, const T* a, const T* b, hipStream_t s, Timing tm) {
  switch (p.block * 16 + p.unroll) {
    case 256 * 16 + 2: launch_shape<T, OP, NT, 256, 2>(p, out, a, b, s, tm); break;
    case 256 * 16 + 8: launch_shape<T, OP, NT, 256, 8>(p, out, a, b, s, tm); break;
    case 512 * 16 + 2: launch_shape<T, OP, NT, 512, 2>(p, out, a, b, s, tm); break;
    case 1024 * 16 + 1: launch_shape<T, OP, NT, 1024, 1>(p, out, a, b, s, tm); break;
    default: launch_shape<T, OP, NT, 256, 4>(p, out, a, b, s, tm);
  }
}

// A single vector launch over more than 512 MiB per operand streams 1.3-4%
// slower than the same operands cut into launches of at most 512 MiB, on two
// boxes, at 1 and 2 GiB per operand, in every tile shape; the block count is
// not the cause (a 32 KiB tile halves it and is slower still;
// tools/lab/split_probe.py, profiles/r02_split_probe.txt).  So the size-chosen
// path cuts such a call into ceil(bytes / 512 MiB) equal pieces, each a whole
// number of 16 KiB tiles (every piece keeps the operands' 16-B phase), launched
// back to back on the caller's stream; the start stamp goes on the first, the
// stop stamp on the last.  A shape forced by pgk_tune_shape stays one launch,
// as the labs measure it.  The element-wise path (misaligned operands) is not
// cut: it is the rare fallback, and one launch keeps its grid-stride tested.
constexpr size_t kSplitBytes = 512ull << 20;

// elements per piece of an n-element vector call (n when it is not cut)
size_t piece_elems(size_t n, size_t es) {
  const size_t pieces = (n * es + kSplitBytes - 1) / kSplitBytes;
  if (g_block || pieces < 2) return n;
  const size_t align = (16u << 10) / es;
  return ((n + pieces - 1) / pieces + align - 1) / align * align;
}

template <typename T, int OP>
hipError_t launch_t(T* out, const T* a, const T* b, size_t n, hipStream_t s, Timing tm) {
  Plan p = plan_for(out, a, b, n, sizeof(T));
  if (p.vec) {
    const size_t piece = piece_elems(n, sizeof(T));
    if (piece >= n) {
      if (g_nontemporal) launch_vec<T, OP, true>(p, out, a, b, s, tm);
      else launch_vec<T, OP, false>(p, out, a, b, s, tm);
      return hipGetLastError();
    }
    for (size_t off = 0; off < n; off += piece) {
      const size_t len = n - off < piece ? n - off : piece;
      const Plan q = plan_for(out + off, a + off, b + off, len, sizeof(T));
      const Timing tq{off == 0 ? tm.start : nullptr, off + len == n ? tm.stop : nullptr};
      if (g_nontemporal) launch_vec<T, OP, true>(q, out + off, a + off, b + off, s, tq);
      else launch_vec<T, OP, false>(q, out + off, a + off, b + off, s, tq);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  hipExtLaunchKernelGGL((k_reduce_scalar<T, OP>), dim3(p.grid), dim3(kScalarBlock), 0, s, tm.start, tm.stop, 0,
                        out, a, b, n);
  return hipGetLastError();
}

// Two ranges of `bytes` that intersect without being the same range.
inline bool partly_overlap(const void* p, const void* q, size_t bytes) {
  const uintptr_t x = (uintptr_t)p, y = (uintptr_t)q;
  return x != y && x < y + bytes && y < x + bytes;
}

int launch(void* out, const void* a, const void* b, size_t n, int dt, int op, void* stream,
           Timing tm = Timing{nullptr, nullptr}) {
  if (dt != PGK_DT_INT32 && dt != PGK_DT_DOUBLE) { set_err("pgk: bad datatype %d", dt); return -1; }
  if (op != PGK_OP_SUM && op != PGK_OP_PROD) { set_err("pgk: bad operation %d", op); return -1; }
  if (n == 0) return 0;
  if (!out || !a || !b) { set_err("pgk: NULL buffer with n=%zu", n); return -1; }
  // The reference loop runs element by element, so operands that overlap
  // at different addresses see each other's results in index order there; a
  // parallel launch cannot reproduce that, and says so instead of guessing.
  const size_t bytes = n * (dt == PGK_DT_INT32 ? 4 : 8);
  if (partly_overlap(out, a, bytes) || partly_overlap(out, b, bytes)) {
    set_err("pgk: the output overlaps an operand at a different address (n=%zu)", n);
    return -1;
  }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (dt == PGK_DT_INT32) {
    uint32_t* o = (uint32_t*)out;
    const uint32_t* x = (const uint32_t*)a;
    const uint32_t* y = (const uint32_t*)b;
    e = op == PGK_OP_SUM ? launch_t<uint32_t, PGK_OP_SUM>(o, x, y, n, s, tm)
                         : launch_t<uint32_t, PGK_OP_PROD>(o, x, y, n, s, tm);
  } else {
    double* o = (double*)out;
    const double* x = (const double*)a;
    const double* y = (const double*)b;
    e = op == PGK_OP_SUM ? launch_t<double, PGK_OP_SUM>(o, x, y, n, s, tm)
                         : launch_t<double, PGK_OP_PROD>(o, x, y, n, s, tm);
  }
  if (e != hipSuccess) { set_err("pgk: launch failed: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

template <typename T, int OP, bool NT, int B, int U>
void launch_ranges_shape(unsigned grid, const RangeList<T>& rl, hipStream_t s, Timing tm) {
  hipExtLaunchKernelGGL((k_reduce_ranges<T, OP, NT, B, U>), dim3(grid), dim3(B), 0, s, tm.start, tm.stop, 0, rl);
}

template <typename T, int OP, bool NT>
void launch_ranges_nt(int block, int unroll, unsigned grid, const RangeList<T>& rl, hipStream_t s, Timing tm) {
  switch (block * 16 + unroll) {
    case 256 * 16 + 2: launch_ranges_shape<T, OP, NT, 256, 2>(grid, rl, s, tm); break;
    case 256 * 16 + 8: launch_ranges_shape<T, OP, NT, 256, 8>(grid, rl, s, tm); break;
    case 512 * 16 + 2: launch_ranges_shape<T, OP, NT, 512, 2>(grid, rl, s, tm); break;
    case 1024 * 16 + 1: launch_ranges_shape<T, OP, NT, 1024, 1>(grid, rl, s, tm); break;
    default: launch_ranges_shape<T, OP, NT, 256, 4>(grid, rl, s, tm);
  }
}

// k ranges, each 16-B congruent (plan_for(...).vec), in one launch; the
// shape is the one a single launch of all the ranges' bytes would use (a launch
// of R ranges streams like one launch of their sum: 2 x 64 MiB runs at 81.6%
// of the HBM peak with the 128 MiB shape, 80.7% with the 64 MiB one, and
// 2 x 128 MiB at 82.2% against 80.6%, kernel-stamped,
// tools/lab/ranges_shape_probe.py), and each range gets the blocks that shape
// gives it.  Returns hipErrorInvalidValue (nothing launched) when the ranges do
// not fit one grid.
template <typename T, int OP>
hipError_t launch_ranges_t(T* const* outs, const T* const* as, const T* const* bs, const size_t* ns, int k,
                           hipStream_t s, Timing tm) {
  RangeList<T> rl{};
  size_t sum = 0;
  for (int j = 0; j < k; ++j) sum += ns[j];
  int block = 0, unroll = 0;
  shape_for(sum * sizeof(T), &block, &unroll);
  const size_t tile = (size_t)block * (size_t)unroll, W = 16 / sizeof(T);
  size_t total = 0;
  rl.k = k;
  for (int j = 0; j < k; ++j) {
    uintptr_t m = (uintptr_t)outs[j] & 15;
    size_t head = m ? (16 - m) / sizeof(T) : 0;
    if (head > ns[j]) head = ns[j];
    rl.out[j] = outs[j];
    rl.a[j] = as[j];
    rl.b[j] = bs[j];
    rl.head[j] = (unsigned)head;
    rl.nvec[j] = (ns[j] - head) / W;
    rl.tail[j] = (unsigned)((ns[j] - head) % W);
    size_t blocks = (rl.nvec[j] + tile - 1) / tile;
    rl.first[j] = (unsigned)total;
    total += blocks ? blocks : 1;
    if (total > grid_cap((unsigned)block)) return hipErrorInvalidValue;
  }
  rl.first[k] = (unsigned)total;
  if (g_nontemporal) launch_ranges_nt<T, OP, true>(block, unroll, (unsigned)total, rl, s, tm);
  else launch_ranges_nt<T, OP, false>(block, unroll, (unsigned)total, rl, s, tm);
  return hipGetLastError();
}

template <typename T, int OP, int NS>
void launch_burst_u(int u, unsigned grid, T* out, const SrcList<T>& sl, unsigned head, size_t v0, size_t v1,
                    unsigned eh, unsigned et, size_t tail_e, hipStream_t s, Timing tm) {
#define PGK_BURST_CASE(U) \
  hipExtLaunchKernelGGL((k_reduce_multi_burst<T, OP, NS, U>), dim3(grid), dim3(kBurstBlock), 0, s, tm.start, tm.stop, \
                        0, out, sl, head, v0, v1, eh, et, tail_e)
  if (u <= 16) PGK_BURST_CASE(16);
  else PGK_BURST_CASE(32);
#undef PGK_BURST_CASE
}

// The next burst launch of a call with `left` vectors per source still to fold:
// how many vectors it takes and with how many tiles per wave; 0 = none (what
// is left goes one tile per wave).
inline size_t burst_next(size_t left, bool shared_gpu, int* tiles) {
  if (!shared_gpu && left >= kBurstVecs32) { *tiles = 32; return kBurstVecs32; }
  if (!shared_gpu && left >= kBurstVecs16) { *tiles = 16; return left; }          // 512 .. 1023 workgroups
  if (left >= kBurstVecs16) { *tiles = 16; return kBurstVecs16; }
  return 0;
}

// The burst fold of a whole call (5 <= nsrc <= 8, nvec * 16 >= kBurstMinBytes),
// as whole launches of the shapes above; what is left (under 32 MiB per source)
// is returned to the caller (`done` = vectors covered), which folds it one tile
// per wave.  The first launch also folds the call's unaligned edge elements.
template <typename T, int OP>
hipError_t launch_burst(T* out, const SrcList<T>& sl, int nsrc, unsigned head, size_t nvec, unsigned tail,
                        bool shared_gpu, hipStream_t s, Timing tm, size_t* done) {
  const size_t tail_e = head + nvec * (16 / sizeof(T));
  size_t v0 = 0;
  while (v0 < nvec) {
    int u;
    const size_t take = burst_next(nvec - v0, shared_gpu, &u);
    if (!take) break;
    const size_t v1 = v0 + take;
    const unsigned grid = (unsigned)((take + (size_t)kBurstBlock * u - 1) / ((size_t)kBurstBlock * u));
    const Timing tq{v0 == 0 ? tm.start : nullptr, v1 == nvec ? tm.stop : nullptr};
    const unsigned eh = v0 == 0 ? head : 0, et = v0 == 0 ? tail : 0;
    switch (nsrc) {
      case 5: launch_burst_u<T, OP, 5>(u, grid, out, sl, head, v0, v1, eh, et, tail_e, s, tq); break;
      case 6: launch_burst_u<T, OP, 6>(u, grid, out, sl, head, v0, v1, eh, et, tail_e, s, tq); break;
      case 7: launch_burst_u<T, OP, 7>(u, grid, out, sl, head, v0, v1, eh, et, tail_e, s, tq); break;
      default: launch_burst_u<T, OP, 8>(u, grid, out, sl, head, v0, v1, eh, et, tail_e, s, tq);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    v0 = v1;
  }
  *done = v0;
  return hipSuccess;
}

template <typename T, int OP>
hipError_t launch_multi_t(T* out, const T* const* srcs, int nsrc, size_t n, hipStream_t s, Timing tm,
                          unsigned flags = 0) {
  SrcList<T> sl{};
  uintptr_t m = (uintptr_t)out & 15;
  bool congruent = (m % sizeof(T)) == 0;
  for (int j = 0; j < nsrc; ++j) {
    sl.p[j] = srcs[j];
    if (((uintptr_t)srcs[j] & 15) != m) congruent = false;
  }
  const size_t W = 16 / sizeof(T);
  if (congruent) {
    size_t head = m ? (16 - m) / sizeof(T) : 0;
    if (head > n) head = n;
    size_t nvec = (n - head) / W, tail = (n - head) % W;
    if (!(flags & PGK_FOLD_REMOTE_SOURCES) && g_fold_burst && nsrc >= 5 && nsrc <= 8 &&
        nvec * 16 >= kBurstMinBytes) {
      size_t done = 0;
      hipError_t e = launch_burst<T, OP>(out, sl, nsrc, (unsigned)head, nvec, (unsigned)tail,
                                         (flags & PGK_FOLD_SHARED_GPU) != 0, s, tm, &done);
      if (e != hipSuccess || done == nvec) return e;
      // the rest (under 32 MiB per source): one tile per wave, behind the bursts on the same stream
      out += head + done * W;
      for (int j = 0; j < nsrc; ++j) sl.p[j] += head + done * W;
      nvec -= done;
      head = tail = 0;
      tm.start = nullptr;
    }
    size_t g = (nvec + kMultiVecBlock - 1) / kMultiVecBlock;
    if (g == 0) g = 1;
    if (g > grid_cap(kMultiVecBlock)) g = grid_cap(kMultiVecBlock);
    dim3 grid((unsigned)g), block(kMultiVecBlock);
    switch (nsrc) {
#define PGK_MULTI_CASE(K) \
      case K: hipExtLaunchKernelGGL((k_reduce_multi_vec<T, OP, K>), grid, block, 0, s, tm.start, tm.stop, 0, out, sl, \
                                    nsrc, (unsigned)head, nvec, (unsigned)tail); break;
      PGK_MULTI_CASE(1) PGK_MULTI_CASE(2) PGK_MULTI_CASE(3) PGK_MULTI_CASE(4)
      PGK_MULTI_CASE(5) PGK_MULTI_CASE(6) PGK_MULTI_CASE(7) PGK_MULTI_CASE(8)
#undef PGK_MULTI_CASE
      default:
        hipExtLaunchKernelGGL((k_reduce_multi_vec<T, OP, 0>), grid, block, 0, s, tm.start, tm.stop, 0, out, sl, nsrc,
                              (unsigned)head, nvec, (unsigned)tail);
    }
  } else {
    size_t g = (n + kMultiBlock - 1) / kMultiBlock;
    if (g > 65536) g = 65536;
    hipExtLaunchKernelGGL((k_reduce_multi_scalar<T, OP>), dim3((unsigned)g), dim3(kMultiBlock), 0, s, tm.start,
                          tm.stop, 0, out, sl, nsrc, n);
  }
  return hipGetLastError();
}

}  // namespace

// Exchange area of pgk_all_reduce_staged: one slot per rank.  Every GPU this
// library runs on holds its own copy of the array, at its own address, until
// the process ends.  In host code the name is only a handle for
// hipGetSymbolAddress; launches and copies use the address that call returns.
static __device__ __align__(256) unsigned char scratch[PGK_STAGED_MAX_BYTES];

namespace {

unsigned char* g_scratch_ptr[kMaxDevices];   // per device, resolved once with that device current

// Device address of `scratch` on the current device (nullptr + message on failure).
unsigned char* scratch_on_current_device() {
  int dev = -1;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess || dev < 0 || dev >= kMaxDevices) {
    set_err("pgk: staged all-reduce: no usable current device (%s)", hipGetErrorString(e));
    return nullptr;
  }
  if (!g_scratch_ptr[dev]) {
    void* p = nullptr;
    e = hipGetSymbolAddress(&p, HIP_SYMBOL(scratch));
    if (e != hipSuccess || !p) {
      set_err("pgk: hipGetSymbolAddress(scratch) on device %d: %s", dev, hipGetErrorString(e));
      return nullptr;
    }
    g_scratch_ptr[dev] = (unsigned char*)p;
  }
  return g_scratch_ptr[dev];
}

template <typename T, int OP>
void launch_fold_bcast(void* const* outs, int nout, const unsigned char* area, size_t slot, int k, size_t n,
                       size_t block_elems, int rings, const RingSteps& rs, hipStream_t s) {
  OutList<T> ol{};
  SrcList<T> sl{};
  for (int j = 0; j < nout; ++j) ol.p[j] = (T*)outs[j];
  for (int j = 0; j < k; ++j) sl.p[j] = (const T*)(area + (size_t)j * slot);
  size_t g = (n + kMultiBlock - 1) / kMultiBlock;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL((k_fold_blocks_bcast<T, OP>), dim3((unsigned)g), dim3(kMultiBlock), 0, s, ol, nout, sl, k, n,
                     block_elems, rings, rs);
}

}  // namespace

extern "C" {

static int reduce_multi(void* out, const void* const* srcs, int nsrc, size_t n, int dt, int op, void* stream,
                        void* start_event, void* stop_event, unsigned flags) {
  if (flags & ~(unsigned)(PGK_FOLD_REMOTE_SOURCES | PGK_FOLD_SHARED_GPU)) {
    set_err("pgk: unknown fold flags 0x%x", flags);
    return -1;
  }
  if (dt != PGK_DT_INT32 && dt != PGK_DT_DOUBLE) { set_err("pgk: bad datatype %d", dt); return -1; }
  if (op != PGK_OP_SUM && op != PGK_OP_PROD) { set_err("pgk: bad operation %d", op); return -1; }
  if (nsrc < 1 || nsrc > kMaxSrc) { set_err("pgk: nsrc %d outside 1..%d", nsrc, kMaxSrc); return -1; }
  if (n == 0) return 0;
  if (!out || !srcs) { set_err("pgk: NULL buffer with n=%zu", n); return -1; }
  for (int j = 0; j < nsrc; ++j)
    if (!srcs[j]) { set_err("pgk: NULL source %d", j); return -1; }
  hipStream_t s = (hipStream_t)stream;
  Timing tm{(hipEvent_t)start_event, (hipEvent_t)stop_event};
  hipError_t e;
  if (dt == PGK_DT_INT32) {
    const uint32_t* const* x = (const uint32_t* const*)srcs;
    e = op == PGK_OP_SUM ? launch_multi_t<uint32_t, PGK_OP_SUM>((uint32_t*)out, x, nsrc, n, s, tm, flags)
                         : launch_multi_t<uint32_t, PGK_OP_PROD>((uint32_t*)out, x, nsrc, n, s, tm, flags);
  } else {
    const double* const* x = (const double* const*)srcs;
    e = op == PGK_OP_SUM ? launch_multi_t<double, PGK_OP_SUM>((double*)out, x, nsrc, n, s, tm, flags)
                         : launch_multi_t<double, PGK_OP_PROD>((double*)out, x, nsrc, n, s, tm, flags);
  }
  if (e != hipSuccess) { set_err("pgk: launch failed: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_reduce_multi_timed(void* out, const void* const* srcs, int nsrc, size_t n, int dt, int op, void* stream,
                           void* start_event, void* stop_event) {
  return reduce_multi(out, srcs, nsrc, n, dt, op, stream, start_event, stop_event, 0);
}

int pgk_fold_geometry(size_t n, int dt, int nsrc, unsigned flags, size_t* launch_bytes, int* launch_tiles,
                      int max_launches, size_t* plain_bytes) {
  if (dt != PGK_DT_INT32 && dt != PGK_DT_DOUBLE) { set_err("pgk: bad datatype %d", dt); return -1; }
  if (nsrc < 1 || nsrc > kMaxSrc || max_launches < 0 || (max_launches && (!launch_bytes || !launch_tiles))) {
    set_err("pgk: bad fold geometry arguments");
    return -1;
  }
  const size_t es = dt == PGK_DT_INT32 ? 4 : 8;
  size_t left = n * es / 16;                      // 16-byte-aligned operands: no edge elements
  int k = 0;
  if (!(flags & PGK_FOLD_REMOTE_SOURCES) && g_fold_burst && nsrc >= 5 && nsrc <= 8 && left * 16 >= kBurstMinBytes) {
    for (;;) {
      int tiles = 0;
      const size_t take = burst_next(left, (flags & PGK_FOLD_SHARED_GPU) != 0, &tiles);
      if (!take) break;
      if (k < max_launches) { launch_bytes[k] = take * 16; launch_tiles[k] = tiles; }
      ++k;
      left -= take;
    }
  }
  if (plain_bytes) *plain_bytes = left * 16 + n * es % 16;
  return k;
}

int pgk_fold_timed(void* out, const void* const* srcs, int nsrc, size_t n, int dt, int op, unsigned flags,
                   void* stream, void* start_event, void* stop_event) {
  return reduce_multi(out, srcs, nsrc, n, dt, op, stream, start_event, stop_event, flags);
}


int pgk_reduce_multi(void* out, const void* const* srcs, int nsrc, size_t n, int dt, int op, void* stream) {
  return pgk_reduce_multi_timed(out, srcs, nsrc, n, dt, op, stream, nullptr, nullptr);
}

// Step of ring `part` among `rings` over `world` ranks: +1, -1, then +3, -3,
// ... kept when coprime with world and new mod world, repeating when they run
// out.  The same rule as pg_ring_offset (pg_plan.c); the kernel library keeps
// its own copy so that include/pgk.h stands alone.
static int ring_step(int world, int rings, int part) {
  int offs[kMaxRings] = {1, -1}, m = 2;
  auto mod = [world](int x) { return ((x % world) + world) % world; };
  auto gcd = [](int a, int b) { while (b) { int t = a % b; a = b; b = t; } return a; };
  for (int c = 3; m < kMaxRings && c < 2 * world; c += 2)
    for (int sgn = 1; sgn >= -1 && m < kMaxRings; sgn -= 2) {
      int d = sgn * c, rd = mod(d);
      if (rd == 0 || gcd(rd, world) != 1) continue;
      bool dup = false;
      for (int i = 0; i < m; ++i) dup |= mod(offs[i]) == rd;
      if (!dup) offs[m++] = d;
    }
  (void)rings;
  return offs[part % m];
}

int pgk_fold_blocks(void* out, const void* const* srcs, int nsrc, size_t n, size_t block_elems, int rings,
                    int dt, int op, void* stream) {
  if (dt != PGK_DT_INT32 && dt != PGK_DT_DOUBLE) { set_err("pgk: bad datatype %d", dt); return -1; }
  if (op != PGK_OP_SUM && op != PGK_OP_PROD) { set_err("pgk: bad operation %d", op); return -1; }
  if (nsrc < 1 || nsrc > kMaxSrc) { set_err("pgk: nsrc %d outside 1..%d", nsrc, kMaxSrc); return -1; }
  if (rings < 1 || rings > kMaxRings) { set_err("pgk: rings %d, expected 1 .. %d", rings, kMaxRings); return -1; }
  if (n == 0) return 0;
  if (!out || !srcs || block_elems == 0 || (n + block_elems - 1) / block_elems > (size_t)nsrc) {
    set_err("pgk: bad fold_blocks arguments");
    return -1;
  }
  size_t g = (n + kMultiBlock - 1) / kMultiBlock;
  if (g > 65536) g = 65536;
  hipStream_t s = (hipStream_t)stream;
  RingSteps rs{};
  for (int p = 0; p < rings; ++p) rs.d[p] = ((ring_step(nsrc, rings, p) % nsrc) + nsrc) % nsrc;
  if (dt == PGK_DT_INT32) {
    SrcList<uint32_t> sl{};
    for (int j = 0; j < nsrc; ++j) sl.p[j] = (const uint32_t*)srcs[j];
    if (op == PGK_OP_SUM)
      hipLaunchKernelGGL((k_fold_blocks<uint32_t, PGK_OP_SUM>), dim3((unsigned)g), dim3(kMultiBlock), 0, s,
                         (uint32_t*)out, sl, nsrc, n, block_elems, rings, rs);
    else
      hipLaunchKernelGGL((k_fold_blocks<uint32_t, PGK_OP_PROD>), dim3((unsigned)g), dim3(kMultiBlock), 0, s,
                         (uint32_t*)out, sl, nsrc, n, block_elems, rings, rs);
  } else {
    SrcList<double> sl{};
    for (int j = 0; j < nsrc; ++j) sl.p[j] = (const double*)srcs[j];
    if (op == PGK_OP_SUM)
      hipLaunchKernelGGL((k_fold_blocks<double, PGK_OP_SUM>), dim3((unsigned)g), dim3(kMultiBlock), 0, s,
                         (double*)out, sl, nsrc, n, block_elems, rings, rs);
    else
      hipLaunchKernelGGL((k_fold_blocks<double, PGK_OP_PROD>), dim3((unsigned)g), dim3(kMultiBlock), 0, s,
                         (double*)out, sl, nsrc, n, block_elems, rings, rs);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err("pgk: launch failed: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_gather(void* const* dsts, const void* const* srcs, const size_t* bytes, int k, void* stream) {
  if (k < 0 || k > kMaxSrc || (k && (!dsts || !srcs || !bytes))) { set_err("pgk: bad gather arguments"); return -1; }
  CopyList cl{};
  size_t most = 0;
  int m = 0;
  for (int j = 0; j < k; ++j) {
    if (!bytes[j]) continue;
    if ((bytes[j] & 3) || (((uintptr_t)dsts[j] | (uintptr_t)srcs[j]) & 3)) {
      set_err("pgk: gather ranges must be 4-byte aligned");
      return -1;
    }
    cl.src[m] = (const char*)srcs[j];
    cl.dst[m] = (char*)dsts[j];
    cl.bytes[m] = bytes[j];
    if (bytes[j] > most) most = bytes[j];
    ++m;
  }
  if (!m) return 0;
  size_t g = (most / 16 + kMultiBlock - 1) / kMultiBlock;
  if (g == 0) g = 1;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_gather, dim3((unsigned)g, (unsigned)m), dim3(kMultiBlock), 0, (hipStream_t)stream, cl);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err("pgk: launch failed: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_all_reduce_staged(void* const* sendbufs, void* const* recvbufs, int world, size_t count, int rings,
                          int dt, int op, void* stream) {
  if (dt != PGK_DT_INT32 && dt != PGK_DT_DOUBLE) { set_err("pgk: bad datatype %d", dt); return -1; }
  if (op != PGK_OP_SUM && op != PGK_OP_PROD) { set_err("pgk: bad operation %d", op); return -1; }
  if (world < 1 || world > kMaxSrc) { set_err("pgk: world %d outside 1..%d", world, kMaxSrc); return -1; }
  if (rings < 1 || rings > kMaxRings) { set_err("pgk: rings %d, expected 1 .. %d", rings, kMaxRings); return -1; }
  const size_t es = dt == PGK_DT_INT32 ? 4 : 8;
  if (count > PGK_STAGED_MAX_BYTES / es) {
    set_err("pgk: staged all-reduce: %zu elements per rank exceed the %zu-byte exchange area", count,
            (size_t)PGK_STAGED_MAX_BYTES);
    return -1;
  }
  const size_t slot = (count * es + 255) & ~(size_t)255;
  if (slot * (size_t)world > PGK_STAGED_MAX_BYTES) {
    set_err("pgk: staged all-reduce: %d ranks x %zu bytes exceed the %zu-byte exchange area (at most %zu bytes "
            "per rank at this world size)", world, count * es, (size_t)PGK_STAGED_MAX_BYTES,
            (size_t)PGK_STAGED_MAX_BYTES / (size_t)world / 256 * 256);
    return -1;
  }
  unsigned char* area = scratch_on_current_device();   // also the whole of a count == 0 set-up call
  if (!area) return -1;
  if (count == 0) return 0;
  if (!sendbufs || !recvbufs) { set_err("pgk: NULL buffer list with count=%zu", count); return -1; }
  for (int q = 0; q < world; ++q)
    if (!sendbufs[q] || !recvbufs[q] || (((uintptr_t)sendbufs[q] | (uintptr_t)recvbufs[q]) & (es - 1))) {
      set_err("pgk: staged all-reduce: buffer of rank %d is NULL or not element-aligned", q);
      return -1;
    }
  hipStream_t s = (hipStream_t)stream;
  // the exchange: every rank's input into its slot, one launch
  CopyList cl{};
  for (int q = 0; q < world; ++q) {
    cl.src[q] = (const char*)sendbufs[q];
    cl.dst[q] = (char*)(area + (size_t)q * slot);
    cl.bytes[q] = count * es;
  }
  size_t g = (count * es / 16 + kMultiBlock - 1) / kMultiBlock;
  if (g == 0) g = 1;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_gather, dim3((unsigned)g, (unsigned)world), dim3(kMultiBlock), 0, s, cl);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_err("pgk: launch failed: %s", hipGetErrorString(e)); return -1; }
  // the fold, each block in its ring order, stored to every rank's output
  const size_t blk = (count + (size_t)world - 1) / (size_t)world;
  RingSteps rs{};
  for (int p = 0; p < rings; ++p) rs.d[p] = ((ring_step(world, rings, p) % world) + world) % world;
  if (dt == PGK_DT_INT32) {
    if (op == PGK_OP_SUM) launch_fold_bcast<uint32_t, PGK_OP_SUM>(recvbufs, world, area, slot, world, count, blk, rings, rs, s);
    else launch_fold_bcast<uint32_t, PGK_OP_PROD>(recvbufs, world, area, slot, world, count, blk, rings, rs, s);
  } else {
    if (op == PGK_OP_SUM) launch_fold_bcast<double, PGK_OP_SUM>(recvbufs, world, area, slot, world, count, blk, rings, rs, s);
    else launch_fold_bcast<double, PGK_OP_PROD>(recvbufs, world, area, slot, world, count, blk, rings, rs, s);
  }
  e = hipGetLastError();
  if (e != hipSuccess) { set_err("pgk: launch failed: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_reduce_ranges(void* const* outs, const void* const* as, const void* const* bs, const size_t* ns, int k,
                      int dt, int op, void* stream, void* start_event, void* stop_event) {
  if (dt != PGK_DT_INT32 && dt != PGK_DT_DOUBLE) { set_err("pgk: bad datatype %d", dt); return -1; }
  if (op != PGK_OP_SUM && op != PGK_OP_PROD) { set_err("pgk: bad operation %d", op); return -1; }
  if (k < 0 || k > kMaxRanges || (k && (!outs || !as || !bs || !ns))) {
    set_err("pgk: reduce_ranges takes 0 .. %d ranges", kMaxRanges);
    return -1;
  }
  const size_t es = dt == PGK_DT_INT32 ? 4 : 8;
  void* o[kMaxRanges];
  const void* a[kMaxRanges];
  const void* b[kMaxRanges];
  size_t n[kMaxRanges];
  int m = 0;
  bool vec = true;
  for (int j = 0; j < k; ++j) {
    if (!ns[j]) continue;
    if (!outs[j] || !as[j] || !bs[j]) { set_err("pgk: NULL buffer in range %d", j); return -1; }
    o[m] = outs[j];
    a[m] = as[j];
    b[m] = bs[j];
    n[m] = ns[j];
    vec = vec && plan_for(o[m], a[m], b[m], n[m], es).vec;
    ++m;
  }
  if (!m) return 0;
  Timing tm{(hipEvent_t)start_event, (hipEvent_t)stop_event};
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipErrorInvalidValue;
  if (vec && m > 1) {
    if (dt == PGK_DT_INT32) {
      e = op == PGK_OP_SUM
              ? launch_ranges_t<uint32_t, PGK_OP_SUM>((uint32_t* const*)o, (const uint32_t* const*)a,
                                                     (const uint32_t* const*)b, n, m, s, tm)
              : launch_ranges_t<uint32_t, PGK_OP_PROD>((uint32_t* const*)o, (const uint32_t* const*)a,
                                                      (const uint32_t* const*)b, n, m, s, tm);
    } else {
      e = op == PGK_OP_SUM
              ? launch_ranges_t<double, PGK_OP_SUM>((double* const*)o, (const double* const*)a,
                                                   (const double* const*)b, n, m, s, tm)
              : launch_ranges_t<double, PGK_OP_PROD>((double* const*)o, (const double* const*)a,
                                                    (const double* const*)b, n, m, s, tm);
    }
    if (e == hipSuccess) return 0;
    if (e != hipErrorInvalidValue) { set_err("pgk: launch failed: %s", hipGetErrorString(e)); return -1; }
  }
  // one launch per range (a misaligned range, a single range, or ranges too
  // large for one grid); the start stamp goes on the first, the stop on the last
  for (int j = 0; j < m; ++j) {
    Timing tj{j == 0 ? tm.start : nullptr, j == m - 1 ? tm.stop : nullptr};
    if (launch(o[j], a[j], b[j], n[j], dt, op, stream, tj)) return -1;
  }
  return 0;
}

int pgk_reduce(void* dst, const void* src, size_t n, int dt, int op, void* stream) {
  return launch(dst, dst, src, n, dt, op, stream);
}

int pgk_reduce_out(void* out, const void* a, const void* b, size_t n, int dt, int op,
                   void* stream) {
  return launch(out, a, b, n, dt, op, stream);
}

int pgk_device_count(int* count) {
  if (!count) { set_err("pgk: NULL count"); return -1; }
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) { *count = 0; set_err("pgk: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_set_device(int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { set_err("pgk: hipSetDevice(%d): %s", device, hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_synchronize(void) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) { set_err("pgk: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_tune(int blocks_per_cu, int nontemporal) {
  if (blocks_per_cu >= 0) g_blocks_per_cu = blocks_per_cu;
  if (nontemporal >= 0) g_nontemporal = nontemporal ? 1 : 0;
  return 0;
}

int pgk_tune_fold(int burst) {
  if (burst >= 0) g_fold_burst = burst ? 1 : 0;
  return 0;
}

int pgk_tune_shape(int block, int unroll) {
  const int ok = (block == 0 && unroll == 0) ||
                 (block == 256 && (unroll == 2 || unroll == 4 || unroll == 8)) ||
                 (block == 512 && unroll == 2) || (block == 1024 && unroll == 1);
  if (!ok) { set_err("pgk: shape %dx%d not instantiated", block, unroll); return -1; }
  g_block = block;
  g_unroll = unroll;
  return 0;
}

int pgk_reduce_timed(void* dst, const void* src, size_t n, int dt, int op, void* stream,
                     void* start_event, void* stop_event) {
  return launch(dst, dst, src, n, dt, op, stream,
                Timing{(hipEvent_t)start_event, (hipEvent_t)stop_event});
}

int pgk_event_create(void** ev) {
  if (!ev) { set_err("pgk: NULL event slot"); return -1; }
  hipError_t e = hipEventCreate((hipEvent_t*)ev);
  if (e != hipSuccess) { set_err("pgk: hipEventCreate: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_event_destroy(void* ev) {
  return ev && hipEventDestroy((hipEvent_t)ev) != hipSuccess ? -1 : 0;
}

int pgk_event_elapsed_ms(void* start, void* stop, float* ms) {
  hipError_t e = hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop);
  if (e != hipSuccess) { set_err("pgk: hipEventElapsedTime: %s", hipGetErrorString(e)); return -1; }
  return 0;
}

int pgk_launch_geometry(size_t n, int dt, unsigned* grid, unsigned* block) {
  if (dt != PGK_DT_INT32 && dt != PGK_DT_DOUBLE) { set_err("pgk: bad datatype %d", dt); return -1; }
  const size_t es = dt == PGK_DT_INT32 ? 4 : 8;
  Plan p = plan_for(nullptr, nullptr, nullptr, piece_elems(n, es), es);   // the first launch of the call
  if (grid) *grid = p.grid;
  if (block) *block = p.vec ? (unsigned)p.block : (unsigned)kScalarBlock;
  return 0;
}

const char* pgk_last_error(void) { return g_err; }

#define PGK_STR2(x) #x
#define PGK_STR(x) PGK_STR2(x)
const char* pgk_version(void) {
  return "pgk gfx950 (HIP " PGK_STR(HIP_VERSION_MAJOR) "." PGK_STR(HIP_VERSION_MINOR) ")";
}

}  // extern "C"
