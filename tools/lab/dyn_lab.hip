// EXPERIMENTS ONLY (tools/lab/run_edge_lab.py --lab dyn): a resident grid
// that takes its tiles from an agent-scope ticket counter.  The timeline lab
// (r02_timeline_lab.txt) shows the 8 XCDs finishing a launch 1.8 us (64 MiB)
// to 6 us (256 MiB) apart: the dispatcher deals blocks to the XCDs in turn, so
// each XCD runs 1/8 of the tiles whatever its rate, and the slowest sets the
// launch's end.  Tickets let a faster XCD take more tiles.
//   dyn    : grid = CUs x blocks/CU, each block grabs G tiles per ticket and
//            prefetches its next ticket while it streams the current tiles
//   static : the same resident grid, grid-strided (the control)
// The counter pair (tickets, finished blocks) is reset by the last block, so
// consecutive launches on one stream reuse it.  Same API as edge_lab.hip.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned ticket(unsigned* c) {
  return __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int B, int U>
__device__ __forceinline__ void tile(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t t, size_t nvec) {
  const size_t i = t * B * U + threadIdx.x;
  if (i + (size_t)(U - 1) * B < nvec) {
    f64x2 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = __builtin_nontemporal_load(d + i + u * B);
      y[u] = __builtin_nontemporal_load(s + i + u * B);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + y[u], d + i + u * B);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * B < nvec)
        __builtin_nontemporal_store(__builtin_nontemporal_load(d + i + u * B) + __builtin_nontemporal_load(s + i + u * B),
                                    d + i + u * B);
  }
}

template <int B, int U, int G>
__global__ __launch_bounds__(B) void k_dyn(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec,
                                           unsigned* ctr, unsigned ngrabs, size_t ntiles) {
  __shared__ unsigned slot[2];
  if (threadIdx.x == 0) slot[0] = ticket(ctr);
  __syncthreads();
  unsigned g = slot[0];
  int p = 0;
  while (g < ngrabs) {
    unsigned nxt = 0;
    if (threadIdx.x == 0) nxt = ticket(ctr);          // in flight while this grab streams
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const size_t t = (size_t)g * G + k;
      if (t < ntiles) tile<B, U>(d, s, t, nvec);
    }
    if (threadIdx.x == 0) slot[p ^ 1] = nxt;
    __syncthreads();
    p ^= 1;
    g = slot[p];
  }
  if (threadIdx.x == 0 && ticket(ctr + 1) == gridDim.x - 1) {   // the last block out resets the pair
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


// Per-XCD queues (second attempt): the one-shot grid keeps one tile
// per block, but blocks from `prefix` on take their tile from the queue of
// the XCD they run on (HW_REG_XCC_ID), and from the other XCDs' queues once
// their own is empty.  The grid has `slack` more blocks than tiles, so a
// faster XCD's extra blocks find work the slower XCDs have not reached yet;
// a block that finds every queue empty exits.  Every tile is taken exactly
// once: tiles [0, prefix) by blocks [0, prefix), the rest by queue grabs,
// and no block exits while a queue still holds a tile.
__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7;
}

constexpr int kHeadStride = 32;   // one 128-B line per head; heads 0..7, finished-block count at 8

template <int B, int U>
__global__ __launch_bounds__(B) void k_xq(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec,
                                          unsigned* ctr, size_t ntiles, unsigned prefix, unsigned qlen) {
  if (blockIdx.x < prefix) {
    tile<B, U>(d, s, blockIdx.x, nvec);
  } else {
    __shared__ long long got;
    if (threadIdx.x == 0) {
      const unsigned x = xcc_id();
      long long t = -1;
      for (int k = 0; k < 8 && t < 0; ++k) {
        const unsigned q = (x + k) & 7;
        const size_t q0 = prefix + (size_t)q * qlen;
        if (q0 >= ntiles) continue;
        const size_t len = ntiles - q0 < qlen ? ntiles - q0 : qlen;
        const unsigned v = ticket(ctr + q * kHeadStride);
        if (v < len) t = (long long)(q0 + v);
      }
      got = t;
    }
    __syncthreads();
    if (got >= 0) tile<B, U>(d, s, (size_t)got, nvec);
  }
  if (threadIdx.x == 0 && ticket(ctr + 8 * kHeadStride) == gridDim.x - 1) {
    for (int q = 0; q <= 8; ++q) __hip_atomic_store(ctr + q * kHeadStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int B, int U>
__global__ __launch_bounds__(B) void k_static(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec,
                                              size_t ntiles) {
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) tile<B, U>(d, s, t, nvec);
}

struct V {
  const char* name;
  int block, unroll, grab, per_cu;   // grab 0 = static; grab -1 = per-XCD queues (per_cu = slack in %)
  int prefix;                        // per-XCD queues: blocks [0, prefix) take tile blockIdx (no ticket)
};
static const V kV[] = {
    {"reduce dyn 512x2 g1 4/CU", 512, 2, 1, 4},   {"reduce dyn 512x2 g2 4/CU", 512, 2, 2, 4},
    {"reduce dyn 512x2 g1 2/CU", 512, 2, 1, 2},   {"reduce dyn 256x2 g1 8/CU", 256, 2, 1, 8},
    {"reduce dyn 1024x1 g1 2/CU", 1024, 1, 1, 2}, {"reduce static 512x2 4/CU", 512, 2, 0, 4},
    {"reduce static 1024x1 2/CU", 1024, 1, 0, 2},
    {"reduce xq 512x2 slack0", 512, 2, -1, 0, 0},      {"reduce xq 512x2 slack4 prefix1024", 512, 2, -1, 4, 1024},
    {"reduce xq 512x2 slack8 prefix1024", 512, 2, -1, 8, 1024}, {"reduce xq 512x2 slack4", 512, 2, -1, 4, 0},
    {"reduce xq 1024x1 slack4 prefix512", 1024, 1, -1, 4, 512},
};

static unsigned* g_ctr = nullptr;   // 9 lines: dyn uses [0], [1]; xq heads at 32-word strides

template <int B, int U>
static void go_xq(const V& x, double* d, const double* s, size_t n, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  const size_t nvec = n / 2, ntiles = (nvec + (size_t)B * U - 1) / ((size_t)B * U);
  const unsigned prefix = (unsigned)((size_t)x.prefix < ntiles ? (size_t)x.prefix : ntiles);
  const size_t rest = ntiles - prefix;
  const unsigned qlen = (unsigned)((rest + 7) / 8);
  const unsigned grid = (unsigned)(prefix + rest + rest * (size_t)x.per_cu / 100 + (rest ? 8 : 0));
  hipExtLaunchKernelGGL((k_xq<B, U>), dim3(grid), dim3(B), 0, st, a, b, 0, (f64x2*)d, (const f64x2*)s, nvec,
                        g_ctr + 64, ntiles, prefix, qlen);
}
static int g_cus = 0;

template <int B, int U, int G>
static void go(const V& x, double* d, const double* s, size_t n, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  const size_t nvec = n / 2, ntiles = (nvec + (size_t)B * U - 1) / ((size_t)B * U);
  const unsigned grid = (unsigned)(g_cus * x.per_cu);
  if (G == 0) {
    hipExtLaunchKernelGGL((k_static<B, U>), dim3(grid), dim3(B), 0, st, a, b, 0, (f64x2*)d, (const f64x2*)s, nvec,
                          ntiles);
  } else {
    const unsigned ngrabs = (unsigned)((ntiles + G - 1) / G);
    hipExtLaunchKernelGGL((k_dyn<B, U, (G ? G : 1)>), dim3(grid), dim3(B), 0, st, a, b, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, g_ctr, ngrabs, ntiles);
  }
}

extern "C" const char* edge_name(int v) { return v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0])) ? kV[v].name : nullptr; }

extern "C" int edge_launch(int v, double* d, const double* s, size_t n, void* stream, void* e0, void* e1) {
  if (!edge_name(v)) return -1;
  if (!g_ctr) {
    if (hipMalloc(&g_ctr, 8192) != hipSuccess || hipMemset(g_ctr, 0, 8192) != hipSuccess) return -3;
    if (hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || g_cus <= 0) return -3;
    if (hipDeviceSynchronize() != hipSuccess) return -3;
  }
  const V& x = kV[v];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  if (x.grab < 0 && x.block == 512) go_xq<512, 2>(x, d, s, n, st, a, b);
  else if (x.grab < 0 && x.block == 1024) go_xq<1024, 1>(x, d, s, n, st, a, b);
  else if (x.block == 512 && x.grab == 1) go<512, 2, 1>(x, d, s, n, st, a, b);
  else if (x.block == 512 && x.grab == 2) go<512, 2, 2>(x, d, s, n, st, a, b);
  else if (x.block == 256 && x.grab == 1) go<256, 2, 1>(x, d, s, n, st, a, b);
  else if (x.block == 1024 && x.grab == 1) go<1024, 1, 1>(x, d, s, n, st, a, b);
  else if (x.block == 512 && x.grab == 0) go<512, 2, 0>(x, d, s, n, st, a, b);
  else if (x.block == 1024 && x.grab == 0) go<1024, 1, 0>(x, d, s, n, st, a, b);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// correctness probe for the runner: 1 if every counter is back at zero
extern "C" int dyn_counters_clear(void) {
  unsigned h[2048];
  if (!g_ctr || hipMemcpy(h, g_ctr, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  for (int i = 0; i < 2048; ++i)
    if (h[i]) return 0;
  return 1;
}
