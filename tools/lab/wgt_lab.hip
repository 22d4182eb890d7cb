// EXPERIMENTS ONLY (tools/lab/run_edge_lab.py --lab wgt): weighted tiles for
// the XCD rate split.  The timeline lab measured block b running on XCD
// b mod 8 in every launch (r02_timeline_xcd.txt, "dealing"), and XCDs 0/2/4/6
// streaming ~4% faster than 1/3/5/7.  Here an even block takes T + D vectors
// and the odd block after it T - D, so the even XCDs get 2·D/T more of the
// bytes.  The tile layout depends on blockIdx only: every vector is covered
// once wherever the blocks run; only the balance depends on the dealing.
// Same API as edge_lab.hip.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

// B threads, nominal tile T = B*U vectors; a pair of blocks covers 2T
template <int B, int U>
__global__ __launch_bounds__(B) void k_wgt(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec, int D) {
  constexpr int T = B * U;
  const size_t pair = blockIdx.x >> 1;
  const bool odd = blockIdx.x & 1;
  const size_t start = pair * 2 * T + (odd ? (size_t)(T + D) : 0);
  size_t end = start + (odd ? T - D : T + D);
  if (end > nvec) end = nvec;
  const size_t i = start + threadIdx.x;
  if (i + (size_t)(U - 1) * B < end && i + (size_t)U * B >= end) {
    // the common case: exactly U vectors per lane, no lane of an extra one
    f64x2 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = __builtin_nontemporal_load(d + i + u * B);
      y[u] = __builtin_nontemporal_load(s + i + u * B);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + y[u], d + i + u * B);
    return;
  }
  f64x2 x[U + 1], y[U + 1];
#pragma unroll
  for (int u = 0; u <= U; ++u)
    if (i + u * B < end) {
      x[u] = __builtin_nontemporal_load(d + i + u * B);
      y[u] = __builtin_nontemporal_load(s + i + u * B);
    }
#pragma unroll
  for (int u = 0; u <= U; ++u)
    if (i + u * B < end) __builtin_nontemporal_store(x[u] + y[u], d + i + u * B);
}


// Dummy blocks instead of ragged tiles: the grid is cut into periods of K
// rounds of 8 blocks (one per XCD per round); in the last round of each period
// the blocks on odd XCDs exit at once, so an odd XCD streams (K-1)/K of an
// even one's tiles.  Tiles stay whole (16-B vectors x B*U, aligned), and real
// block r(b) takes tile r(b), a function of blockIdx only.
template <int B, int U>
__global__ __launch_bounds__(B) void k_skip(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec, int K,
                                            size_t ntiles) {
  const size_t per = 8 * (size_t)K;
  const size_t p = blockIdx.x / per, w = blockIdx.x % per, j = w / 8, x = w % 8;
  if (j == (size_t)K - 1 && (x & 1)) return;
  const size_t r = p * (per - 4) + (j < (size_t)K - 1 ? w : 8 * ((size_t)K - 1) + x / 2);
  if (r >= ntiles) return;
  const size_t i = r * B * U + threadIdx.x;
  if (i + (size_t)(U - 1) * B < nvec) {
    f64x2 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = __builtin_nontemporal_load(d + i + u * B);
      b[u] = __builtin_nontemporal_load(s + i + u * B);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u] + b[u], d + i + u * B);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * B < nvec)
        __builtin_nontemporal_store(__builtin_nontemporal_load(d + i + u * B) + __builtin_nontemporal_load(s + i + u * B),
                                    d + i + u * B);
  }
}


// Parity swap: block b takes tile b ^ ((b >> 3) & 1), so every XCD (b mod 8)
// alternates between even and odd tiles; grid padded to a multiple of 16.
template <int B, int U>
__global__ __launch_bounds__(B) void k_swap(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec) {
  const size_t t = blockIdx.x ^ ((blockIdx.x >> 3) & 1);
  const size_t i = t * B * U + threadIdx.x;
  if (i + (size_t)(U - 1) * B < nvec) {
    f64x2 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = __builtin_nontemporal_load(d + i + u * B);
      b[u] = __builtin_nontemporal_load(s + i + u * B);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u] + b[u], d + i + u * B);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * B < nvec)
        __builtin_nontemporal_store(__builtin_nontemporal_load(d + i + u * B) + __builtin_nontemporal_load(s + i + u * B),
                                    d + i + u * B);
  }
}

struct V {
  const char* name;
  int block, unroll, D;   // D < 0: k_skip with K = -D; D = 1 << 20: k_swap
};
static const V kV[] = {
    {"reduce wgt 512x2 D0", 512, 2, 0},      {"reduce wgt 512x2 D16", 512, 2, 16},
    {"reduce wgt 512x2 D24", 512, 2, 24},    {"reduce wgt 512x2 D40", 512, 2, 40},
    {"reduce wgt 1024x1 D0", 1024, 1, 0},    {"reduce wgt 1024x1 D16", 1024, 1, 16},
    {"reduce wgt 1024x1 D24", 1024, 1, 24},  {"reduce wgt 256x4 D24", 256, 4, 24},
    {"reduce skip 512x2 K13", 512, 2, -13},  {"reduce skip 512x2 K25", 512, 2, -25},
    {"reduce skip 512x2 K50", 512, 2, -50},  {"reduce skip 1024x1 K25", 1024, 1, -25},
    {"reduce swap 512x2", 512, 2, 1 << 20},  {"reduce swap 1024x1", 1024, 1, 1 << 20},
    {"reduce swap 256x4", 256, 4, 1 << 20},
};

template <int B, int U>
static void go(int D, double* d, const double* s, size_t n, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  const size_t nvec = n / 2, pairs = (nvec + 2 * (size_t)B * U - 1) / (2 * (size_t)B * U);
  if (D == (1 << 20)) {
    const size_t ntiles = (nvec + (size_t)B * U - 1) / ((size_t)B * U);
    hipExtLaunchKernelGGL((k_swap<B, U>), dim3((unsigned)((ntiles + 15) / 16 * 16)), dim3(B), 0, st, a, b, 0,
                          (f64x2*)d, (const f64x2*)s, nvec);
    return;
  }
  if (D < 0) {
    const size_t K = (size_t)-D, ntiles = (nvec + (size_t)B * U - 1) / ((size_t)B * U);
    const size_t periods = (ntiles + 8 * K - 4 - 1) / (8 * K - 4);
    hipExtLaunchKernelGGL((k_skip<B, U>), dim3((unsigned)(periods * 8 * K)), dim3(B), 0, st, a, b, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, (int)K, ntiles);
    return;
  }
  hipExtLaunchKernelGGL((k_wgt<B, U>), dim3((unsigned)(2 * pairs)), dim3(B), 0, st, a, b, 0, (f64x2*)d,
                        (const f64x2*)s, nvec, D);
}

extern "C" const char* edge_name(int v) { return v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0])) ? kV[v].name : nullptr; }

extern "C" int edge_launch(int v, double* d, const double* s, size_t n, void* stream, void* e0, void* e1) {
  if (!edge_name(v) || n % 2) return -1;
  const V& x = kV[v];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  if (x.block == 512) go<512, 2>(x.D, d, s, n, st, a, b);
  else if (x.block == 1024) go<1024, 1>(x.D, d, s, n, st, a, b);
  else if (x.block == 256) go<256, 4>(x.D, d, s, n, st, a, b);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int dyn_counters_clear(void) { return 1; }   // check_dyn_lab.py compatibility: no counters here
