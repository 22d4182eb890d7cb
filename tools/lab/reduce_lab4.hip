// tools/lab/reduce_lab4.hip -- EXPERIMENTS ONLY (not part of libpg_amd.so).
//
// Cache-policy split of the double-sum streaming reduce at 64 MiB-1 GiB per
// operand: the shipped kernel marks loads AND stores non-temporal; these
// variants mark only one side, so the Infinity Cache (MALL) may hold what the
// other side touches.  Shapes 512x2 (shipped below 128 MiB) and 1024x1.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

template <bool NTL, bool NTS, int B, int U>
__global__ __launch_bounds__(B) void pol(f64x2* __restrict__ d, const f64x2* __restrict__ s) {
  const size_t base = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = NTL ? __builtin_nontemporal_load(d + base + u * B) : d[base + u * B];
#pragma unroll
  for (int u = 0; u < U; ++u) y[u] = NTL ? __builtin_nontemporal_load(s + base + u * B) : s[base + u * B];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (NTS) __builtin_nontemporal_store(x[u] + y[u], d + base + u * B);
    else d[base + u * B] = x[u] + y[u];
  }
}

// src non-temporal, dst (read then written) default policy: the dst lines may
// be kept for the write that follows
template <int B, int U>
__global__ __launch_bounds__(B) void mixsrc(f64x2* __restrict__ d, const f64x2* __restrict__ s) {
  const size_t base = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = d[base + u * B];
#pragma unroll
  for (int u = 0; u < U; ++u) y[u] = __builtin_nontemporal_load(s + base + u * B);
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + y[u], d + base + u * B);
}

struct V { const char* name; void (*k)(f64x2*, const f64x2*); int B, U; };

static const V kV[] = {
  {"512x2 ntload+ntstore (as shipped)", pol<true, true, 512, 2>, 512, 2},
  {"512x2 ntload+store", pol<true, false, 512, 2>, 512, 2},
  {"512x2 load+ntstore", pol<false, true, 512, 2>, 512, 2},
  {"512x2 load+store", pol<false, false, 512, 2>, 512, 2},
  {"512x2 dst load, src ntload, ntstore", mixsrc<512, 2>, 512, 2},
  {"1024x1 ntload+ntstore", pol<true, true, 1024, 1>, 1024, 1},
  {"1024x1 ntload+store", pol<true, false, 1024, 1>, 1024, 1},
  {"1024x1 load+ntstore", pol<false, true, 1024, 1>, 1024, 1},
  {"256x4 ntload+ntstore", pol<true, true, 256, 4>, 256, 4},
  {"256x4 ntload+store", pol<true, false, 256, 4>, 256, 4},
};

extern "C" const char* lab2_name(int v) {
  return (v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0]))) ? kV[v].name : nullptr;
}

extern "C" int lab2_launch(int vi, double* d, const double* s, size_t n, void* stream) {
  if (!lab2_name(vi) || n % 8192) return -4;
  const V& v = kV[vi];
  const size_t nv = n / 2, tile = (size_t)v.B * v.U;
  if (nv % tile) return -5;
  hipLaunchKernelGGL(v.k, dim3((unsigned)(nv / tile)), dim3(v.B), 0, (hipStream_t)stream,
                     reinterpret_cast<f64x2*>(d), reinterpret_cast<const f64x2*>(s));
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
