// EXPERIMENTS ONLY (tools/lab/run_fold_lab.py): the 8-source fold
// out = s0 op s1 op ... op s7 (the direct exchange's and the xgmi transport's
// kernel, pgk_reduce_multi) in several shapes, kernel-stamped.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
struct Src8 { const f64x2* p[8]; };

// B threads, U vectors per source per thread (at i + u*B), all 8*U loads issued
// before the fold
template <int B, int U>
__global__ __launch_bounds__(B) void k_fold(f64x2* __restrict__ out, Src8 s, size_t nvec) {
  size_t i = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 x[8][U];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i + u * B < nvec) x[j][u] = __builtin_nontemporal_load(s.p[j] + i + u * B);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (i + u * B >= nvec) continue;
    f64x2 acc = x[0][u];
#pragma unroll
    for (int j = 1; j < 8; ++j) acc += x[j][u];
    __builtin_nontemporal_store(acc, out + i + u * B);
  }
}

// two halves: sources 0-3 loaded and folded, then 4-7 (half the registers)
template <int B>
__global__ __launch_bounds__(B) void k_fold_halves(f64x2* __restrict__ out, Src8 s, size_t nvec) {
  size_t i = (size_t)blockIdx.x * B + threadIdx.x;
  if (i >= nvec) return;
  f64x2 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = __builtin_nontemporal_load(s.p[j] + i);
  f64x2 acc = a[0] + a[1];
  acc += a[2];
  acc += a[3];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = __builtin_nontemporal_load(s.p[4 + j] + i);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc += a[j];
  __builtin_nontemporal_store(acc, out + i);
}

struct V { const char* name; int kind, block, unroll; };
static const V kV[] = {
    {"fold 512x1", 0, 512, 1}, {"fold 256x1", 0, 256, 1}, {"fold 1024x1", 0, 1024, 1},
    {"fold 256x2", 0, 256, 2}, {"fold 512x2", 0, 512, 2}, {"fold 128x2", 0, 128, 2},
    {"fold halves 512", 1, 512, 1}, {"fold halves 256", 1, 256, 1},
};

extern "C" const char* fold_name(int v) { return v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0])) ? kV[v].name : nullptr; }

template <int B, int U>
static void go(int kind, f64x2* out, Src8 s, size_t nvec, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  unsigned grid = (unsigned)((nvec + (size_t)B * U - 1) / ((size_t)B * U));
  if (kind == 0) hipExtLaunchKernelGGL((k_fold<B, U>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec);
  else hipExtLaunchKernelGGL((k_fold_halves<B>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec);
}

extern "C" int fold_launch(int v, double* out, const double* const* srcs, size_t n, void* stream, void* e0, void* e1) {
  if (!fold_name(v)) return -1;
  Src8 s;
  for (int j = 0; j < 8; ++j) s.p[j] = (const f64x2*)srcs[j];
  const V& x = kV[v];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  f64x2* o = (f64x2*)out;
  size_t nvec = n / 2;
  switch (x.block * 16 + x.unroll) {
    case 512 * 16 + 1: go<512, 1>(x.kind, o, s, nvec, st, a, b); break;
    case 256 * 16 + 1: go<256, 1>(x.kind, o, s, nvec, st, a, b); break;
    case 1024 * 16 + 1: go<1024, 1>(x.kind, o, s, nvec, st, a, b); break;
    case 256 * 16 + 2: go<256, 2>(x.kind, o, s, nvec, st, a, b); break;
    case 512 * 16 + 2: go<512, 2>(x.kind, o, s, nvec, st, a, b); break;
    case 128 * 16 + 2: go<128, 2>(x.kind, o, s, nvec, st, a, b); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
