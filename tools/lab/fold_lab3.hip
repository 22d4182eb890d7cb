// EXPERIMENTS ONLY (tools/lab/run_fold_lab3.py): what holds the 8-source fold
// at ~75% of the HBM peak when its eight reads alone stream at 85%?  Variants
// of the store side and of the wave turnover, all on separate source regions
// (the runner also skews the regions against each other):
//   kind 0  one-shot grid, nt loads, nt store            (as shipped)
//   kind 1  one-shot grid, nt loads, plain store
//   kind 2  one-shot grid, plain loads, nt store
//   kind 3  resident grid: each block walks tiles grid-strided and issues tile
//           t+1's loads before it folds and stores tile t
//   kind 4  one-shot grid, nt loads, nt store, the sum kept in a register and
//           stored only after a block barrier (all of a block's stores leave together)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
struct Src8 { const f64x2* p[8]; };

template <bool NT> __device__ __forceinline__ f64x2 ldv(const f64x2* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT> __device__ __forceinline__ void stv(f64x2* p, f64x2 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int B, int U, bool NTL, bool NTS, bool BAR>
__global__ __launch_bounds__(B) void k_fold(f64x2* __restrict__ out, Src8 s, size_t nvec) {
  size_t i = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 x[8][U];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i + u * B < nvec) x[j][u] = ldv<NTL>(s.p[j] + i + u * B);
  f64x2 acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    acc[u] = x[0][u];
#pragma unroll
    for (int j = 1; j < 8; ++j) acc[u] += x[j][u];
  }
  if (BAR) __syncthreads();
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) stv<NTS>(out + i + u * B, acc[u]);
}

// resident grid with the next tile's loads in flight across the store
template <int B>
__global__ __launch_bounds__(B) void k_fold_pipe(f64x2* __restrict__ out, Src8 s, size_t nvec) {
  const size_t stride = (size_t)gridDim.x * B;
  size_t i = (size_t)blockIdx.x * B + threadIdx.x;
  f64x2 x[8], y[8];
  if (i < nvec) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = ldv<true>(s.p[j] + i);
  }
  while (i < nvec) {
    const size_t nx = i + stride;
    if (nx < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = ldv<true>(s.p[j] + nx);
    }
    f64x2 acc = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) acc += x[j];
    stv<true>(out + i, acc);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = y[j];
    i = nx;
  }
}

template <int B, int U>
static int go(int kind, f64x2* out, Src8 s, size_t nvec, int blocks_per_cu, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  const size_t tile = (size_t)B * U;
  unsigned grid = (unsigned)((nvec + tile - 1) / tile);
  switch (kind) {
    case 0: hipExtLaunchKernelGGL((k_fold<B, U, true, true, false>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec); break;
    case 1: hipExtLaunchKernelGGL((k_fold<B, U, true, false, false>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec); break;
    case 2: hipExtLaunchKernelGGL((k_fold<B, U, false, true, false>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec); break;
    case 3: {
      unsigned g = 256u * (unsigned)blocks_per_cu;
      if (g > grid) g = grid;
      hipExtLaunchKernelGGL((k_fold_pipe<B>), dim3(g), dim3(B), 0, st, a, b, 0, out, s, nvec);
      break;
    }
    case 4: hipExtLaunchKernelGGL((k_fold<B, U, true, true, true>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int fold3_launch(int kind, int block, int unroll, int blocks_per_cu, double* out, const double* const* srcs,
                            size_t n, void* stream, void* e0, void* e1) {
  Src8 s;
  for (int j = 0; j < 8; ++j) s.p[j] = (const f64x2*)srcs[j];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  f64x2* o = (f64x2*)out;
  const size_t nvec = n / 2;
  switch (block * 16 + unroll) {
    case 512 * 16 + 1: return go<512, 1>(kind, o, s, nvec, blocks_per_cu, st, a, b);
    case 256 * 16 + 1: return go<256, 1>(kind, o, s, nvec, blocks_per_cu, st, a, b);
    case 128 * 16 + 1: return go<128, 1>(kind, o, s, nvec, blocks_per_cu, st, a, b);
    case 64 * 16 + 1: return go<64, 1>(kind, o, s, nvec, blocks_per_cu, st, a, b);
    case 64 * 16 + 4: return go<64, 4>(kind, o, s, nvec, blocks_per_cu, st, a, b);
    case 256 * 16 + 4: return go<256, 4>(kind, o, s, nvec, blocks_per_cu, st, a, b);
    case 1024 * 16 + 1: return go<1024, 1>(kind, o, s, nvec, blocks_per_cu, st, a, b);
    default: return -1;
  }
}
