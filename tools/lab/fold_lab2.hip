// EXPERIMENTS ONLY (tools/lab/run_fold_lab2.py): does it matter WHERE the
// eight sources of the fold lie?  The shipped fold reads eight separate
// regions, so the tiles in flight span eight distant address ranges.  Here the
// same fold reads sources interleaved by granule inside one region:
//     vector i of source j  =  base[((i / G) * NS + j) * G + i % G]
// (G vectors per granule, a power of two and a multiple of the block's tile),
// against the separate layout, in the same run.  Also: the eight reads alone
// (no store), to see what the read side reaches on its own.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
struct Src8 { const f64x2* p[8]; };

// separate regions: B threads, U vectors per source per thread
template <int B, int U, bool STORE>
__global__ __launch_bounds__(B) void k_fold_sep(f64x2* __restrict__ out, Src8 s, size_t nvec) {
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
    if (STORE) __builtin_nontemporal_store(acc, out + i + u * B);
    else if (acc.x == 1.2345e300) out[0] = acc;
  }
}

// NI sources interleaved by granule (2^lg vectors) in `base`, the other 8 - NI
// separate in s.p[NI..7]; fold order j = 0..7 as in the separate kernel
template <int B, int U, int NI>
__global__ __launch_bounds__(B) void k_fold_il(f64x2* __restrict__ out, const f64x2* __restrict__ base, Src8 s,
                                               size_t nvec, int lg) {
  const size_t i0 = (size_t)blockIdx.x * B * U;          // the block's tile lies inside one granule
  const size_t g = i0 >> lg, in = i0 & (((size_t)1 << lg) - 1);
  const f64x2* gb = base + ((g * NI) << lg) + in + threadIdx.x;
  const size_t i = i0 + threadIdx.x;
  f64x2 x[8][U];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i + u * B < nvec)
        x[j][u] = j < NI ? __builtin_nontemporal_load(gb + ((size_t)j << lg) + u * B)
                         : __builtin_nontemporal_load(s.p[j] + i + u * B);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (i + u * B >= nvec) continue;
    f64x2 acc = x[0][u];
#pragma unroll
    for (int j = 1; j < 8; ++j) acc += x[j][u];
    __builtin_nontemporal_store(acc, out + i + u * B);
  }
}

template <int B, int U>
static int go(int kind, f64x2* out, const f64x2* base, Src8 s, size_t nvec, int lg, hipStream_t st, hipEvent_t a,
              hipEvent_t b) {
  const size_t tile = (size_t)B * U;
  unsigned grid = (unsigned)((nvec + tile - 1) / tile);
  if (kind >= 2 && (((size_t)1 << lg) % tile || nvec % ((size_t)1 << lg))) return -3;
  switch (kind) {
    case 0: hipExtLaunchKernelGGL((k_fold_sep<B, U, true>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec); break;
    case 1: hipExtLaunchKernelGGL((k_fold_sep<B, U, false>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec); break;
    case 2: hipExtLaunchKernelGGL((k_fold_il<B, U, 8>), dim3(grid), dim3(B), 0, st, a, b, 0, out, base, s, nvec, lg); break;
    case 3: hipExtLaunchKernelGGL((k_fold_il<B, U, 7>), dim3(grid), dim3(B), 0, st, a, b, 0, out, base, s, nvec, lg); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// kind: 0 separate, 1 separate reads only, 2 all 8 interleaved, 3 sources 0-6
// interleaved + source 7 separate.  granule = 2^lg vectors of 16 B.
extern "C" int fold2_launch(int kind, int block, int unroll, double* out, const double* base,
                            const double* const* srcs, size_t n, int lg, void* stream, void* e0, void* e1) {
  Src8 s;
  for (int j = 0; j < 8; ++j) s.p[j] = (const f64x2*)srcs[j];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  f64x2* o = (f64x2*)out;
  const f64x2* bs = (const f64x2*)base;
  const size_t nvec = n / 2;
  switch (block * 16 + unroll) {
    case 512 * 16 + 1: return go<512, 1>(kind, o, bs, s, nvec, lg, st, a, b);
    case 256 * 16 + 2: return go<256, 2>(kind, o, bs, s, nvec, lg, st, a, b);
    case 1024 * 16 + 1: return go<1024, 1>(kind, o, bs, s, nvec, lg, st, a, b);
    case 256 * 16 + 1: return go<256, 1>(kind, o, bs, s, nvec, lg, st, a, b);
    default: return -1;
  }
}
