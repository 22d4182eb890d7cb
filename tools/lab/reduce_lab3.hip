// tools/lab/reduce_lab3.hip -- EXPERIMENTS ONLY (not part of libpg_amd.so).
// Multi-source fold out = s0 op s1 op ... op s7 (double sum, 8 local sources):
// block size and vectors per thread, one-shot grid, nt loads and stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
struct Src8 { const f64x2* p[8]; };

template <int B, int U, bool SRC_MAJOR>
__global__ __launch_bounds__(B) void fold8(f64x2* __restrict__ out, Src8 s) {
  const size_t base = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 acc[U], x[U][8];
  if (SRC_MAJOR) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) x[u][j] = __builtin_nontemporal_load(s.p[j] + base + u * B);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) x[u][j] = __builtin_nontemporal_load(s.p[j] + base + u * B);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    acc[u] = x[u][0];
#pragma unroll
    for (int j = 1; j < 8; ++j) acc[u] = acc[u] + x[u][j];
    __builtin_nontemporal_store(acc[u], out + base + u * B);
  }
}

struct V { const char* name; int block, unroll, src_major; };
static const V kV[] = {
    {"fold8 256x1 (shipped shape)", 256, 1, 0}, {"fold8 512x1", 512, 1, 0}, {"fold8 1024x1", 1024, 1, 0},
    {"fold8 256x2", 256, 2, 0}, {"fold8 256x2 src-major", 256, 2, 1}, {"fold8 512x2", 512, 2, 0},
    {"fold8 128x2", 128, 2, 0}, {"fold8 128x4", 128, 4, 0}, {"fold8 64x4", 64, 4, 0}};

extern "C" const char* lab3_name(int v) {
  return (v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0]))) ? kV[v].name : nullptr;
}

template <int B, int U, bool SM>
static void go(f64x2* out, Src8 s, size_t nvec, hipStream_t st) {
  hipLaunchKernelGGL((fold8<B, U, SM>), dim3((unsigned)(nvec / (B * U))), dim3(B), 0, st, out, s);
}

// srcs: 8 pointers; n doubles, a multiple of 8192
extern "C" int lab3_launch(int vi, double* out, const double* const* srcs, size_t n, void* stream) {
  if (!lab3_name(vi) || n % 8192) return -4;
  Src8 s;
  for (int j = 0; j < 8; ++j) s.p[j] = (const f64x2*)srcs[j];
  size_t nvec = n / 2;
  hipStream_t st = (hipStream_t)stream;
  const V& v = kV[vi];
  switch (v.block * 100 + v.unroll * 10 + v.src_major) {
    case 25610: go<256, 1, false>((f64x2*)out, s, nvec, st); break;
    case 51210: go<512, 1, false>((f64x2*)out, s, nvec, st); break;
    case 102410: go<1024, 1, false>((f64x2*)out, s, nvec, st); break;
    case 25620: go<256, 2, false>((f64x2*)out, s, nvec, st); break;
    case 25621: go<256, 2, true>((f64x2*)out, s, nvec, st); break;
    case 51220: go<512, 2, false>((f64x2*)out, s, nvec, st); break;
    case 12820: go<128, 2, false>((f64x2*)out, s, nvec, st); break;
    case 12840: go<128, 4, false>((f64x2*)out, s, nvec, st); break;
    case 6440: go<64, 4, false>((f64x2*)out, s, nvec, st); break;
    default: return -5;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
