// EXPERIMENTS ONLY (tools/lab/run_edge_lab.py --lab policy): the reduce's
// store cache policy.  nt stores keep the written line in the XCD's L2 (dirty,
// written back on eviction or at the end-of-kernel release); sc1 stores are
// write-through and drop it.  Each variant is the shipped k_reduce_vec body
// (nt loads, 16-B vectors) with its stores issued as buffer stores carrying
// the named aux bits (gfx950: sc0 = 1, nt = 2, sc1 = 16), so the fit of
// run_edge_lab.py shows whether the policy moves the launch edge (t0) or the
// streaming rate (bw).  Same exported API as edge_lab.hip.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// one descriptor per block over the block's own tile (wave-uniform base)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)bytes, 0x00020000);
}

template <int B, int U, int AUX>
__global__ __launch_bounds__(B) void k_reduce_pol(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec) {
  const size_t tile0 = (size_t)blockIdx.x * B * U;
  const size_t i = tile0 + threadIdx.x;
  f64x2 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) x[u] = __builtin_nontemporal_load(d + i + u * B);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) y[u] = __builtin_nontemporal_load(s + i + u * B);
  const size_t left = nvec - tile0;
  const uint32_t tile_bytes = (uint32_t)((left < (size_t)B * U ? left : (size_t)B * U) * sizeof(f64x2));
  __amdgpu_buffer_rsrc_t r = tile_rsrc(d + tile0, tile_bytes);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) {
      f64x2 z = x[u] + y[u];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, z), r,
                                             (int)((threadIdx.x + u * B) * sizeof(f64x2)), 0, AUX);
    }
}

template <int B, int U, int AUX>
__global__ __launch_bounds__(B) void k_write_pol(f64x2* __restrict__ d, size_t nvec) {
  const size_t tile0 = (size_t)blockIdx.x * B * U;
  const size_t i = tile0 + threadIdx.x;
  const size_t left = nvec - tile0;
  const uint32_t tile_bytes = (uint32_t)((left < (size_t)B * U ? left : (size_t)B * U) * sizeof(f64x2));
  __amdgpu_buffer_rsrc_t r = tile_rsrc(d + tile0, tile_bytes);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, f64x2{1.0, 2.0}), r,
                                             (int)((threadIdx.x + u * B) * sizeof(f64x2)), 0, AUX);
}

struct V {
  const char* name;
  int kind;  // 2 write, 4 reduce
  int block, unroll, aux;
};
static const V kV[] = {
    {"reduce 512x2 buf nt", 4, 512, 2, 2},      {"reduce 512x2 buf plain", 4, 512, 2, 0},
    {"reduce 512x2 buf sc1", 4, 512, 2, 16},    {"reduce 512x2 buf sc0 sc1", 4, 512, 2, 17},
    {"reduce 512x2 buf sc1 nt", 4, 512, 2, 18}, {"reduce 1024x1 buf nt", 4, 1024, 1, 2},
    {"reduce 1024x1 buf sc1", 4, 1024, 1, 16},  {"reduce 1024x1 buf sc1 nt", 4, 1024, 1, 18},
    {"write 512x2 buf nt", 2, 512, 2, 2},       {"write 512x2 buf sc1", 2, 512, 2, 16},
    {"write 512x2 buf sc1 nt", 2, 512, 2, 18},
};

template <int B, int U, int AUX>
static void go(int kind, double* d, const double* s, size_t n, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  size_t nvec = n / 2;
  unsigned grid = (unsigned)((nvec + (size_t)B * U - 1) / ((size_t)B * U));
  if (kind == 2)
    hipExtLaunchKernelGGL((k_write_pol<B, U, AUX>), dim3(grid), dim3(B), 0, st, e0, e1, 0, (f64x2*)d, nvec);
  else
    hipExtLaunchKernelGGL((k_reduce_pol<B, U, AUX>), dim3(grid), dim3(B), 0, st, e0, e1, 0, (f64x2*)d,
                          (const f64x2*)s, nvec);
}

template <int B, int U>
static int by_aux(int aux, int kind, double* d, const double* s, size_t n, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  switch (aux) {
    case 0: go<B, U, 0>(kind, d, s, n, st, a, b); break;
    case 2: go<B, U, 2>(kind, d, s, n, st, a, b); break;
    case 16: go<B, U, 16>(kind, d, s, n, st, a, b); break;
    case 17: go<B, U, 17>(kind, d, s, n, st, a, b); break;
    case 18: go<B, U, 18>(kind, d, s, n, st, a, b); break;
    default: return -1;
  }
  return 0;
}

extern "C" const char* edge_name(int v) { return v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0])) ? kV[v].name : nullptr; }

extern "C" int edge_launch(int v, double* d, const double* s, size_t n, void* stream, void* e0, void* e1) {
  if (!edge_name(v)) return -1;
  const V& x = kV[v];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  int rc;
  if (x.block == 512 && x.unroll == 2) rc = by_aux<512, 2>(x.aux, x.kind, d, s, n, st, a, b);
  else if (x.block == 1024 && x.unroll == 1) rc = by_aux<1024, 1>(x.aux, x.kind, d, s, n, st, a, b);
  else return -1;
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
