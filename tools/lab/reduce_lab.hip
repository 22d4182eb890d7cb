// tools/lab/reduce_lab.hip -- EXPERIMENTS ONLY (not part of libpg_amd.so).
//
// Variants of the double-sum streaming reduce used to decide the shipped
// kernel's cache policy and geometry.  Buffer
// loads/stores with explicit gfx950 cache-policy bits (aux: 1 = sc0,
// 2 = nt, 16 = sc1), block sizes, an XCD-contiguous block remap and the load
// order.  One tile per block (one-shot grid); n must be a multiple of the tile.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int LAUX, int SAUX, int BLOCK, int U, bool XCD, bool INTERLEAVE>
__global__ __launch_bounds__(BLOCK) void lab(double* dst, const double* src) {
  unsigned b = blockIdx.x;
  if (XCD) b = (b % 8u) * (gridDim.x / 8u) + b / 8u;
  const size_t tile_bytes = (size_t)BLOCK * U * 16;
  char* d = (char*)dst + (size_t)b * tile_bytes;
  const char* s = (const char*)src + (size_t)b * tile_bytes;
  __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(d, (short)0, (int)tile_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)s, (short)0, (int)tile_bytes, 0x00020000);
  u32x4 x[U], y[U];
  if (INTERLEAVE) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = __builtin_amdgcn_raw_buffer_load_b128(rd, (threadIdx.x + u * BLOCK) * 16, 0, LAUX);
      y[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (threadIdx.x + u * BLOCK) * 16, 0, LAUX);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
      x[u] = __builtin_amdgcn_raw_buffer_load_b128(rd, (threadIdx.x + u * BLOCK) * 16, 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; ++u)
      y[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (threadIdx.x + u * BLOCK) * 16, 0, LAUX);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    f64x2 a = __builtin_bit_cast(f64x2, x[u]);
    f64x2 c = __builtin_bit_cast(f64x2, y[u]);
    a = a + c;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), rd, (threadIdx.x + u * BLOCK) * 16, 0, SAUX);
  }
}

template <int LAUX, int SAUX, int BLOCK, int U, bool XCD, bool IL>
static int go(double* d, const double* s, size_t n, hipStream_t st) {
  size_t tile = (size_t)BLOCK * U * 2;  // doubles per tile
  if (n % tile) return -2;
  size_t grid = n / tile;
  if (XCD && grid % 8) return -3;
  hipLaunchKernelGGL((lab<LAUX, SAUX, BLOCK, U, XCD, IL>), dim3((unsigned)grid), dim3(BLOCK), 0, st, d, s);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" const char* lab_name(int v) {
  static const char* names[] = {
      "buf aux 0/0 b256 u4", "buf nt/nt b256 u4", "buf nt/0 b256 u4", "buf 0/nt b256 u4",
      "buf nt+sc1/nt b256 u4", "buf nt/nt+sc1 b256 u4", "buf nt+sc1/nt+sc1 b256 u4", "buf nt+sc0/nt b256 u4",
      "buf nt/nt+sc0 b256 u4", "buf sc1/sc1 b256 u4", "buf nt/nt b256 u4 XCD-remap", "buf nt/nt b512 u2",
      "buf nt/nt b1024 u1", "buf nt/nt b256 u8", "buf nt/nt b256 u4 interleaved", "buf nt/nt b512 u4",
      "buf all/all b256 u4", "buf nt/nt b128 u8", "buf nt/nt b256 u2", "buf nt/nt b1024 u2"};
  return (v >= 0 && v < (int)(sizeof(names) / sizeof(names[0]))) ? names[v] : nullptr;
}

extern "C" int lab_launch(int v, double* d, const double* s, size_t n, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (v) {
    case 0: return go<0, 0, 256, 4, false, false>(d, s, n, st);
    case 1: return go<2, 2, 256, 4, false, false>(d, s, n, st);
    case 2: return go<2, 0, 256, 4, false, false>(d, s, n, st);
    case 3: return go<0, 2, 256, 4, false, false>(d, s, n, st);
    case 4: return go<18, 2, 256, 4, false, false>(d, s, n, st);
    case 5: return go<2, 18, 256, 4, false, false>(d, s, n, st);
    case 6: return go<18, 18, 256, 4, false, false>(d, s, n, st);
    case 7: return go<3, 2, 256, 4, false, false>(d, s, n, st);
    case 8: return go<2, 3, 256, 4, false, false>(d, s, n, st);
    case 9: return go<16, 16, 256, 4, false, false>(d, s, n, st);
    case 10: return go<2, 2, 256, 4, true, false>(d, s, n, st);
    case 11: return go<2, 2, 512, 2, false, false>(d, s, n, st);
    case 12: return go<2, 2, 1024, 1, false, false>(d, s, n, st);
    case 13: return go<2, 2, 256, 8, false, false>(d, s, n, st);
    case 14: return go<2, 2, 256, 4, false, true>(d, s, n, st);
    case 15: return go<2, 2, 512, 4, false, false>(d, s, n, st);
    case 16: return go<19, 19, 256, 4, false, false>(d, s, n, st);
    case 17: return go<2, 2, 128, 8, false, false>(d, s, n, st);
    case 18: return go<2, 2, 256, 2, false, false>(d, s, n, st);
    case 19: return go<2, 2, 1024, 2, false, false>(d, s, n, st);
  }
  return -4;
}
