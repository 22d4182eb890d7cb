// tools/lab/reduce_lab2.hip -- EXPERIMENTS ONLY (not part of libpg_amd.so).
//
// Occupancy and pipelining variants of the double-sum streaming reduce:
//  - one-shot tiles (as shipped) with the workgroups per CU capped by a
//    dynamic LDS reservation (no LDS is touched; the reservation only limits
//    how many workgroups a CU holds, i.e. the HBM requests in flight per CU);
//  - a persistent grid whose threads load tile t + grid before storing tile t;
//  - LDS-DMA staging of both operands (global_load_lds_dwordx4 -> ds_read_b128).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int B, int U>
__global__ __launch_bounds__(B) void oneshot(f64x2* __restrict__ d, const f64x2* __restrict__ s) {
  const size_t base = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(d + base + u * B);
#pragma unroll
  for (int u = 0; u < U; ++u) y[u] = __builtin_nontemporal_load(s + base + u * B);
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + y[u], d + base + u * B);
}

template <int B>
__global__ __launch_bounds__(B) void persist(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t ntiles) {
  size_t t = blockIdx.x;
  if (t >= ntiles) return;
  f64x2 x = __builtin_nontemporal_load(d + t * B + threadIdx.x);
  f64x2 y = __builtin_nontemporal_load(s + t * B + threadIdx.x);
  for (; t < ntiles; t += gridDim.x) {
    const size_t tn = t + gridDim.x;
    f64x2 xn = x, yn = y;
    if (tn < ntiles) {
      xn = __builtin_nontemporal_load(d + tn * B + threadIdx.x);
      yn = __builtin_nontemporal_load(s + tn * B + threadIdx.x);
    }
    __builtin_nontemporal_store(x + y, d + t * B + threadIdx.x);
    x = xn;
    y = yn;
  }
}

// LDS staging: both operands land in LDS by LDS-DMA (global_load_lds_dwordx4,
// nt), each wave reads back its own 64 lanes' vectors (ds_read_b128), adds,
// and stores from registers.  LDS destination is wave-uniform base + lane*16.
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

template <int B, int U>
__global__ __launch_bounds__(B) void glds(f64x2* __restrict__ d, const f64x2* __restrict__ s) {
  __shared__ f64x2 la[B * U], lb[B * U];
  const size_t base = (size_t)blockIdx.x * B * U + threadIdx.x;
  const int w = threadIdx.x / 64;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    __builtin_amdgcn_global_load_lds((glb_void*)(d + base + u * B), (lds_void*)(la + u * B + w * 64), 16, 0, 2);
    __builtin_amdgcn_global_load_lds((glb_void*)(s + base + u * B), (lds_void*)(lb + u * B + w * 64), 16, 0, 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < U; ++u)
    __builtin_nontemporal_store(la[u * B + threadIdx.x] + lb[u * B + threadIdx.x], d + base + u * B);
}

struct V {
  const char* name;
  int kind;        // 0 oneshot, 1 persist, 2 LDS-DMA staged oneshot
  int block, unroll, lds_kib, per_cu;
};

static const V kV[] = {
    {"oneshot 1024x1 lds0", 0, 1024, 1, 0, 0},
    {"oneshot 1024x1 lds96 (1 WG/CU)", 0, 1024, 1, 96, 0},
    {"oneshot 1024x2 lds96 (1 WG/CU)", 0, 1024, 2, 96, 0},
    {"oneshot 512x2 lds0", 0, 512, 2, 0, 0},
    {"oneshot 512x2 lds64 (2 WG/CU)", 0, 512, 2, 64, 0},
    {"oneshot 512x2 lds96 (1 WG/CU)", 0, 512, 2, 96, 0},
    {"oneshot 512x4 lds96 (1 WG/CU)", 0, 512, 4, 96, 0},
    {"oneshot 256x4 lds48 (3 WG/CU)", 0, 256, 4, 48, 0},
    {"oneshot 256x4 lds32 (5 WG/CU)", 0, 256, 4, 32, 0},
    {"oneshot 256x8 lds96 (1 WG/CU)", 0, 256, 8, 96, 0},
    {"oneshot 256x2 lds0", 0, 256, 2, 0, 0},
    {"oneshot 256x4 lds0", 0, 256, 4, 0, 0},
    {"oneshot 256x8 lds0", 0, 256, 8, 0, 0},
    {"oneshot 512x4 lds0", 0, 512, 4, 0, 0},
    {"glds (LDS-DMA staged) 1024x1", 2, 1024, 1, 0, 0},
    {"glds (LDS-DMA staged) 512x2", 2, 512, 2, 0, 0},
    {"glds (LDS-DMA staged) 256x4", 2, 256, 4, 0, 0},
    {"persist 1024 x2/CU", 1, 1024, 1, 0, 2},
    {"persist 1024 x1/CU", 1, 1024, 1, 0, 1},
    {"persist 512 x4/CU", 1, 512, 1, 0, 4},
    {"persist 256 x8/CU", 1, 256, 1, 0, 8},
};

extern "C" const char* lab2_name(int v) {
  return (v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0]))) ? kV[v].name : nullptr;
}

template <int B, int U>
static void go1(const V& v, f64x2* d, const f64x2* s, size_t nvec, hipStream_t st) {
  size_t grid = nvec / (B * U);
  hipLaunchKernelGGL((oneshot<B, U>), dim3((unsigned)grid), dim3(B), (size_t)v.lds_kib * 1024, st, d, s);
}

template <int B>
static void go2(const V& v, f64x2* d, const f64x2* s, size_t nvec, hipStream_t st) {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipLaunchKernelGGL((persist<B>), dim3((unsigned)(cus * v.per_cu)), dim3(B), 0, st, d, s, nvec / B);
}

// n doubles, a multiple of 2 * 1024 * 4
extern "C" int lab2_launch(int vi, double* d, const double* s, size_t n, void* stream) {
  if (!lab2_name(vi) || n % 8192) return -4;
  const V& v = kV[vi];
  f64x2* vd = (f64x2*)d;
  const f64x2* vs = (const f64x2*)s;
  size_t nvec = n / 2;
  hipStream_t st = (hipStream_t)stream;
  if (v.kind == 0) {
    switch (v.block * 16 + v.unroll) {
      case 1024 * 16 + 1: go1<1024, 1>(v, vd, vs, nvec, st); break;
      case 1024 * 16 + 2: go1<1024, 2>(v, vd, vs, nvec, st); break;
      case 512 * 16 + 2: go1<512, 2>(v, vd, vs, nvec, st); break;
      case 512 * 16 + 4: go1<512, 4>(v, vd, vs, nvec, st); break;
      case 256 * 16 + 2: go1<256, 2>(v, vd, vs, nvec, st); break;
      case 256 * 16 + 4: go1<256, 4>(v, vd, vs, nvec, st); break;
      case 256 * 16 + 8: go1<256, 8>(v, vd, vs, nvec, st); break;
      default: return -5;
    }
  } else if (v.kind == 2) {
    size_t grid = nvec / (v.block * v.unroll);
    switch (v.block) {
      case 1024: hipLaunchKernelGGL((glds<1024, 1>), dim3((unsigned)grid), dim3(1024), 0, st, vd, vs); break;
      case 512: hipLaunchKernelGGL((glds<512, 2>), dim3((unsigned)grid), dim3(512), 0, st, vd, vs); break;
      case 256: hipLaunchKernelGGL((glds<256, 4>), dim3((unsigned)grid), dim3(256), 0, st, vd, vs); break;
      default: return -5;
    }
  } else {
    switch (v.block) {
      case 1024: go2<1024>(v, vd, vs, nvec, st); break;
      case 512: go2<512>(v, vd, vs, nvec, st); break;
      case 256: go2<256>(v, vd, vs, nvec, st); break;
      default: return -5;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
