// EXPERIMENTS ONLY (tools/lab/run_edge_lab.py): where the fixed cost of one
// reduce launch goes.  Kernel-stamped (hipExtLaunchKernelGGL start/stop)
// durations of: an empty grid of the reduce's shape, read-only and write-only
// streams of the same bytes, a copy, and the reduce itself in several tile
// sizes, across operand sizes -- a linear fit t = t0 + bytes / bw per variant
// separates the per-launch edge (t0) from the streaming rate (bw).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int B>
__global__ __launch_bounds__(B) void k_empty(f64x2* d) {
  if (threadIdx.x == 0x7fffffff) d[0] = f64x2{0, 0};
}

// read a and b, keep a running sum; store only if it equals an impossible
// value, so the loads stay live and nothing is written
template <int B, int U>
__global__ __launch_bounds__(B) void k_read(const f64x2* __restrict__ a, const f64x2* __restrict__ b, size_t nvec,
                                            f64x2* sink) {
  size_t i = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 acc{0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) acc += __builtin_nontemporal_load(a + i + u * B) + __builtin_nontemporal_load(b + i + u * B);
  if (acc.x == 1.2345e300) sink[0] = acc;
}

template <int B, int U>
__global__ __launch_bounds__(B) void k_write(f64x2* __restrict__ d, size_t nvec) {
  size_t i = (size_t)blockIdx.x * B * U + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) __builtin_nontemporal_store(f64x2{1.0, 2.0}, d + i + u * B);
}

template <int B, int U>
__global__ __launch_bounds__(B) void k_copy(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec) {
  size_t i = (size_t)blockIdx.x * B * U + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i + u * B), d + i + u * B);
}

template <int B, int U>
__global__ __launch_bounds__(B) void k_reduce(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec) {
  size_t i = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) x[u] = __builtin_nontemporal_load(d + i + u * B);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) y[u] = __builtin_nontemporal_load(s + i + u * B);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * B < nvec) __builtin_nontemporal_store(x[u] + y[u], d + i + u * B);
}

struct V {
  const char* name;
  int kind;      // 0 empty, 1 read, 2 write, 3 copy, 4 reduce
  int block, unroll;
};
static const V kV[] = {
    {"empty 512x2 grid", 0, 512, 2}, {"empty 1 block", 0, 64, 0},
    {"read a+b 512x2", 1, 512, 2},   {"write d 512x2", 2, 512, 2},
    {"copy s->d 512x2", 3, 512, 2},  {"reduce 512x2 (shipped <128MiB)", 4, 512, 2},
    {"reduce 256x1", 4, 256, 1},     {"reduce 256x2", 4, 256, 2},
    {"reduce 1024x1", 4, 1024, 1},   {"reduce 1024x4", 4, 1024, 4},
    {"reduce 512x4", 4, 512, 4},
    {"reduce 128x2", 4, 128, 2},     {"reduce 128x4", 4, 128, 4},
    {"reduce 256x4", 4, 256, 4},     {"reduce 512x1", 4, 512, 1},
    {"reduce 768x1", 4, 768, 1},     {"reduce 1024x2", 4, 1024, 2},
};

template <int B, int U>
static void go(int kind, double* d, const double* s, size_t n, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  size_t nvec = n / 2;
  unsigned grid = (unsigned)((nvec + (size_t)B * U - 1) / ((size_t)B * U));
  f64x2* vd = (f64x2*)d;
  const f64x2* vs = (const f64x2*)s;
  switch (kind) {
    case 0: hipExtLaunchKernelGGL((k_empty<B>), dim3(grid), dim3(B), 0, st, e0, e1, 0, vd); break;
    case 1: hipExtLaunchKernelGGL((k_read<B, U>), dim3(grid), dim3(B), 0, st, e0, e1, 0, (const f64x2*)vd, vs, nvec, vd); break;
    case 2: hipExtLaunchKernelGGL((k_write<B, U>), dim3(grid), dim3(B), 0, st, e0, e1, 0, vd, nvec); break;
    case 3: hipExtLaunchKernelGGL((k_copy<B, U>), dim3(grid), dim3(B), 0, st, e0, e1, 0, vd, vs, nvec); break;
    default: hipExtLaunchKernelGGL((k_reduce<B, U>), dim3(grid), dim3(B), 0, st, e0, e1, 0, vd, vs, nvec);
  }
}

extern "C" const char* edge_name(int v) { return v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0])) ? kV[v].name : nullptr; }

extern "C" int edge_launch(int v, double* d, const double* s, size_t n, void* stream, void* e0, void* e1) {
  if (!edge_name(v)) return -1;
  const V& x = kV[v];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  if (x.kind == 0 && x.unroll == 0) {
    hipExtLaunchKernelGGL((k_empty<64>), dim3(1), dim3(64), 0, st, a, b, 0, (f64x2*)d);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  switch (x.block * 16 + x.unroll) {
    case 512 * 16 + 2: go<512, 2>(x.kind, d, s, n, st, a, b); break;
    case 256 * 16 + 1: go<256, 1>(x.kind, d, s, n, st, a, b); break;
    case 256 * 16 + 2: go<256, 2>(x.kind, d, s, n, st, a, b); break;
    case 1024 * 16 + 1: go<1024, 1>(x.kind, d, s, n, st, a, b); break;
    case 1024 * 16 + 4: go<1024, 4>(x.kind, d, s, n, st, a, b); break;
    case 512 * 16 + 4: go<512, 4>(x.kind, d, s, n, st, a, b); break;
    case 128 * 16 + 2: go<128, 2>(x.kind, d, s, n, st, a, b); break;
    case 128 * 16 + 4: go<128, 4>(x.kind, d, s, n, st, a, b); break;
    case 256 * 16 + 4: go<256, 4>(x.kind, d, s, n, st, a, b); break;
    case 512 * 16 + 1: go<512, 1>(x.kind, d, s, n, st, a, b); break;
    case 768 * 16 + 1: go<768, 1>(x.kind, d, s, n, st, a, b); break;
    case 1024 * 16 + 2: go<1024, 2>(x.kind, d, s, n, st, a, b); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
