// EXPERIMENTS ONLY (tools/lab/run_timeline_lab.py): a diagnostic build of the
// reduce that stamps every workgroup's life on the GPU's constant 100 MHz
// clock (s_memrealtime), so one launch's time can be split into dispatch,
// ramp (first loads in flight), steady streaming and drain.  Per block:
//   [0] entry          wave 0, first instruction
//   [1] loaded         wave 0, its dst and src vectors returned
//   [2] stored         every wave's stores acknowledged (vmcnt 0), after a barrier
//   [3] XCC id         HW_REG_XCC_ID
// The stamps' waits forbid overlaps the shipped kernel has, so the runner
// reads shares of the timeline and compares the build's stamped duration with
// the shipped kernel's, never quotes this build's length as the kernel's.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

// SWAP: block b takes tile b ^ ((b >> 3) & 1), so the XCD of block b (b mod 8)
// works on tiles of both parities (address bit 14 at 16 KiB tiles) in turn.
// MODE 0: the reduce; 1: loads only (the sum is stored only if it is NaN,
// which the runner's inputs never are); 2: stores only (dst = src's address
// as a double, no loads).  Modes 1 and 2 ask which stream the rate decay
// over a long launch belongs to.
template <int B, int U, bool SWAP, int MODE = 0>
__global__ __launch_bounds__(B) void k_reduce_tl(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec,
                                                 unsigned long long* __restrict__ ts) {
  const unsigned long long t_entry = stamp();
  const size_t t = SWAP ? (blockIdx.x ^ ((blockIdx.x >> 3) & 1)) : blockIdx.x;
  const size_t i = t * B * U + threadIdx.x;
  const bool full = (t + 1) * B * U <= nvec;   // every tile but a ragged last one
  f64x2 x[U], y[U];
  if (MODE == 2) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = f64x2{(double)(i + u * B), 0.0};
      y[u] = f64x2{0.0, 0.0};
    }
  } else if (full) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = __builtin_nontemporal_load(d + i + u * B);
      y[u] = __builtin_nontemporal_load(s + i + u * B);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * B < nvec) {
        x[u] = __builtin_nontemporal_load(d + i + u * B);
        y[u] = __builtin_nontemporal_load(s + i + u * B);
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t_loaded = stamp();
  if (MODE == 1) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f64x2 v = x[u] + y[u];
      if (i + u * B < nvec && (v.x != v.x)) __builtin_nontemporal_store(v, d + i + u * B);
    }
  } else if (full) {
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + y[u], d + i + u * B);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * B < nvec) __builtin_nontemporal_store(x[u] + y[u], d + i + u * B);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t_stored = stamp();
  if (threadIdx.x == 0) {
    unsigned long long* r = ts + 4 * (size_t)blockIdx.x;
    r[0] = t_entry;
    r[1] = t_loaded;
    r[2] = t_stored;
    r[3] = xcc_id();
  }
}

extern "C" int tl_clock_khz(int* khz) {
  return hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, 0) == hipSuccess ? 0 : -1;
}

// shape 0: 512x2 (shipped below 128 MiB per operand), 1: 1024x1 (shipped from 256 MiB); 2, 3: the same, SWAP
extern "C" unsigned tl_grid(int shape, size_t n) {
  const size_t tiles = (n / 2 + 1023) / 1024;   // 512 x 2 and 1024 x 1: 1024 vectors per block either way
  return (unsigned)(shape == 2 || shape == 3 ? (tiles + 15) / 16 * 16 : tiles);   // swapped shapes permute within 16
}

extern "C" int tl_launch(int shape, double* d, const double* s, size_t n, unsigned long long* ts, void* stream,
                         void* e0, void* e1) {
  if (n % 2) return -1;
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  const size_t nvec = n / 2;
  const unsigned grid = tl_grid(shape, n);
  if (shape == 0)
    hipExtLaunchKernelGGL((k_reduce_tl<512, 2, false>), dim3(grid), dim3(512), 0, st, a, b, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, ts);
  else if (shape == 1)
    hipExtLaunchKernelGGL((k_reduce_tl<1024, 1, false>), dim3(grid), dim3(1024), 0, st, a, b, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, ts);
  else if (shape == 2)
    hipExtLaunchKernelGGL((k_reduce_tl<512, 2, true>), dim3(grid), dim3(512), 0, st, a, b, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, ts);
  else if (shape == 3)
    hipExtLaunchKernelGGL((k_reduce_tl<1024, 1, true>), dim3(grid), dim3(1024), 0, st, a, b, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, ts);
  else if (shape == 4)   // 1024 x 1, loads only
    hipExtLaunchKernelGGL((k_reduce_tl<1024, 1, false, 1>), dim3(grid), dim3(1024), 0, st, a, b, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, ts);
  else if (shape == 5)   // 1024 x 1, stores only
    hipExtLaunchKernelGGL((k_reduce_tl<1024, 1, false, 2>), dim3(grid), dim3(1024), 0, st, a, b, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, ts);
  else
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
