// EXPERIMENTS ONLY (tools/lab/run_burst_lab.py): the mix lab shows that a thin
// stream of writes spread evenly through many read streams costs several
// times more per byte than the same bytes written densely.  Can the 8-source
// fold make its writes dense in TIME?  A resident grid; every wave folds U
// tiles into registers (reads only), then stores its U results in one go.  All
// waves start together and do equal work, so their store bursts coincide at
// first; optionally the bursts are re-aligned to the GPU's constant 100 MHz
// clock (s_memrealtime): a wave that is ready before the period's write window
// opens sleeps until it does (bounded: it goes ahead after `max_spins` looks).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
struct Src8 { const f64x2* p[8]; };

template <int R, int U, int B>
__global__ __launch_bounds__(B) void k_burst(f64x2* __restrict__ out, Src8 s, size_t nvec, unsigned period,
                                             unsigned read_ticks, int max_spins) {
  const size_t chunk = (size_t)B * U;
  const size_t stride = (size_t)gridDim.x * chunk;
  for (size_t base = (size_t)blockIdx.x * chunk; base < nvec; base += stride) {
    f64x2 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * B + threadIdx.x;
      if (i < nvec) {
        f64x2 x[R];
#pragma unroll
        for (int j = 0; j < R; ++j) x[j] = __builtin_nontemporal_load(s.p[j] + i);
        f64x2 acc = x[0];
#pragma unroll
        for (int j = 1; j < R; ++j) acc += x[j];
        r[u] = acc;
      }
    }
    if (period) {
      for (int spin = 0; spin < max_spins; ++spin) {
        const unsigned pos = (unsigned)(__builtin_amdgcn_s_memrealtime() % period);
        if (pos >= read_ticks) break;
        __builtin_amdgcn_s_sleep(16);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * B + threadIdx.x;
      if (i < nvec) __builtin_nontemporal_store(r[u], out + i);
    }
  }
}

template <int R, int U, int B>
static int go(f64x2* out, Src8 s, size_t nvec, int blocks_per_cu, unsigned period, unsigned read_ticks, int max_spins,
              hipStream_t st, hipEvent_t a, hipEvent_t b) {
  const size_t chunk = (size_t)B * U;
  size_t need = (nvec + chunk - 1) / chunk;
  unsigned grid = 256u * (unsigned)blocks_per_cu;
  if (grid > need) grid = (unsigned)need;
  hipExtLaunchKernelGGL((k_burst<R, U, B>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec, period, read_ticks,
                        max_spins);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int R>
static int pick(int unroll, int block, f64x2* o, Src8 s, size_t nvec, int blocks_per_cu, unsigned period,
                unsigned read_ticks, int max_spins, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  switch (block * 64 + unroll) {
    case 256 * 64 + 2: return go<R, 2, 256>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 256 * 64 + 4: return go<R, 4, 256>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 256 * 64 + 8: return go<R, 8, 256>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 256 * 64 + 16: return go<R, 16, 256>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 256 * 64 + 24: return go<R, 24, 256>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 256 * 64 + 32: return go<R, 32, 256>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 512 * 64 + 8: return go<R, 8, 512>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 512 * 64 + 16: return go<R, 16, 512>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 128 * 64 + 32: return go<R, 32, 128>(o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    default: return -1;
  }
}

// nread = 2 .. 8 sources; out may be srcs[j] (every lane reads its elements of every source before it writes them)
extern "C" int burst_launch_k(int nread, int unroll, int block, int blocks_per_cu, unsigned period,
                              unsigned read_ticks, int max_spins, double* out, const double* const* srcs, size_t n,
                              void* stream, void* e0, void* e1) {
  if ((n & 1) || blocks_per_cu < 1 || blocks_per_cu > 16 || max_spins < 0 || max_spins > 100000) return -1;
  if (period && read_ticks >= period) return -1;
  if (nread < 2 || nread > 8) return -1;
  Src8 s;
  for (int j = 0; j < 8; ++j) s.p[j] = (const f64x2*)srcs[j < nread ? j : 0];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  f64x2* o = (f64x2*)out;
  const size_t nvec = n / 2;
  switch (nread) {
    case 2: return pick<2>(unroll, block, o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 3: return pick<3>(unroll, block, o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 4: return pick<4>(unroll, block, o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 5: return pick<5>(unroll, block, o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 6: return pick<6>(unroll, block, o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 7: return pick<7>(unroll, block, o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    case 8: return pick<8>(unroll, block, o, s, nvec, blocks_per_cu, period, read_ticks, max_spins, st, a, b);
    default: return -1;
  }
}

extern "C" int burst_launch(int unroll, int block, int blocks_per_cu, unsigned period, unsigned read_ticks,
                            int max_spins, double* out, const double* const* srcs, size_t n, void* stream, void* e0,
                            void* e1) {
  return burst_launch_k(8, unroll, block, blocks_per_cu, period, read_ticks, max_spins, out, srcs, n, stream, e0, e1);
}

// The same kernel (8 sources, 256 lanes) with its burst of stores issued as
// buffer stores carrying the cache-policy bits AUX (gfx950: sc0 = 1, nt = 2,
// sc1 = 16; 0 = plain): does the policy of a DENSE run of stores matter?
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int U, int AUX>
__global__ __launch_bounds__(256) void k_burst_pol(f64x2* __restrict__ out, Src8 s, size_t nvec) {
  constexpr int B = 256;
  const size_t tile0 = (size_t)blockIdx.x * B * U;
  if (tile0 >= nvec) return;
  f64x2 r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = tile0 + (size_t)u * B + threadIdx.x;
    if (i < nvec) {
      f64x2 x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = __builtin_nontemporal_load(s.p[j] + i);
      f64x2 acc = x[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) acc += x[j];
      r[u] = acc;
    }
  }
  asm volatile("" ::: "memory");
  const size_t left = nvec - tile0;
  const uint32_t bytes = (uint32_t)((left < (size_t)B * U ? left : (size_t)B * U) * sizeof(f64x2));
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + tile0, (short)0, (int)bytes, 0x00020000);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = tile0 + (size_t)u * B + threadIdx.x;
    if (i < nvec)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, r[u]), rs,
                                             (int)((threadIdx.x + u * B) * sizeof(f64x2)), 0, AUX);
  }
}

template <int U, int AUX>
static int go_pol(f64x2* o, Src8 s, size_t nvec, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  const unsigned grid = (unsigned)((nvec + 256 * (size_t)U - 1) / (256 * (size_t)U));
  hipExtLaunchKernelGGL((k_burst_pol<U, AUX>), dim3(grid), dim3(256), 0, st, a, b, 0, o, s, nvec);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int burst_policy_launch(int unroll, int aux, double* out, const double* const* srcs, size_t n, void* stream,
                                   void* e0, void* e1) {
  if (n & 1) return -1;
  Src8 s;
  for (int j = 0; j < 8; ++j) s.p[j] = (const f64x2*)srcs[j];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  f64x2* o = (f64x2*)out;
  const size_t nvec = n / 2;
  switch (unroll * 100 + aux) {
    case 3200: return go_pol<32, 0>(o, s, nvec, st, a, b);
    case 3202: return go_pol<32, 2>(o, s, nvec, st, a, b);
    case 3216: return go_pol<32, 16>(o, s, nvec, st, a, b);
    case 3218: return go_pol<32, 18>(o, s, nvec, st, a, b);
    case 3201: return go_pol<32, 1>(o, s, nvec, st, a, b);
    case 1600: return go_pol<16, 0>(o, s, nvec, st, a, b);
    case 1602: return go_pol<16, 2>(o, s, nvec, st, a, b);
    case 1616: return go_pol<16, 16>(o, s, nvec, st, a, b);
    default: return -1;
  }
}
