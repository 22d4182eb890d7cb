// EXPERIMENTS ONLY (tools/lab/run_edge_lab.py --lab lock): keep the eight
// XCDs in step through one launch.  The spread lab (r02_spread_lab.txt) shows
// that tiles in flight spread over 16 MiB of each operand cost 7% at 256 MiB,
// and the timeline lab shows the XCDs drifting that far apart over a long
// launch (the odd ones stream ~4% slower).  Here every block (1024 x 1, one
// 16 KiB tile, block b on XCD slot b mod 8) issues its loads, then lane 0
// reads the eight slots' completed-block counters (agent-scope atomic loads,
// in flight beside the tile loads) and holds the block -- and so its CU slot
// -- while its slot has completed more than `slack` blocks beyond the slowest
// unfinished slot.  The slowest slot never waits, so the launch always
// progresses; a cap on the polls bounds any wait anyway.  The block then
// stores and adds 1 to its slot's counter.  The counters are cleared before
// each launch (outside the stamps).  Same API as edge_lab.hip.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

constexpr int kB = 1024;
constexpr int kLine = 32;            // one 128-B line per counter

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool THROTTLE>
__global__ __launch_bounds__(kB) void k_lock(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec,
                                             unsigned* ctr, unsigned slack, unsigned grid, unsigned period) {
  const unsigned x = blockIdx.x & 7;
  // only every period-th block of a slot polls and counts (adding `period`):
  // the counters see 1/period of the blocks' traffic
  const bool pacer = ((blockIdx.x >> 3) % period) == 0;
  const size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  f64x2 a = {0, 0}, b = {0, 0};
  if (i < nvec) {
    a = __builtin_nontemporal_load(d + i);
    b = __builtin_nontemporal_load(s + i);
  }
  if (THROTTLE && pacer) {
    if (threadIdx.x < 64) {            // wave 0: lane j < 8 reads slot j's counter
      const unsigned lane = threadIdx.x;
      for (int polls = 0; polls < 4096; ++polls) {
        unsigned c = 0, fin = 1;
        if (lane < 8) {
          c = ld_agent(ctr + lane * kLine);
          fin = c + period > (grid - lane + 7) / 8;      // slot `lane` has (about) completed all its blocks
        }
        // min over unfinished slots of the completed count; mine from lane x
        unsigned m = fin ? 0xFFFFFFFFu : c;
        for (int off = 1; off < 8; off <<= 1) {
          unsigned o = __shfl_xor(m, off, 64);
          m = o < m ? o : m;
        }
        const unsigned mine = __shfl(c, (int)x, 64);
        if (m == 0xFFFFFFFFu || mine <= m + slack) break;
        __builtin_amdgcn_s_sleep(8);
      }
    }
    __syncthreads();
  }
  if (i < nvec) __builtin_nontemporal_store(a + b, d + i);
  if (THROTTLE && pacer) {
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr + x * kLine, period, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct V {
  const char* name;
  int slack;        // < 0: no throttle (plain 1024 x 1, same grid)
  int period;
};
static const V kV[] = {{"reduce lock 1024x1 off", -1, 1},           {"reduce lock 1024x1 slack32 p16", 32, 16},
                       {"reduce lock 1024x1 slack128 p16", 128, 16}, {"reduce lock 1024x1 slack32 p64", 32, 64},
                       {"reduce lock 1024x1 slack128 p64", 128, 64}, {"reduce lock 1024x1 slack4096 p64", 4096, 64},
                       {"reduce lock 1024x1 slack64 p32", 64, 32}};
static unsigned* g_ctr = nullptr;

extern "C" const char* edge_name(int v) { return v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0])) ? kV[v].name : nullptr; }

extern "C" int edge_launch(int v, double* d, const double* s, size_t n, void* stream, void* e0, void* e1) {
  if (!edge_name(v) || n % 2) return -1;
  if (!g_ctr && hipMalloc(&g_ctr, 8 * kLine * sizeof(unsigned)) != hipSuccess) return -3;
  hipStream_t st = (hipStream_t)stream;
  const size_t nvec = n / 2;
  const unsigned grid = (unsigned)((nvec + kB - 1) / kB);
  if (kV[v].slack < 0) {
    hipExtLaunchKernelGGL(k_lock<false>, dim3(grid), dim3(kB), 0, st, (hipEvent_t)e0, (hipEvent_t)e1, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, g_ctr, 0u, grid, 1u);
  } else {
    if (hipMemsetAsync(g_ctr, 0, 8 * kLine * sizeof(unsigned), st) != hipSuccess) return -3;
    hipExtLaunchKernelGGL(k_lock<true>, dim3(grid), dim3(kB), 0, st, (hipEvent_t)e0, (hipEvent_t)e1, 0, (f64x2*)d,
                          (const f64x2*)s, nvec, g_ctr, (unsigned)kV[v].slack, grid, (unsigned)kV[v].period);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
