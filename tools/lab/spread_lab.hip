// EXPERIMENTS ONLY (tools/lab/run_edge_lab.py --lab spread): does it cost
// bandwidth when the XCDs work far apart in the buffer?  Over a long launch
// the eight XCDs drift apart (the odd ones stream ~4% slower), and the rate
// decays while they do (profiles/r02_timeline_long.txt).  Here the drift is
// put in on purpose from the first block: XCD x (block b runs on XCD b mod 8)
// starts its walk through its tiles x * delta tiles-of-its-own later, and
// wraps, so the tiles in flight at one moment are spread over about S MiB of
// each operand from the start.  Every tile is still reduced exactly once.
// Same API as edge_lab.hip.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

constexpr int kB = 1024;    // 1024 x 1: one 16-B vector per operand per thread, 16 KiB tiles

__global__ __launch_bounds__(kB) void k_rot(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec,
                                            size_t per, size_t delta) {
  const size_t x = blockIdx.x & 7, k = blockIdx.x >> 3;
  const size_t t = ((k + x * delta) % per) * 8 + x;
  const size_t i = t * kB + threadIdx.x;
  if (i < nvec) {
    f64x2 a = __builtin_nontemporal_load(d + i);
    f64x2 b = __builtin_nontemporal_load(s + i);
    __builtin_nontemporal_store(a + b, d + i);
  }
}

struct V {
  const char* name;
  int spread_mib;   // 0: no offset (the shipped dealing)
};
static const V kV[] = {{"reduce rot 1024x1 S0", 0},   {"reduce rot 1024x1 S4", 4},    {"reduce rot 1024x1 S16", 16},
                       {"reduce rot 1024x1 S48", 48}, {"reduce rot 1024x1 S96", 96},  {"reduce rot 1024x1 S192", 192}};

extern "C" const char* edge_name(int v) { return v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0])) ? kV[v].name : nullptr; }

// n doubles per operand; needs a multiple of 8 tiles (8 x 2048 doubles)
extern "C" int edge_launch(int v, double* d, const double* s, size_t n, void* stream, void* e0, void* e1) {
  if (!edge_name(v) || n % (8 * 2048)) return -1;
  const size_t nvec = n / 2, tiles = nvec / kB, per = tiles / 8;
  // XCD x starts x * delta of its own tiles (8 tiles of 16 KiB apart in the buffer each) later: 7 * delta * 128 KiB = S
  const size_t delta = (size_t)kV[v].spread_mib * 1024 / (7 * 128);
  hipExtLaunchKernelGGL(k_rot, dim3((unsigned)tiles), dim3(kB), 0, (hipStream_t)stream, (hipEvent_t)e0, (hipEvent_t)e1,
                        0, (f64x2*)d, (const f64x2*)s, nvec, per, delta % per);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
