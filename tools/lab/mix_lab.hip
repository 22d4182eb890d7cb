// EXPERIMENTS ONLY (tools/lab/run_mix_lab.py): how does the streaming rate
// depend on the read:write mix, apart from the number of read streams?  One
// tile shape (512 threads x one 16-B vector per stream, one-shot grid, nt
// loads and stores, as the shipped fold); every tile reads R source streams
// and sums them; only every M-th GROUP of eight consecutive tiles stores its
// sums (M = 0: none does; the sum is then kept alive by a store behind a
// condition no input meets).  Groups of eight, because block b runs on XCD
// b mod 8: "every M-th tile" would put all the stores on one or two XCDs.  The
// stored tiles are packed, group g landing at group position g / M, so the
// output is one dense stream 1/M as long as a source (in place they would be a
// strided write that loads some memory channels and leaves others idle).
// Traffic per launch = R x size + size / M.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
struct Src8 { const f64x2* p[8]; };

template <int R, int B>
__global__ __launch_bounds__(B) void k_mix(f64x2* __restrict__ out, Src8 s, size_t nvec, unsigned every) {
  const size_t i = (size_t)blockIdx.x * B + threadIdx.x;
  if (i >= nvec) return;
  f64x2 x[R];
#pragma unroll
  for (int j = 0; j < R; ++j) x[j] = __builtin_nontemporal_load(s.p[j] + i);
  f64x2 acc = x[0];
#pragma unroll
  for (int j = 1; j < R; ++j) acc += x[j];
  const unsigned group = blockIdx.x >> 3;
  const bool store = every ? (group % every == 0) : (acc.x == 1.2345e300);
  const size_t tile = every ? (size_t)(group / every) * 8 + (blockIdx.x & 7) : 0;
  if (store) __builtin_nontemporal_store(acc, out + tile * B + threadIdx.x);
}

template <int R>
static int go(f64x2* out, Src8 s, size_t nvec, unsigned every, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  constexpr int B = 512;
  const unsigned grid = (unsigned)((nvec + B - 1) / B);
  hipExtLaunchKernelGGL((k_mix<R, B>), dim3(grid), dim3(B), 0, st, a, b, 0, out, s, nvec, every);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int mix_launch(int nread, int every, double* out, const double* const* srcs, size_t n, void* stream,
                          void* e0, void* e1) {
  if (nread < 1 || nread > 8 || every < 0 || (n & 1)) return -1;
  Src8 s;
  for (int j = 0; j < 8; ++j) s.p[j] = (const f64x2*)srcs[j < nread ? j : 0];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  f64x2* o = (f64x2*)out;
  const size_t nvec = n / 2;
  switch (nread) {
    case 1: return go<1>(o, s, nvec, (unsigned)every, st, a, b);
    case 2: return go<2>(o, s, nvec, (unsigned)every, st, a, b);
    case 3: return go<3>(o, s, nvec, (unsigned)every, st, a, b);
    case 4: return go<4>(o, s, nvec, (unsigned)every, st, a, b);
    case 6: return go<6>(o, s, nvec, (unsigned)every, st, a, b);
    case 8: return go<8>(o, s, nvec, (unsigned)every, st, a, b);
    default: return -1;
  }
}
