// EXPERIMENTS ONLY (tools/lab/run_edge_lab.py --lab wait): does holding a
// wave until its stores are acknowledged change the reduce's rate?  The
// timeline build (timeline_lab.hip), whose waves wait for their loads, then
// for their stores' acknowledgement and a block barrier, ran 4% faster than
// the shipped kernel at 64 MiB on the same box.  Each variant below adds one
// of those waits to the shipped body (nt loads, nt stores, 16-B vectors):
//   order   : loads interleaved dst/src per vector (as shipped)
//   split   : every load waited for (vmcnt 0) before the first store
//   ack     : vmcnt 0 after the stores -- the wave ends only when the L2 has
//             acknowledged them, so its slot is not refilled earlier
//   barrier : ack, then a block barrier (the whole block leaves together)
// Same exported API as edge_lab.hip.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));

enum { SPLIT = 1, ACK = 2, BAR = 4 };

template <int B, int U, int F>
__global__ __launch_bounds__(B) void k_reduce_w(f64x2* __restrict__ d, const f64x2* __restrict__ s, size_t nvec) {
  const size_t i = (size_t)blockIdx.x * B * U + threadIdx.x;
  f64x2 x[U], y[U];
  if ((size_t)(blockIdx.x + 1) * B * U <= nvec) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = __builtin_nontemporal_load(d + i + u * B);
      y[u] = __builtin_nontemporal_load(s + i + u * B);
    }
    if (F & SPLIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + y[u], d + i + u * B);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * B < nvec) __builtin_nontemporal_store(__builtin_nontemporal_load(d + i + u * B) +
                                                        __builtin_nontemporal_load(s + i + u * B), d + i + u * B);
  }
  if (F & ACK) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (F & BAR) __syncthreads();
}

struct V {
  const char* name;
  int block, unroll, flags;
};
static const V kV[] = {
    {"reduce 512x2 order", 512, 2, 0},           {"reduce 512x2 split", 512, 2, SPLIT},
    {"reduce 512x2 ack", 512, 2, ACK},           {"reduce 512x2 split ack", 512, 2, SPLIT | ACK},
    {"reduce 512x2 split ack barrier", 512, 2, SPLIT | ACK | BAR},
    {"reduce 1024x1 order", 1024, 1, 0},         {"reduce 1024x1 ack", 1024, 1, ACK},
    {"reduce 1024x1 ack barrier", 1024, 1, ACK | BAR},
    {"reduce 256x4 order", 256, 4, 0},           {"reduce 256x4 split ack", 256, 4, SPLIT | ACK},
    {"reduce 256x2 split ack", 256, 2, SPLIT | ACK},
};

template <int B, int U, int F>
static void go(double* d, const double* s, size_t n, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  size_t nvec = n / 2;
  unsigned grid = (unsigned)((nvec + (size_t)B * U - 1) / ((size_t)B * U));
  hipExtLaunchKernelGGL((k_reduce_w<B, U, F>), dim3(grid), dim3(B), 0, st, e0, e1, 0, (f64x2*)d, (const f64x2*)s,
                        nvec);
}

extern "C" const char* edge_name(int v) { return v >= 0 && v < (int)(sizeof(kV) / sizeof(kV[0])) ? kV[v].name : nullptr; }

#define CASE(B, U, F) \
  if (x.block == B && x.unroll == U && x.flags == (F)) { go<B, U, F>(d, s, n, st, a, b); return hipGetLastError() == hipSuccess ? 0 : -2; }

extern "C" int edge_launch(int v, double* d, const double* s, size_t n, void* stream, void* e0, void* e1) {
  if (!edge_name(v)) return -1;
  const V& x = kV[v];
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t a = (hipEvent_t)e0, b = (hipEvent_t)e1;
  CASE(512, 2, 0) CASE(512, 2, SPLIT) CASE(512, 2, ACK) CASE(512, 2, SPLIT | ACK) CASE(512, 2, SPLIT | ACK | BAR)
  CASE(1024, 1, 0) CASE(1024, 1, ACK) CASE(1024, 1, ACK | BAR)
  CASE(256, 4, 0) CASE(256, 4, SPLIT | ACK) CASE(256, 2, SPLIT | ACK)
  return -1;
}
