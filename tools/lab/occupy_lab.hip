// EXPERIMENTS ONLY (tools/lab/burst_occupied_probe.py): a kernel that only
// occupies: `grid` workgroups of 256 lanes, 128 VGPRs per lane reserved, each
// wave sleeping until `ticks` of the GPU's constant 100 MHz clock have passed
// since it started (bounded: at most `max_spins` looks).  It stands in for
// another library's communication kernels sharing the GPU with a fold.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void k_occupy(unsigned ticks, int max_spins, unsigned* sink) {
  asm volatile("v_mov_b32 v127, 0" ::: "v127");        // the wave is allocated 128 VGPRs
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int spin = 0; spin < max_spins; ++spin) {
    if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(32);
  }
  if (ticks == 0xffffffffu) sink[threadIdx.x] = 1;     // never: keeps the kernel from being empty
}

extern "C" int occupy_launch(int grid, unsigned ticks, int max_spins, void* stream) {
  if (grid < 1 || grid > 1024 || max_spins < 0 || max_spins > 200000 || ticks > 1000000u) return -1;
  hipLaunchKernelGGL(k_occupy, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, ticks, max_spins,
                     (unsigned*)nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
