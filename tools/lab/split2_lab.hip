// EXPERIMENTS ONLY (tools/lab/run_split2_lab.py): one reduce call cut into two
// halves launched on two streams, so that one half's drain can overlap the
// other half's ramp.  The call keeps stream semantics on stream A: B waits
// for a fork event recorded on A, and A waits for a join event recorded on B,
// both created beforehand.  Timed like the bench's kernel_us: HIP events on A
// bracketing `reps` back-to-back calls over rotating operand pairs.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int (*reduce_fn)(void* dst, const void* src, size_t n, int dt, int op, void* stream);

// mode 0: one launch on A.  mode 1: halves on A and B, fork/join per call.
// mode 2: both halves on A (what the cut alone costs).  mode 3: whole calls
// alternate between A and B, joined only at the end (independent calls; an
// upper bound on what overlapping neighbours can give, not a drop-in).
extern "C" int split2_run(void* fn, char* base, size_t pair_stride, int pairs, size_t n, int reps, int warm, int mode,
                          float* us_per_call) {
  reduce_fn reduce = (reduce_fn)fn;
  hipStream_t A, B;
  if (hipStreamCreateWithFlags(&A, hipStreamNonBlocking) != hipSuccess) return -1;
  if (hipStreamCreateWithFlags(&B, hipStreamNonBlocking) != hipSuccess) return -1;
  hipEvent_t t0, t1, fork, join;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  hipEventCreateWithFlags(&fork, hipEventDisableTiming);
  hipEventCreateWithFlags(&join, hipEventDisableTiming);
  const size_t h = (n / 2 + 2047) / 2048 * 2048;      // halves on a 16 KiB boundary
  int rc = 0, k = 0;
  for (int i = 0; i < warm + reps && !rc; ++i) {
    if (i == warm) {
      // the timed region starts with both streams idle and B held behind t0: a
      // stream that ran ahead through the warm-up must not start timed work early
      hipStreamSynchronize(A);
      hipStreamSynchronize(B);
      hipEventRecord(t0, A);
      hipStreamWaitEvent(B, t0, 0);
    }
    char* d = base + pair_stride * (size_t)(k++ % pairs);
    char* s = d + pair_stride / 2;
    switch (mode) {
      case 0: rc = reduce(d, s, n, 1, 0, A); break;
      case 1:
        hipEventRecord(fork, A);
        hipStreamWaitEvent(B, fork, 0);
        rc = reduce(d, s, h, 1, 0, A);
        if (!rc) rc = reduce(d + h * 8, s + h * 8, n - h, 1, 0, B);
        hipEventRecord(join, B);
        hipStreamWaitEvent(A, join, 0);
        break;
      case 2:
        rc = reduce(d, s, h, 1, 0, A);
        if (!rc) rc = reduce(d + h * 8, s + h * 8, n - h, 1, 0, A);
        break;
      default: rc = reduce(d, s, n, 1, 0, (i & 1) ? B : A);
    }
  }
  if (mode == 3) {
    hipEventRecord(join, B);
    hipStreamWaitEvent(A, join, 0);
  }
  hipEventRecord(t1, A);
  hipError_t e = hipStreamSynchronize(A);
  hipStreamSynchronize(B);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
  *us_per_call = ms * 1e3f / (float)reps;
  hipEventDestroy(t0); hipEventDestroy(t1); hipEventDestroy(fork); hipEventDestroy(join);
  hipStreamDestroy(A); hipStreamDestroy(B);
  return rc ? rc : (e == hipSuccess ? 0 : -2);
}
