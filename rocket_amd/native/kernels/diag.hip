// Diagnostic kernels (probes only, never on a training path).
//
// rk_spin: `blocks` workgroups of 64 threads that each stay resident for `us` microseconds
// (s_memrealtime, 100 MHz) while occupying one wave slot — a kernel of known duration and known
// footprint, used to tell whether two graph branches / streams actually run concurrently.
#include "rk_common.h"

namespace {
__global__ void __launch_bounds__(64) spin_kernel(uint64_t ticks, float* sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  float acc = 0.f;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(2);
    acc += 1.f;
  }
  if (acc < 0.f) sink[threadIdx.x] = acc;  // never true: keeps the loop
}
}  // namespace

RK_API int rk_spin(double us, int blocks, float* sink, hipStream_t s) {
  if (blocks < 1 || us < 0) return (int)hipErrorInvalidValue;
  spin_kernel<<<blocks, 64, 0, s>>>((uint64_t)(us * 100.0), sink);
  return (int)hipGetLastError();
}
