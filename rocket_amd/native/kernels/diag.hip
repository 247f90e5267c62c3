// Diagnostic kernels (probes only, never on a training path).
//
// rk_spin: `blocks` workgroups of 64 threads that each stay resident for `us` microseconds
// (s_memrealtime, 100 MHz) while occupying one wave slot — a kernel of known duration and known
// footprint, used to tell whether two graph branches / streams actually run concurrently.
#include "rk_common.h"

#include <hip/hip_ext.h>

using rk::f32x4;

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

// rk_gap_write / rk_gap_stamp: the dispatch gap between two dependent kernels as a function of the
// bytes the first one wrote (kernel-boundary release cost).  The writer's blocks stamp their start
// and end into trace[block][0..1] and each writes `bytes_per_block` bytes (nt: nontemporal stores);
// the stamper's blocks stamp their start into trace[block][0].  All stamps: s_memrealtime, 100 MHz.
namespace {
__global__ void __launch_bounds__(256) gap_write_kernel(f32x4* __restrict__ buf, int64_t n4, int nt,
                                                        uint64_t* __restrict__ trace) {
  if (threadIdx.x == 0) trace[blockIdx.x * 2] = __builtin_amdgcn_s_memrealtime();
  f32x4* p = buf + (int64_t)blockIdx.x * n4;
  const f32x4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
  for (int64_t i = threadIdx.x; i < n4; i += 256) {
    if (nt) __builtin_nontemporal_store(v, p + i);
    else p[i] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) trace[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime();
}
__global__ void __launch_bounds__(64) gap_stamp_kernel(uint64_t* __restrict__ trace) {
  if (threadIdx.x == 0) trace[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}
// the same stamp from a LeNet-step-shaped workgroup: 1024 threads and `lds` bytes of dynamic LDS
__global__ void __launch_bounds__(1024) gap_stamp_big_kernel(uint64_t* __restrict__ trace) {
  extern __shared__ char dyn[];
  if (threadIdx.x == 0) {
    trace[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    dyn[0] = 0;
  }
}
}  // namespace

RK_API int rk_gap_write(void* buf, int64_t bytes_per_block, int blocks, int nt, void* trace, hipStream_t s) {
  if (blocks < 1 || bytes_per_block < 0 || (bytes_per_block & 15) || ((uintptr_t)buf & 15)) return (int)hipErrorInvalidValue;
  gap_write_kernel<<<blocks, 256, 0, s>>>((f32x4*)buf, bytes_per_block / 16, nt, (uint64_t*)trace);
  return (int)hipGetLastError();
}

// any_order: launched with hipExtAnyOrderLaunch (AQL barrier bit clear: may start before the
// previous packet on the stream completes)
RK_API int rk_gap_stamp_big(int blocks, void* trace, int lds, hipStream_t s) {
  if (blocks < 1 || lds < 0 || lds > 160 * 1024) return (int)hipErrorInvalidValue;
  if (lds > 64 * 1024) hipFuncSetAttribute((const void*)gap_stamp_big_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  gap_stamp_big_kernel<<<blocks, 1024, lds, s>>>((uint64_t*)trace);
  return (int)hipGetLastError();
}

RK_API int rk_gap_stamp(int blocks, void* trace, int any_order, hipStream_t s) {
  if (blocks < 1) return (int)hipErrorInvalidValue;
  if (!any_order) {
    gap_stamp_kernel<<<blocks, 64, 0, s>>>((uint64_t*)trace);
    return (int)hipGetLastError();
  }
  void* args[] = {&trace};
  return (int)hipExtLaunchKernel((const void*)gap_stamp_kernel, dim3(blocks), dim3(64), args, 0, s, nullptr, nullptr,
                                 hipExtAnyOrderLaunch);
}
