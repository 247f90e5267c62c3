// Device-side pieces of the fused optimizers shared by optim.hip (the multi-tensor update launch)
// and gradient-producing kernels that apply the update in their epilogue (mlp.hip: the LeNet
// weight-gradient launch on a single-replica sync step, see AdamEpi).
#pragma once
#include "rk_common.h"

namespace rk_opt {

using rk::f2bf;
using rk::f2h;

struct TensorRec {  // 8 x int64: a parameter tensor as the update kernels see it
  int64_t p, g, s0, s1, n, group;
  int64_t shadow_map, shadow_buf;  // int32 [n][2] (or 1 = dense bf16, 2 = dense fp16) / buffer, or 0
};

constexpr int64_t kDenseShadow = 1;     // buffer laid out like p, bf16
constexpr int64_t kDenseShadowF16 = 2;  // buffer laid out like p, fp16 (fp16 autocast compute copies)
// index-mapped shadows: the map pointer (16-byte aligned) with bit 0 set = the buffer is fp16
// (e.g. the fused LeNet's fp16 fragment table), clear = bf16
__device__ __forceinline__ const int2* shadow_map_ptr(int64_t m) { return (const int2*)(m & ~(int64_t)1); }
__device__ __forceinline__ uint16_t shadow_cvt(int64_t m, float v) { return (m & 1) ? f2h(v) : f2bf(v); }

struct AdamHyper {  // 8 floats per group
  float lr, beta1, beta2, eps, wd, decoupled, maximize, pad;
};

__device__ __forceinline__ void shadow_store(const TensorRec& tr, int64_t i, float v) {
  uint16_t* buf = (uint16_t*)tr.shadow_buf;
  if (tr.shadow_map == kDenseShadowF16) {
    buf[i] = f2h(v);
    return;
  }
  if (tr.shadow_map == kDenseShadow) {
    buf[i] = f2bf(v);
    return;
  }
  const uint16_t b = shadow_cvt(tr.shadow_map, v);
  const int2 m = shadow_map_ptr(tr.shadow_map)[i];
  if (m.x >= 0) buf[m.x] = b;
  if (m.y >= 0) buf[m.y] = b;
}

// Device step counter: every block reads it first thing; each block takes a ticket at its END
// (the atomic's round trip then overlaps nothing on the block's critical path) and the last one
// advances the counter — every block has read the old value by then.
__device__ __forceinline__ float read_step(const float* step) {
  __shared__ float s_step;
  if (threadIdx.x == 0) s_step = step[0];
  __syncthreads();
  return s_step;
}

// Device-resident dynamic loss scaling (fp16 AMP; torch.amp.GradScaler semantics):
//   amp[0] scale, amp[1] 1/scale, amp[2] found_inf (set by rk_amp_check, consumed + cleared here),
//   amp[3] growth tracker, amp[4] growth factor, amp[5] backoff factor, amp[6] growth interval,
//   amp[7] found_inf of the last step, amp[8] number of updates so far (uint32 bits),
//   amp[10..11] 0 or the device address of a host-mapped int32 ring[kAmpRing]: update number n
//   publishes (n << 1) | found_inf into ring[n % kAmpRing] (one 4-byte store, so the host reads a
//   step's skip flag with a plain load: no copy, no event on the stream).
enum AmpSlot { kAmpScale = 0, kAmpInv, kAmpFound, kAmpTracker, kAmpGrowth, kAmpBackoff, kAmpInterval, kAmpLast,
               kAmpSeq, kAmpHost = 10, kAmpSlots = 12 };
constexpr int kAmpRing = 64;

// torch._amp_update_scale_, executed by the optimizer launch's last block
__device__ __forceinline__ void amp_update(float* amp) {
  const float found = amp[kAmpFound];
  float scale = amp[kAmpScale];
  if (found != 0.f) {
    scale *= amp[kAmpBackoff];
    amp[kAmpTracker] = 0.f;
  } else {
    const float ok = amp[kAmpTracker] + 1.f;
    if (ok >= amp[kAmpInterval]) {
      const float grown = scale * amp[kAmpGrowth];
      if (__builtin_isfinite(grown)) scale = grown;
      amp[kAmpTracker] = 0.f;
    } else {
      amp[kAmpTracker] = ok;
    }
  }
  amp[kAmpScale] = scale;
  amp[kAmpInv] = 1.f / scale;
  amp[kAmpLast] = found;
  amp[kAmpFound] = 0.f;  // every block has read it: each took its ticket after its first read
  const uint32_t seq = __float_as_uint(amp[kAmpSeq]) + 1u;
  amp[kAmpSeq] = __uint_as_float(seq);
  const uint64_t ring = *reinterpret_cast<const uint64_t*>(amp + kAmpHost);
  if (ring) {  // system-scope (write-through) vector store into host memory
    int* e = reinterpret_cast<int*>(ring) + (seq % kAmpRing);
    __hip_atomic_store(e, (int)((seq << 1) | (found != 0.f ? 1u : 0u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ void advance_step(float* step, unsigned* counter, bool skip, float cur,
                                             float* amp = nullptr) {
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      if (!skip) step[0] = cur + 1.f;
      if (amp) amp_update(amp);
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Per-group constants of one Adam/AdamW step t (1-based), as the multi-tensor kernel computes them.
struct AdamStep {
  float b1, b2, eps, step_size, rbc2, decay, l2, sgn;
};
// Bias corrections as 1 - beta^t = -expm1(t * log1p(beta - 1)): beta - 1 is exact in f32, and at
// beta2 = 0.999, t = 1 the direct 1 - powf(beta, t) cancels away ~3 digits of a fast pow's error
// (the update then drifts ~1e-3 relative from torch's double-precision bias corrections).
__device__ __forceinline__ float bias_correction(float beta, float t) {
  return -expm1f(t * log1pf(beta - 1.f));
}
__device__ __forceinline__ AdamStep adam_step(const AdamHyper& h, float t) {
  const float bc1 = bias_correction(h.beta1, t);
  const float bc2 = bias_correction(h.beta2, t);
  AdamStep k;
  k.b1 = h.beta1;
  k.b2 = h.beta2;
  k.eps = h.eps;
  k.step_size = h.lr / bc1;
  k.rbc2 = rsqrtf(bc2);
  k.decay = h.decoupled != 0.f ? 1.f - h.lr * h.wd : 1.f;
  k.l2 = h.decoupled != 0.f ? 0.f : h.wd;
  k.sgn = h.maximize != 0.f ? -1.f : 1.f;
  return k;
}
// one element: gg = raw gradient * gs.  Every multiply-add is an explicit fmaf and no plain
// multiply feeds an add: the result cannot depend on how the compiler contracts it in a given
// kernel, so the multi-tensor launch and a producer's epilogue update bitwise alike.
__device__ __forceinline__ void adam_update(const AdamStep& k, float& pp, float gg, float& mm, float& vv) {
  gg = __builtin_fmaf(k.l2, pp, k.sgn * gg);
  mm = __builtin_fmaf(k.b1, mm, (1.f - k.b1) * gg);
  const float g2 = gg * gg;
  vv = __builtin_fmaf(k.b2, vv, (1.f - k.b2) * g2);
  const float den = __builtin_fmaf(sqrtf(vv), k.rbc2, k.eps);
  const float upd = k.step_size * mm;
  pp = __builtin_fmaf(pp, k.decay, -(upd / den));
}

// Epilogue fusion: the producer of a parameter's FINAL gradient element (single replica, sync
// step, no AMP scaler — the host only arms it then) applies the Adam/AdamW update to it directly:
// p/m/v/shadow written, the gradient cleared (zero_grads) or stored.  The producer launch takes
// over the optimizer launch of that step, including the device step counter.
struct AdamEpi {
  const AdamHyper* hyper;
  float* step;
  unsigned* counter;
  int on;  // 0 = off, else the number of param groups (hyper rows)
  int zero_grads;
};
struct EpiElem {  // an element's operands, fetched before its gradient is known
  float p, m, v;
  int2 map;
};
__device__ __forceinline__ EpiElem epi_fetch(const TensorRec& tr, int64_t i) {
  EpiElem e;
  e.p = ((const float*)tr.p)[i];
  e.m = ((const float*)tr.s0)[i];
  e.v = ((const float*)tr.s1)[i];
  e.map = tr.shadow_map > kDenseShadowF16 ? shadow_map_ptr(tr.shadow_map)[i] : make_int2(-1, -1);
  return e;
}
__device__ __forceinline__ void epi_apply(const TensorRec& tr, const AdamStep& k, int64_t i, EpiElem e, float g,
                                          int zero_grads) {
  adam_update(k, e.p, g, e.m, e.v);
  ((float*)tr.p)[i] = e.p;
  ((float*)tr.s0)[i] = e.m;
  ((float*)tr.s1)[i] = e.v;
  ((float*)tr.g)[i] = zero_grads ? 0.f : g;
  if (tr.shadow_map == kDenseShadow) {
    ((uint16_t*)tr.shadow_buf)[i] = f2bf(e.p);
  } else if (tr.shadow_map == kDenseShadowF16) {
    ((uint16_t*)tr.shadow_buf)[i] = f2h(e.p);
  } else if (tr.shadow_map) {
    const uint16_t b = shadow_cvt(tr.shadow_map, e.p);
    if (e.map.x >= 0) ((uint16_t*)tr.shadow_buf)[e.map.x] = b;
    if (e.map.y >= 0) ((uint16_t*)tr.shadow_buf)[e.map.y] = b;
  }
}

}  // namespace rk_opt
