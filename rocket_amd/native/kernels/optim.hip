// Fused multi-tensor optimizers: AdamW / Adam and SGD(momentum, nesterov).
//
// One launch updates every parameter tensor of an optimizer: a device-resident
// tensor table (param/grad/state pointers, sizes, group id) and a block table
// (tensor, chunk) are built once on the host and re-uploaded only when a
// pointer changes, so the launch is graph-capturable.  Hyper-parameters live in
// a small device array per param group (lr, betas, eps, weight decay) that the
// host refreshes only when a scheduler changes them, and the step counter lives
// in device memory: every block reads it first, and the last block to take a ticket
// advances it, so bias corrections need no host round trip.
//
// Optional bf16 shadows: a tensor record may carry an index map (int32 [n][2], -1 = none) and a
// bf16 buffer; every updated element is also written, rounded to bf16, to buf[map[i][0]] and
// buf[map[i][1]] — or, with the map pointer 1 ("dense"), to buf[i] (a bf16 copy of the weights
// that GEMMs read directly instead of casting the fp32 master every forward; map pointer 2: the
// same as an fp16 copy, for fp16 autocast).  A kernel that consumes the weights as pre-arranged bf16 MFMA fragments (the
// fused LeNet's fragment table) then needs no per-step re-layout launch.
//
// Optional AMP (fp16 dynamic loss scaling, all on the device): rk_amp_check flags non-finite
// gradients; the update multiplies every gradient by 1/scale (GradScaler's unscale folded into the
// update), a set flag makes the launch a no-op, and its last block runs the scale update.
// `zero_grads` clears each gradient chunk after it is consumed (the
// optimizer.step(); optimizer.zero_grad() pair in one pass over the gradient).
//
// Memory: each block streams one chunk of J*1024 elements (J float4 per thread per array):
// params/grads/exp_avg/exp_avg_sq read once, written once.  J = 4 (4096-element chunks) for big
// models; J = 1 for small ones (LeNet's 61,706 parameters: 4x the blocks, one load round trip).
#include <cstring>

#include "optim_common.h"

using namespace rk;
using namespace rk_opt;

namespace {

constexpr int kChunk = 4096;  // largest chunk (J = 4)
constexpr int kThreads = 256;

// Index-mapped shadows: the 4 map entries of elements i..i+3 (two 16-byte loads), fetched together
// with the parameter data so the shadow stores do not wait on a dependent load after the update.
struct Map4 {
  int4 a, b;
};
__device__ __forceinline__ Map4 shadow_map4(const TensorRec& tr, int64_t i) {
  if (tr.shadow_map <= kDenseShadowF16) return Map4{};
  const int4* m = (const int4*)(shadow_map_ptr(tr.shadow_map) + i);
  return Map4{m[0], m[1]};
}
// four consecutive elements (i % 4 == 0, 16-byte aligned parameter rows): dense shadows take one
// 8-byte store, mapped ones use the prefetched map entries
__device__ __forceinline__ void shadow_store4(const TensorRec& tr, int64_t i, const float4& v, const Map4& mp) {
  uint16_t* buf = (uint16_t*)tr.shadow_buf;
  if (tr.shadow_map == kDenseShadow) {
    *(uint2*)(buf + i) = make_uint2((uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16),
                                    (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16));
    return;
  }
  if (tr.shadow_map == kDenseShadowF16) {
    *(uint2*)(buf + i) = make_uint2((uint32_t)f2h(v.x) | ((uint32_t)f2h(v.y) << 16),
                                    (uint32_t)f2h(v.z) | ((uint32_t)f2h(v.w) << 16));
    return;
  }
  const int idx[8] = {mp.a.x, mp.a.y, mp.a.z, mp.a.w, mp.b.x, mp.b.y, mp.b.z, mp.b.w};
  const float val[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint16_t b = shadow_cvt(tr.shadow_map, val[e]);
    if (idx[2 * e] >= 0) buf[idx[2 * e]] = b;
    if (idx[2 * e + 1] >= 0) buf[idx[2 * e + 1]] = b;
  }
}


template <typename G>
__device__ __forceinline__ float gload(const G* g, int64_t i);
template <> __device__ __forceinline__ float gload<float>(const float* g, int64_t i) { return g[i]; }
template <> __device__ __forceinline__ float gload<uint16_t>(const uint16_t* g, int64_t i) { return bf2f(g[i]); }

template <typename G>
__device__ __forceinline__ void zero_chunk(G* g, int64_t start, int64_t end) {
  for (int64_t i = start + threadIdx.x; i < end; i += kThreads) g[i] = G(0);
}

template <typename G, bool ZG, int J>
__global__ void __launch_bounds__(kThreads) adam_mt_kernel(const TensorRec* __restrict__ tensors,
                                                          const int2* __restrict__ blocks,
                                                          const AdamHyper* __restrict__ hyper, float* step,
                                                          float* amp, unsigned* counter) {
  // block record + chunk index + step counter loads all in flight at once (the tensor table holds
  // one record per BLOCK: no dependent table walk before the data loads)
  const int2 bt = blocks[blockIdx.x];
  const TensorRec tr = tensors[blockIdx.x];
  const bool skip = amp != nullptr && amp[kAmpFound] != 0.f;
  const float cur = read_step(step);
  const float t = cur + 1.f;
  if (!skip) {
    const AdamHyper h = hyper[tr.group];
    float* __restrict__ p = (float*)tr.p;
    G* __restrict__ g = (G*)tr.g;
    float* __restrict__ m = (float*)tr.s0;
    float* __restrict__ v = (float*)tr.s1;
    const AdamStep k = adam_step(h, t);
    const float gs = amp ? amp[kAmpInv] : 1.f;
    constexpr int CH = J * 4 * kThreads;
    const int64_t start = (int64_t)bt.y * CH;
    const int64_t end = min(start + (int64_t)CH, tr.n);
    auto upd = [&](float& pp, float gg, float& mm, float& vv) { adam_update(k, pp, gg * gs, mm, vv); };
    const bool vec = sizeof(G) == 4 && ((tr.p | tr.g | tr.s0 | tr.s1) & 15) == 0;
    if (vec && end - start == CH) {
      // full chunk: all 4*J float4 loads of the thread in flight before the first update
      float4 pp[J], mm[J], vv[J], gg[J];
      Map4 mp[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int64_t i = start + 4 * (threadIdx.x + j * kThreads);
        pp[j] = *(const float4*)(p + i);
        mm[j] = *(const float4*)(m + i);
        vv[j] = *(const float4*)(v + i);
        gg[j] = *(const float4*)((const float*)g + i);
        mp[j] = shadow_map4(tr, i);
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int64_t i = start + 4 * (threadIdx.x + j * kThreads);
        upd(pp[j].x, gg[j].x, mm[j].x, vv[j].x);
        upd(pp[j].y, gg[j].y, mm[j].y, vv[j].y);
        upd(pp[j].z, gg[j].z, mm[j].z, vv[j].z);
        upd(pp[j].w, gg[j].w, mm[j].w, vv[j].w);
        *(float4*)(p + i) = pp[j];
        *(float4*)(m + i) = mm[j];
        *(float4*)(v + i) = vv[j];
        if (ZG) *(float4*)((float*)g + i) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (tr.shadow_map) shadow_store4(tr, i, pp[j], mp[j]);
      }
    } else if (vec) {
      for (int64_t i = start + 4 * threadIdx.x; i < end; i += 4 * kThreads) {
        if (i + 4 <= end) {
          float4 pp = *(float4*)(p + i), mm = *(float4*)(m + i), vv = *(float4*)(v + i);
          float4 gg = *(const float4*)((const float*)g + i);
          const Map4 mp = shadow_map4(tr, i);
          upd(pp.x, gg.x, mm.x, vv.x);
          upd(pp.y, gg.y, mm.y, vv.y);
          upd(pp.z, gg.z, mm.z, vv.z);
          upd(pp.w, gg.w, mm.w, vv.w);
          *(float4*)(p + i) = pp;
          *(float4*)(m + i) = mm;
          *(float4*)(v + i) = vv;
          if (ZG) *(float4*)((float*)g + i) = make_float4(0.f, 0.f, 0.f, 0.f);
          if (tr.shadow_map) shadow_store4(tr, i, pp, mp);
        } else {
          for (int64_t k = i; k < end; ++k) {
            upd(p[k], gload<G>(g, k), m[k], v[k]);
            if (ZG) g[k] = G(0);
            if (tr.shadow_map) shadow_store(tr, k, p[k]);
          }
        }
      }
    } else {
      for (int64_t i = start + threadIdx.x; i < end; i += kThreads) {
        upd(p[i], gload<G>(g, i), m[i], v[i]);
        if (ZG) g[i] = G(0);
        if (tr.shadow_map) shadow_store(tr, i, p[i]);
      }
    }
  } else if (ZG) {
    constexpr int CH = J * 4 * kThreads;
    const int64_t start = (int64_t)bt.y * CH;
    zero_chunk<G>((G*)tr.g, start, min(start + (int64_t)CH, tr.n));
  }
  advance_step(step, counter, skip, cur, amp);
}

struct SgdHyper {  // 8 floats per group
  float lr, momentum, dampening, wd, nesterov, maximize, first, pad;
};

template <typename G, bool ZG, int J>
__global__ void __launch_bounds__(kThreads) sgd_mt_kernel(const TensorRec* __restrict__ tensors,
                                                         const int2* __restrict__ blocks,
                                                         const SgdHyper* __restrict__ hyper, float* step,
                                                         float* amp, unsigned* counter) {
  const int2 bt = blocks[blockIdx.x];
  const TensorRec tr = tensors[blockIdx.x];
  const bool skip = amp != nullptr && amp[kAmpFound] != 0.f;
  const float cur = read_step(step);
  if (!skip) {
    const SgdHyper h = hyper[tr.group];
    float* __restrict__ p = (float*)tr.p;
    G* __restrict__ g = (G*)tr.g;
    float* __restrict__ buf = (float*)tr.s0;
    const bool first = cur == 0.f;  // momentum buffer initialised with the first gradient (torch semantics)
    const float gs = amp ? amp[kAmpInv] : 1.f;
    const float sgn = h.maximize != 0.f ? -1.f : 1.f;
    constexpr int CH = J * 4 * kThreads;
    const int64_t start = (int64_t)bt.y * CH;
    const int64_t end = min(start + (int64_t)CH, tr.n);
    const bool mom = h.momentum != 0.f;
    auto upd = [&](float& pp, float gg, float& bb) {
      gg = gg * gs + h.wd * pp;
      if (mom) {
        bb = first ? gg : h.momentum * bb + (1.f - h.dampening) * gg;
        gg = h.nesterov != 0.f ? gg + h.momentum * bb : bb;
      }
      pp -= sgn * h.lr * gg;
    };
    const bool vec = sizeof(G) == 4 && ((tr.p | tr.g | (mom ? tr.s0 : 0)) & 15) == 0;
    if (vec && end - start == CH) {
      // full chunk: every float4 load of the thread in flight before the first update (the scalar
      // loop below keeps one element per thread in flight: ~half of HBM bandwidth on ResNet-18)
      float4 pp[J], gg[J], bb[J];
      Map4 mp[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int64_t i = start + 4 * (threadIdx.x + j * kThreads);
        pp[j] = *(const float4*)(p + i);
        gg[j] = *(const float4*)((const float*)g + i);
        bb[j] = (mom && !first) ? *(const float4*)(buf + i) : make_float4(0.f, 0.f, 0.f, 0.f);
        mp[j] = shadow_map4(tr, i);
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int64_t i = start + 4 * (threadIdx.x + j * kThreads);
        upd(pp[j].x, gg[j].x, bb[j].x);
        upd(pp[j].y, gg[j].y, bb[j].y);
        upd(pp[j].z, gg[j].z, bb[j].z);
        upd(pp[j].w, gg[j].w, bb[j].w);
        *(float4*)(p + i) = pp[j];
        if (mom) *(float4*)(buf + i) = bb[j];
        if (ZG) *(float4*)((float*)g + i) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (tr.shadow_map) shadow_store4(tr, i, pp[j], mp[j]);
      }
    } else {
      for (int64_t i = start + threadIdx.x; i < end; i += kThreads) {
        float pv = p[i], bv = (mom && !first) ? buf[i] : 0.f;
        upd(pv, gload<G>(g, i), bv);
        p[i] = pv;
        if (mom) buf[i] = bv;
        if (ZG) g[i] = G(0);
        if (tr.shadow_map) shadow_store(tr, i, pv);
      }
    }
  } else if (ZG) {
    constexpr int CH = J * 4 * kThreads;
    const int64_t start = (int64_t)bt.y * CH;
    zero_chunk<G>((G*)tr.g, start, min(start + (int64_t)CH, tr.n));
  }
  advance_step(step, counter, skip, cur, amp);
}

}  // namespace

// elements per block-table chunk for a parameter set of `total` elements (the host builds the
// block table with it and passes it back to rk_optim_mt)
RK_API int rk_optim_chunk_for(int64_t total) { return total <= (int64_t)(1 << 21) ? kChunk / 4 : kChunk; }
RK_API int rk_optim_chunk() { return kChunk; }

// Non-finite check of every gradient of the tables (fp16 AMP): any inf/NaN in a block's chunk sets
// amp[kAmpFound] (plain stores of the same value; the optimizer launch consumes and clears it).
template <typename G, int J>
__global__ void __launch_bounds__(kThreads) amp_check_kernel(const TensorRec* __restrict__ tensors,
                                                            const int2* __restrict__ blocks, float* amp) {
  const int2 bt = blocks[blockIdx.x];
  const TensorRec tr = tensors[blockIdx.x];
  constexpr int CH = J * 4 * kThreads;
  const int64_t start = (int64_t)bt.y * CH;
  const int64_t end = min(start + (int64_t)CH, tr.n);
  const G* g = (const G*)tr.g;
  bool bad = false;
  for (int64_t i = start + threadIdx.x; i < end; i += kThreads) bad |= !(fabsf(gload<G>(g, i)) <= 3.4028235e38f);
  if (__syncthreads_or(bad) && threadIdx.x == 0) amp[kAmpFound] = 1.f;
}

RK_API int rk_amp_check(int gdtype, const void* tensors, const void* blocks, int nblocks, float* amp, int chunk,
                        hipStream_t s) {
  if (nblocks <= 0) return 0;
  if (chunk != kChunk && chunk != kChunk / 4) return (int)hipErrorInvalidValue;
  const TensorRec* t = (const TensorRec*)tensors;
  const int2* b = (const int2*)blocks;
  if (gdtype == BF16)
    chunk == kChunk ? amp_check_kernel<uint16_t, 4><<<nblocks, kThreads, 0, s>>>(t, b, amp)
                    : amp_check_kernel<uint16_t, 1><<<nblocks, kThreads, 0, s>>>(t, b, amp);
  else
    chunk == kChunk ? amp_check_kernel<float, 4><<<nblocks, kThreads, 0, s>>>(t, b, amp)
                    : amp_check_kernel<float, 1><<<nblocks, kThreads, 0, s>>>(t, b, amp);
  return (int)hipGetLastError();
}

// kind: 0 = Adam/AdamW, 1 = SGD.  gdtype: grads dtype (0 f32, 1 bf16).  chunk: 1024 or 4096.
// amp: nullptr, or the device loss-scaling state (AmpSlot layout): gradients are unscaled by
// amp[kAmpInv] inside the update, a set found flag makes the step a no-op (step counter kept),
// and the last block applies the scale update.
RK_API int rk_optim_mt(int kind, int gdtype, const void* tensors, const void* blocks, int nblocks, const void* hyper,
                       float* step, float* amp, unsigned* counter, int zero_grads, int chunk, hipStream_t s) {
  if (nblocks <= 0) return 0;
  if (chunk != kChunk && chunk != kChunk / 4) return (int)hipErrorInvalidValue;
  const TensorRec* t = (const TensorRec*)tensors;
  const int2* b = (const int2*)blocks;
#define RK_OPT_LAUNCH_J(KERNEL, G, H, J)                                                                              \
  (zero_grads ? KERNEL<G, true, J><<<nblocks, kThreads, 0, s>>>(t, b, (const H*)hyper, step, amp, counter) \
              : KERNEL<G, false, J><<<nblocks, kThreads, 0, s>>>(t, b, (const H*)hyper, step, amp, counter))
#define RK_OPT_LAUNCH(KERNEL, G, H) \
  (chunk == kChunk ? RK_OPT_LAUNCH_J(KERNEL, G, H, 4) : RK_OPT_LAUNCH_J(KERNEL, G, H, 1))
  if (kind == 0) {
    if (gdtype == BF16)
      RK_OPT_LAUNCH(adam_mt_kernel, uint16_t, AdamHyper);
    else
      RK_OPT_LAUNCH(adam_mt_kernel, float, AdamHyper);
  } else {
    if (gdtype == BF16)
      RK_OPT_LAUNCH(sgd_mt_kernel, uint16_t, SgdHyper);
    else
      RK_OPT_LAUNCH(sgd_mt_kernel, float, SgdHyper);
  }
#undef RK_OPT_LAUNCH
#undef RK_OPT_LAUNCH_J
  return (int)hipGetLastError();
}

// Host-mapped (coherent) memory for device-published values the host polls with plain loads (the
// fp16 scaler's skip-flag ring, AmpSlot kAmpHost).  Returns the host address; *dev gets the
// device address to hand to kernels.  nullptr on failure.
RK_API void* rk_host_mapped_alloc(int64_t bytes, void** dev) {
  void* h = nullptr;
  if (hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  memset(h, 0, (size_t)bytes);
  if (hipHostGetDevicePointer(dev, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return nullptr;
  }
  return h;
}
RK_API void rk_host_mapped_free(void* h) {
  if (h) (void)hipHostFree(h);
}

