// Common device helpers for the rocket_amd CDNA4 (gfx950) kernels.
//
// Conventions
//  * every entry point is `extern "C"`, takes raw device pointers plus the HIP
//    stream to launch on (the current PyTorch stream, so calls are captured by
//    hipGraphs), and returns a hipError_t code;
//  * wave size is 64 (never 32): all cross-lane reductions cover 64 lanes;
//  * bf16 is stored as `__bf16` / raw uint16 and widened to f32 for math.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RK_API extern "C" __attribute__((visibility("default")))

namespace rk {

constexpr int kWave = 64;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

enum DType : int { F32 = 0, BF16 = 1, F16 = 2 };

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even; NaN stays NaN (plain cast lowers to v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// IEEE half (fp16 autocast): storage type _Float16, widened to f32 for math
typedef _Float16 f16_t;
__device__ __forceinline__ float h2f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// 16-bit storage chosen at run time (dt = BF16 / F16; wave-uniform, so the branch is free):
// pack two f32 into one 32-bit word, widen its low / high element, round an f32 to the storage type
__device__ __forceinline__ uint32_t pack16(float a, float b, int dt) {
  return dt == F16 ? (uint32_t)f2h(a) | ((uint32_t)f2h(b) << 16) : (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
__device__ __forceinline__ float lo16(uint32_t w, int dt) {
  return dt == F16 ? h2f((uint16_t)(w & 0xffffu)) : __uint_as_float(w << 16);
}
__device__ __forceinline__ float hi16(uint32_t w, int dt) {
  return dt == F16 ? h2f((uint16_t)(w >> 16)) : __uint_as_float(w & 0xffff0000u);
}
__device__ __forceinline__ float round16(float v, int dt) { return dt == F16 ? h2f(f2h(v)) : bf2f(f2bf(v)); }
// the same with the format fixed at compile time (H: fp16, else bf16) for kernels templated on it
template <bool H> __device__ __forceinline__ uint32_t pack16t(float a, float b) { return pack16(a, b, H ? F16 : BF16); }
template <bool H> __device__ __forceinline__ float lo16t(uint32_t w) { return lo16(w, H ? F16 : BF16); }
template <bool H> __device__ __forceinline__ float hi16t(uint32_t w) { return hi16(w, H ? F16 : BF16); }
template <bool H> __device__ __forceinline__ float round16t(float v) { return round16(v, H ? F16 : BF16); }

template <typename T> struct Ld;
template <> struct Ld<float> {
  static __device__ __forceinline__ float get(const float* p, int64_t i) { return p[i]; }
  static __device__ __forceinline__ void put(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Ld<uint16_t> {
  static __device__ __forceinline__ float get(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void put(uint16_t* p, int64_t i, float v) { p[i] = f2bf(v); }
};
template <> struct Ld<f16_t> {
  static __device__ __forceinline__ float get(const f16_t* p, int64_t i) { return (float)p[i]; }
  static __device__ __forceinline__ void put(f16_t* p, int64_t i, float v) { p[i] = (f16_t)v; }
};

// erf for the GELU kernels and epilogues: Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16
// output's 2^-9), one reciprocal + one exp + 5 FMAs instead of the ~20-instruction libm erff;
// e^{-u^2} is shared with gelu'.  Returns erf(u) given e = exp(-u*u).
__device__ __forceinline__ float erf_as(float u, float e) {
  const float a = fabsf(u);
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, a, 1.f));  // v_rcp_f32 (1 ulp), not an IEEE divide
  float p = __builtin_fmaf(1.061405429f, t, -1.453152027f);
  p = __builtin_fmaf(p, t, 1.421413741f);
  p = __builtin_fmaf(p, t, -0.284496736f);
  p = __builtin_fmaf(p, t, 0.254829592f);
  const float r = __builtin_fmaf(-p * t, e, 1.f);
  return copysignf(r, u);
}
__device__ __forceinline__ float gelu_f(float x) {
  const float u = x * 0.7071067811865476f;
  return 0.5f * x * (1.f + erf_as(u, __expf(-u * u)));
}
__device__ __forceinline__ float gelu_grad(float z) {
  const float u = z * 0.7071067811865476f;
  const float e = __expf(-u * u);  // = exp(-z^2/2): the Gaussian term of gelu' too
  return 0.5f * (1.f + erf_as(u, e)) + z * 0.3989422804014327f * e;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
// The same sum on the DPP network (no LDS traffic: __shfl_xor lowers to ds_bpermute, an LDS
// instruction that queues behind and bank-conflicts with the kernel's own LDS work): butterflies
// inside each 16-lane row, then the four row sums read out through SGPRs.  All 64 lanes must be
// active; the result is wave-uniform.
__device__ __forceinline__ float wave_sum_dpp(float v) {
  int t = __builtin_bit_cast(int, v);
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0xb1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
  t = __builtin_bit_cast(int, v);
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x4e, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
  t = __builtin_bit_cast(int, v);
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x141, 0xf, 0xf, false));  // row_half_mirror
  t = __builtin_bit_cast(int, v);
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x140, 0xf, 0xf, false));  // row_mirror
  t = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(t, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(t, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(t, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(t, 48)));
}
// Reduction over each 16-lane row (DPP butterflies, no LDS): every lane gets its row's sum / max.
__device__ __forceinline__ float row16_sum(float v) {
  int t = __builtin_bit_cast(int, v);
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0xb1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
  t = __builtin_bit_cast(int, v);
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x4e, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
  t = __builtin_bit_cast(int, v);
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x141, 0xf, 0xf, false));  // row_half_mirror
  t = __builtin_bit_cast(int, v);
  return v + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x140, 0xf, 0xf, false));  // row_mirror
}
__device__ __forceinline__ float row16_max(float v) {
  int t = __builtin_bit_cast(int, v);
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0xb1, 0xf, 0xf, false)));
  t = __builtin_bit_cast(int, v);
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x4e, 0xf, 0xf, false)));
  t = __builtin_bit_cast(int, v);
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x141, 0xf, 0xf, false)));
  t = __builtin_bit_cast(int, v);
  return fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x140, 0xf, 0xf, false)));
}
// sum of lanes 0, 16, 32, 48 (one value per 16-lane row), wave-uniform
__device__ __forceinline__ float rows4_sum(float v) {
  const int t = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(t, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(t, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(t, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(t, 48)));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum; `scratch` must hold blockDim.x/64 floats. Result valid in every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

// Write-through (sc1) stores / L1-bypassing (sc1) loads of data handed between workgroups in
// one launch (cdna guide §6 G16 R1): the hand-off then needs no agent-scope fences (no L2
// write-back, no L1 invalidate — each ≈1.7 µs on the critical path).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Last-arriving-block election for in-launch grid reductions.  Protocol: every partial the last
// block will read was stored with st_sc1 (by any wave of the producing block), and the last block
// reads EVERY such partial with ld_sc1.  Call from ALL threads after the partial stores: each wave
// drains its stores (vmcnt), the barrier orders them before lane 0's ticket.  Returns true in
// every thread of the block that arrived last.  `counter` must be 0 before the launch; the last
// block resets it (reset_counter), so graph replays stay valid.
__device__ __forceinline__ bool last_block_arrived(unsigned* counter, int* smem_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *smem_flag = (t == gridDim.x * gridDim.y * gridDim.z - 1);
  }
  __syncthreads();
  return *smem_flag != 0;
}

__device__ __forceinline__ void reset_counter(unsigned* counter) {
  if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bijective XCD-aware remap of a linear block id (8 XCDs, round-robin dispatch):
// consecutive logical tiles land on the same XCD (shared L2). Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nx = 8;
  if (nblocks < nx) return bid;
  int q = nblocks / nx, r = nblocks % nx, x = bid % nx, k = bid / nx;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// Grouped tile walk: linear tile id t (after xcd_remap the ids an XCD runs at once are
// consecutive) -> (tm, tn) in groups of gh tile-rows, column by column inside a group, so an
// XCD's concurrent tiles form a gh-row block sharing few A- and B-panels in its L2.  gh <= 1: the
// row-major walk.  A bijection for any tiles_m (the last group is shorter).
__device__ __forceinline__ void grouped_tile(int t, int tiles_m, int tiles_n, int gh, int& tm, int& tn) {
  if (gh <= 1) {
    tm = t / tiles_n;
    tn = t - tm * tiles_n;
    return;
  }
  const int per = gh * tiles_n;
  const int g = t / per, first = g * gh;
  const int h = min(tiles_m - first, gh);
  const int r = t - g * per;
  tm = first + r % h;
  tn = r / h;
}

}  // namespace rk
