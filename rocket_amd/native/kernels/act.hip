// Elementwise / row-wise activation kernels for the transformer path (ViT-B/16):
//
//   gelu_fwd     y = gelu(x) (erf form; erf to 1.5e-7, rk_common.h), bf16/fp16/f32 in/out, 4 elements per access.
//   gelu_bwd     dx = dy * gelu'(x), recomputed from the saved pre-activation (no extra tensor).
//   softmax_fwd  y = softmax(x * scale) over rows of length L (attention scores), one wave per
//                row, values held in registers (L <= 1024): one read, one write.
//   softmax_bwd  dx = scale * y * (dy - sum(dy * y)), one wave per row.
#include "rk_common.h"

using namespace rk;

namespace {

constexpr int T = 256;

template <typename E> struct V4;
template <> struct V4<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const float4 a = *(const float4*)p;
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* v) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
};
template <> struct V4<uint16_t> {
  static __device__ __forceinline__ void load(const uint16_t* p, float* v) {
    const uint2 u = *(const uint2*)p;
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float* v) {
    uint2 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *(uint2*)p = u;
  }
};

template <> struct V4<f16_t> {  // IEEE half (fp16 autocast)
  static __device__ __forceinline__ void load(const f16_t* p, float* v) {
    const uint2 u = *(const uint2*)p;
    v[0] = h2f((uint16_t)(u.x & 0xffffu)); v[1] = h2f((uint16_t)(u.x >> 16));
    v[2] = h2f((uint16_t)(u.y & 0xffffu)); v[3] = h2f((uint16_t)(u.y >> 16));
  }
  static __device__ __forceinline__ void store(f16_t* p, const float* v) {
    uint2 u;
    u.x = (uint32_t)f2h(v[0]) | ((uint32_t)f2h(v[1]) << 16);
    u.y = (uint32_t)f2h(v[2]) | ((uint32_t)f2h(v[3]) << 16);
    *(uint2*)p = u;
  }
};

// 4 elements per thread per iteration (8-byte bf16 / 16-byte f32 accesses); n % 4 == 0 (host)
template <typename TI, typename TO>
__global__ void __launch_bounds__(T) gelu_fwd_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
  for (int64_t i = ((int64_t)blockIdx.x * T + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * T * 4) {
    float v[4];
    V4<TI>::load(x + i, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = gelu_f(v[k]);
    V4<TO>::store(y + i, v);
  }
}

// 16-bit in and out (bf16 / fp16, same type), n % 8 == 0: 16-byte accesses, GU chunks of 8 elements
// per thread with all their loads issued first, and (NT) nontemporal loads / stores — the pass
// touches each element once and the tensors are far larger than L2 (ViT fc1: 25216 x 3072).
// (The 4-element form above kept one 8-byte load in flight per thread: 4.3 TB/s on the ViT shape.)
template <typename E, bool NT>
__global__ void __launch_bounds__(T) gelu_fwd16_kernel(const E* __restrict__ x, E* __restrict__ y, int64_t n) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int GU = 4;
  const int64_t stride = (int64_t)gridDim.x * T * 8;
  for (int64_t i0 = ((int64_t)blockIdx.x * T + threadIdx.x) * 8; i0 < n; i0 += stride * GU) {
    u32x4 w[GU];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int64_t i = i0 + u * stride;
      const u32x4* p = (const u32x4*)(x + (i < n ? i : 0));
      w[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n) break;
      float v[8];
      V4<E>::load((const E*)&w[u], v);
      V4<E>::load((const E*)&w[u] + 4, v + 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = gelu_f(v[k]);
      u32x4 o;
      V4<E>::store((E*)&o, v);
      V4<E>::store((E*)&o + 4, v + 4);
      if (NT) __builtin_nontemporal_store(o, (u32x4*)(y + i));
      else *(u32x4*)(y + i) = o;
    }
  }
}

template <typename TI, typename TG>
__global__ void __launch_bounds__(T) gelu_bwd_kernel(const TG* __restrict__ dy, const TI* __restrict__ x,
                                                     TI* __restrict__ dx, int64_t n) {
  for (int64_t i = ((int64_t)blockIdx.x * T + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * T * 4) {
    float g[4], v[4];
    V4<TG>::load(dy + i, g);
    V4<TI>::load(x + i, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = g[k] * gelu_grad(v[k]);
    V4<TI>::store(dx + i, v);
  }
}

constexpr int SM_MAXJ = 16;  // 16 x 64 lanes = L <= 1024

template <typename TI, typename TO, int NJ>
__global__ void __launch_bounds__(T) softmax_fwd_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t rows,
                                                        int L, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (T / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TI* xr = x + row * L;
  float v[NJ];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 64 + lane;
    v[j] = c < L ? Ld<TI>::get(xr, c) * scale : -INFINITY;
    m = fmaxf(m, v[j]);
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    v[j] = (j * 64 + lane) < L ? __expf(v[j] - m) : 0.f;
    s += v[j];
  }
  const float inv = 1.f / wave_sum(s);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 64 + lane;
    if (c < L) Ld<TO>::put(y + row * L, c, v[j] * inv);
  }
}

template <typename TY, typename TG, int NJ>
__global__ void __launch_bounds__(T) softmax_bwd_kernel(const TG* __restrict__ dy, const TY* __restrict__ y,
                                                        TG* __restrict__ dx, int64_t rows, int L, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (T / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  float yv[NJ], gv[NJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 64 + lane;
    yv[j] = c < L ? Ld<TY>::get(y + row * L, c) : 0.f;
    gv[j] = c < L ? Ld<TG>::get(dy + row * L, c) : 0.f;
    s += yv[j] * gv[j];
  }
  s = wave_sum(s);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 64 + lane;
    if (c < L) Ld<TG>::put(dx + row * L, c, scale * yv[j] * (gv[j] - s));
  }
}

int egrid(int64_t n) {
  int64_t g = (n + T - 1) / T;
  return (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

}  // namespace

// element type per dtype code (F32 / BF16 / F16), for the two-type elementwise dispatches below
#define RK_ACT_T(dt, T0, ...)                                     \
  do {                                                            \
    if ((dt) == BF16) { typedef uint16_t T0; __VA_ARGS__ }        \
    else if ((dt) == F16) { typedef f16_t T0; __VA_ARGS__ }       \
    else { typedef float T0; __VA_ARGS__ }                        \
  } while (0)

RK_API int rk_gelu_fwd(int dti, int dto, const void* x, void* y, int64_t n, hipStream_t s) {
  if (n % 4 || dti < 0 || dti > 2 || dto < 0 || dto > 2) return (int)hipErrorInvalidValue;
  // ROCKET_GELU_EW: 0 = the 4-element kernel, 1 = 16-byte chunks, 2 = 16-byte chunks, nontemporal (default)
  static const int ev = getenv("ROCKET_GELU_EW") ? atoi(getenv("ROCKET_GELU_EW")) : 2;
  if (ev > 0 && dti == dto && dti != F32 && n % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    const int g = egrid((n / 8 + 3) / 4);
    if (dti == BF16) {
      if (ev == 2) gelu_fwd16_kernel<uint16_t, true><<<g, T, 0, s>>>((const uint16_t*)x, (uint16_t*)y, n);
      else gelu_fwd16_kernel<uint16_t, false><<<g, T, 0, s>>>((const uint16_t*)x, (uint16_t*)y, n);
    } else {
      if (ev == 2) gelu_fwd16_kernel<f16_t, true><<<g, T, 0, s>>>((const f16_t*)x, (f16_t*)y, n);
      else gelu_fwd16_kernel<f16_t, false><<<g, T, 0, s>>>((const f16_t*)x, (f16_t*)y, n);
    }
    return (int)hipGetLastError();
  }
  const int g = egrid(n / 4);
  RK_ACT_T(dti, TI, RK_ACT_T(dto, TO, gelu_fwd_kernel<TI, TO><<<g, T, 0, s>>>((const TI*)x, (TO*)y, n);););
  return (int)hipGetLastError();
}

// dti: dtype of x / dx; dtg: dtype of dy
RK_API int rk_gelu_bwd(int dti, int dtg, const void* dy, const void* x, void* dx, int64_t n, hipStream_t s) {
  if (n % 4 || dti < 0 || dti > 2 || dtg < 0 || dtg > 2) return (int)hipErrorInvalidValue;
  const int g = egrid(n / 4);
  RK_ACT_T(dti, TI, RK_ACT_T(dtg, TG, gelu_bwd_kernel<TI, TG><<<g, T, 0, s>>>((const TG*)dy, (const TI*)x, (TI*)dx, n);););
  return (int)hipGetLastError();
}

RK_API int rk_softmax_fwd(int dti, int dto, const void* x, void* y, int64_t rows, int L, float scale, hipStream_t s) {
  if (L <= 0 || L > 64 * SM_MAXJ) return (int)hipErrorInvalidValue;
  const int grid = (int)((rows + T / 64 - 1) / (T / 64));
  const int nj = (L + 63) / 64;
#define RK_SF(TI, TO, NJ) softmax_fwd_kernel<TI, TO, NJ><<<grid, T, 0, s>>>((const TI*)x, (TO*)y, rows, L, scale)
#define RK_SFN(TI, TO)                 \
  if (nj <= 2) RK_SF(TI, TO, 2);       \
  else if (nj <= 4) RK_SF(TI, TO, 4);  \
  else if (nj <= 8) RK_SF(TI, TO, 8);  \
  else RK_SF(TI, TO, 16);
  if (dti == BF16 && dto == BF16) { RK_SFN(uint16_t, uint16_t) }
  else if (dti == BF16) { RK_SFN(uint16_t, float) }
  else if (dto == BF16) { RK_SFN(float, uint16_t) }
  else { RK_SFN(float, float) }
#undef RK_SFN
#undef RK_SF
  return (int)hipGetLastError();
}

// dty: dtype of y; dtg: dtype of dy and dx
RK_API int rk_softmax_bwd(int dty, int dtg, const void* dy, const void* y, void* dx, int64_t rows, int L, float scale,
                          hipStream_t s) {
  if (L <= 0 || L > 64 * SM_MAXJ) return (int)hipErrorInvalidValue;
  const int grid = (int)((rows + T / 64 - 1) / (T / 64));
  const int nj = (L + 63) / 64;
#define RK_SB(TY, TG, NJ) softmax_bwd_kernel<TY, TG, NJ><<<grid, T, 0, s>>>((const TG*)dy, (const TY*)y, (TG*)dx, rows, L, scale)
#define RK_SBN(TY, TG)                 \
  if (nj <= 2) RK_SB(TY, TG, 2);       \
  else if (nj <= 4) RK_SB(TY, TG, 4);  \
  else if (nj <= 8) RK_SB(TY, TG, 8);  \
  else RK_SB(TY, TG, 16);
  if (dty == BF16 && dtg == BF16) { RK_SBN(uint16_t, uint16_t) }
  else if (dty == BF16) { RK_SBN(uint16_t, float) }
  else if (dtg == BF16) { RK_SBN(float, uint16_t) }
  else { RK_SBN(float, float) }
#undef RK_SBN
#undef RK_SB
  return (int)hipGetLastError();
}
