// Fused small-channel convolution + bias + ReLU + 2x2 max-pool (LeNet: SURVEY K1-K4, K9-K11).
//
// Forward (one launch): each thread owns one pooled output (n, co, ph, pw), computes the
// 2x2 window of conv outputs from a (K+1)x(K+1) input patch per input channel, applies
// bias + ReLU, max-pools, and stores the pooled value (bf16 or f32) plus a 1-byte
// code = argmax position in the window (0..3), or 0xFF when the window is all <= 0
// (ReLU kills the gradient).  The pre-pool activation never touches HBM.
// The block's output channel is uniform (grid.y = co), so its weights live in LDS.
//
// Backward: the pooled gradient is routed through the saved code, which folds
// max_pool2d_with_indices_backward + threshold_backward into the consumers:
//  * wgrad/bias-grad: threads own one weight element (co, ci, kh, kw) and reduce over a
//    chunk of samples' pooled windows; chunk partials are added with f32 atomics into the
//    (persistent) gradient buffers;
//  * dgrad: threads own one input pixel (n, ih, iw) and produce all input channels.
#include "rk_common.h"

#include <algorithm>

using namespace rk;

namespace {

template <typename TI, typename TO>
__global__ void __launch_bounds__(256) conv_pool_fwd_kernel(const TI* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, TO* __restrict__ y,
                                                            uint8_t* __restrict__ code, int N, int Ci, int H, int W,
                                                            int Co, int K, int P, int Hp, int Wp) {
  extern __shared__ float wsh[];  // Ci*K*K weights of this block's output channel
  const int co = blockIdx.y;
  const int wn = Ci * K * K;
  for (int i = threadIdx.x; i < wn; i += blockDim.x) wsh[i] = w[(int64_t)co * wn + i];
  __syncthreads();
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)N * Hp * Wp;
  if (idx >= total) return;
  const int pw = idx % Wp;
  const int ph = (idx / Wp) % Hp;
  const int n = idx / ((int64_t)Wp * Hp);
  const int oh0 = 2 * ph, ow0 = 2 * pw;
  float a00 = 0.f, a01 = 0.f, a10 = 0.f, a11 = 0.f;
  for (int ci = 0; ci < Ci; ++ci) {
    const TI* xc = x + ((int64_t)n * Ci + ci) * H * W;
    const float* wc = wsh + ci * K * K;
    for (int r = 0; r <= K; ++r) {
      const int ih = oh0 + r - P;
      const bool rin = ih >= 0 && ih < H;
      float xv[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (c <= K) {
          const int iw = ow0 + c - P;
          xv[c] = (rin && iw >= 0 && iw < W) ? Ld<TI>::get(xc, (int64_t)ih * W + iw) : 0.f;
        }
      }
      // conv row r contributes to output row 0 with kernel row r and to output row 1 with kernel row r-1
#pragma unroll
      for (int c = 0; c < 15; ++c) {
        if (c < K) {
          if (r < K) {
            const float wv = wc[r * K + c];
            a00 = fmaf(xv[c], wv, a00);
            a01 = fmaf(xv[c + 1], wv, a01);
          }
          if (r >= 1) {
            const float wv = wc[(r - 1) * K + c];
            a10 = fmaf(xv[c], wv, a10);
            a11 = fmaf(xv[c + 1], wv, a11);
          }
        }
      }
    }
  }
  const float b = bias ? bias[co] : 0.f;
  a00 += b; a01 += b; a10 += b; a11 += b;
  float m = a00;
  int arg = 0;
  if (a01 > m) { m = a01; arg = 1; }
  if (a10 > m) { m = a10; arg = 2; }
  if (a11 > m) { m = a11; arg = 3; }
  const int64_t o = (((int64_t)n * Co + co) * Hp + ph) * Wp + pw;
  if (m > 0.f) {
    Ld<TO>::put(y, o, m);
    code[o] = (uint8_t)arg;
  } else {
    Ld<TO>::put(y, o, 0.f);
    code[o] = 0xFF;
  }
}

// Weight + bias gradient.  grid.x = chunks of samples, grid.y = co; threads own (ci,kh,kw).
template <typename TI, typename TG>
__global__ void __launch_bounds__(256) conv_pool_wgrad_kernel(const TI* __restrict__ x, const TG* __restrict__ dy,
                                                              const uint8_t* __restrict__ code, float* __restrict__ dw,
                                                              float* __restrict__ db, int N, int Ci, int H, int W,
                                                              int Co, int K, int P, int Hp, int Wp, int spc) {
  const int co = blockIdx.y;
  const int wn = Ci * K * K;
  const int n0 = blockIdx.x * spc, n1 = min(N, n0 + spc);
  for (int e = threadIdx.x; e < wn; e += blockDim.x) {
    const int ci = e / (K * K), kh = (e / K) % K, kw = e % K;
    float acc = 0.f, bacc = 0.f;
    for (int n = n0; n < n1; ++n) {
      const TI* xc = x + ((int64_t)n * Ci + ci) * H * W;
      const int64_t ob = ((int64_t)n * Co + co) * Hp * Wp;
      for (int p = 0; p < Hp * Wp; ++p) {
        const uint8_t cd = code[ob + p];
        if (cd == 0xFF) continue;
        const float g = Ld<TG>::get(dy, ob + p);
        const int oh = 2 * (p / Wp) + (cd >> 1), ow = 2 * (p % Wp) + (cd & 1);
        const int ih = oh + kh - P, iw = ow + kw - P;
        if (ih >= 0 && ih < H && iw >= 0 && iw < W) acc = fmaf(g, Ld<TI>::get(xc, (int64_t)ih * W + iw), acc);
        bacc += g;
      }
    }
    atomicAdd(dw + (int64_t)co * wn + e, acc);
    if (e == 0 && db) atomicAdd(db + co, bacc);
  }
}

// Input gradient: threads own (n, ih, iw) and produce all Ci channels (Ci <= 16).
template <typename TG, typename TO>
__global__ void __launch_bounds__(256) conv_pool_dgrad_kernel(const TG* __restrict__ dy, const uint8_t* __restrict__ code,
                                                              const float* __restrict__ w, TO* __restrict__ dx, int N,
                                                              int Ci, int H, int W, int Co, int K, int P, int Hp,
                                                              int Wp) {
  extern __shared__ float wsh[];  // all weights [Co][Ci][K][K]
  const int wn = Co * Ci * K * K;
  for (int i = threadIdx.x; i < wn; i += blockDim.x) wsh[i] = w[i];
  __syncthreads();
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * H * W) return;
  const int iw = idx % W, ih = (idx / W) % H;
  const int n = idx / ((int64_t)W * H);
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int kh = 0; kh < K; ++kh) {
    const int oh = ih + P - kh;
    if (oh < 0 || oh >= 2 * Hp) continue;
    for (int kw = 0; kw < K; ++kw) {
      const int ow = iw + P - kw;
      if (ow < 0 || ow >= 2 * Wp) continue;
      const int pos = ((oh & 1) << 1) | (ow & 1);
      const int64_t pbase = (int64_t)n * Co * Hp * Wp + (oh >> 1) * Wp + (ow >> 1);
      for (int co = 0; co < Co; ++co) {
        const int64_t o = pbase + (int64_t)co * Hp * Wp;
        if (code[o] != pos) continue;
        const float g = Ld<TG>::get(dy, o);
        const float* wc = wsh + ((co * Ci) * K + kh) * K + kw;
#pragma unroll
        for (int ci = 0; ci < 16; ++ci)
          if (ci < Ci) acc[ci] = fmaf(g, wc[ci * K * K], acc[ci]);
      }
    }
  }
#pragma unroll
  for (int ci = 0; ci < 16; ++ci)
    if (ci < Ci) Ld<TO>::put(dx, (((int64_t)n * Ci + ci) * H + ih) * W + iw, acc[ci]);
}

}  // namespace

RK_API int rk_conv_pool_fwd(const void* x, int x_dt, const float* w, const float* b, void* y, int y_dt, uint8_t* code,
                            int N, int Ci, int H, int W, int Co, int K, int P, hipStream_t s) {
  const int Hc = H + 2 * P - K + 1, Wc = W + 2 * P - K + 1;
  const int Hp = Hc / 2, Wp = Wc / 2;
  if (K > 15 || Hp <= 0 || Wp <= 0) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)N * Hp * Wp;
  dim3 grid((unsigned)((total + 255) / 256), Co);
  const size_t sh = sizeof(float) * Ci * K * K;
  if (x_dt == BF16 && y_dt == BF16)
    conv_pool_fwd_kernel<uint16_t, uint16_t><<<grid, 256, sh, s>>>((const uint16_t*)x, w, b, (uint16_t*)y, code, N, Ci, H, W, Co, K, P, Hp, Wp);
  else if (x_dt == F32 && y_dt == BF16)
    conv_pool_fwd_kernel<float, uint16_t><<<grid, 256, sh, s>>>((const float*)x, w, b, (uint16_t*)y, code, N, Ci, H, W, Co, K, P, Hp, Wp);
  else if (x_dt == F32 && y_dt == F32)
    conv_pool_fwd_kernel<float, float><<<grid, 256, sh, s>>>((const float*)x, w, b, (float*)y, code, N, Ci, H, W, Co, K, P, Hp, Wp);
  else
    conv_pool_fwd_kernel<uint16_t, float><<<grid, 256, sh, s>>>((const uint16_t*)x, w, b, (float*)y, code, N, Ci, H, W, Co, K, P, Hp, Wp);
  return (int)hipGetLastError();
}

// dw/db are ACCUMULATED into (f32 atomics): pass zeroed or persistent gradient buffers.
RK_API int rk_conv_pool_wgrad(const void* x, int x_dt, const void* dy, int dy_dt, const uint8_t* code, float* dw,
                              float* db, int N, int Ci, int H, int W, int Co, int K, int P, hipStream_t s) {
  const int Hp = (H + 2 * P - K + 1) / 2, Wp = (W + 2 * P - K + 1) / 2;
  const int wn = Ci * K * K;
  // ~2048 blocks in total: enough waves for 256 CUs, few enough atomics per weight
  const int want_chunks = std::max(1, 2048 / std::max(1, Co));
  const int spc = std::max(1, (N + want_chunks - 1) / want_chunks);
  const int chunks = (N + spc - 1) / spc;
  dim3 grid(chunks, Co);
  const int threads = wn >= 256 ? 256 : ((wn + 63) / 64) * 64;
#define RK_WG(TI, TG) conv_pool_wgrad_kernel<TI, TG><<<grid, threads, 0, s>>>((const TI*)x, (const TG*)dy, code, dw, db, N, Ci, H, W, Co, K, P, Hp, Wp, spc)
  if (x_dt == BF16 && dy_dt == BF16) RK_WG(uint16_t, uint16_t);
  else if (x_dt == F32 && dy_dt == BF16) RK_WG(float, uint16_t);
  else if (x_dt == F32 && dy_dt == F32) RK_WG(float, float);
  else RK_WG(uint16_t, float);
#undef RK_WG
  return (int)hipGetLastError();
}

RK_API int rk_conv_pool_dgrad(const void* dy, int dy_dt, const uint8_t* code, const float* w, void* dx, int dx_dt,
                              int N, int Ci, int H, int W, int Co, int K, int P, hipStream_t s) {
  const int Hp = (H + 2 * P - K + 1) / 2, Wp = (W + 2 * P - K + 1) / 2;
  if (Ci > 16) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)N * H * W;
  const size_t sh = sizeof(float) * Co * Ci * K * K;
  const unsigned grid = (unsigned)((total + 255) / 256);
#define RK_DG(TG, TO) conv_pool_dgrad_kernel<TG, TO><<<grid, 256, sh, s>>>((const TG*)dy, code, w, (TO*)dx, N, Ci, H, W, Co, K, P, Hp, Wp)
  if (dy_dt == BF16 && dx_dt == BF16) RK_DG(uint16_t, uint16_t);
  else if (dy_dt == BF16 && dx_dt == F32) RK_DG(uint16_t, float);
  else if (dy_dt == F32 && dx_dt == F32) RK_DG(float, float);
  else RK_DG(float, uint16_t);
#undef RK_DG
  return (int)hipGetLastError();
}
