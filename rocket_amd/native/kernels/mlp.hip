// Fused ReLU MLP head, 3 linear layers (LeNet classifier fc1-ReLU-fc2-ReLU-fc3: SURVEY K4/K5/K8/K9).
//
// Three launches per training step, all on v_mfma_f32_16x16x32_bf16 (f32 accumulate):
//
//  mlp3_fwd    A block owns 16 batch rows and runs the whole chain
//              h1 = relu(x W1^T + b1), h2 = relu(h1 W2^T + b2), y = h2 W3^T + b3
//              with activations resident in LDS (bf16).  Weights come straight from the
//              fp32 master copy (L2-resident), every k-step's B fragment of a tile is
//              prefetched before the first MFMA (one L2 latency per tile, not one per k-step).
//              Side outputs for the backward are written TRANSPOSED (x^T, h1^T, h2^T:
//              [features][batch]) so the weight-gradient GEMM reads K-contiguous rows.
//  mlp3_dgrad  Same row blocking: d2 = (dy W3)[h2>0], d1 = (d2 W2)[h1>0], dx = d1 W1; writes
//              dy^T, d2^T, d1^T for the weight gradients and dx (row-major) for the conv backward.
//  mlp3_wgrad  All three dW_l += d_l^T-rows . x_l^T-rows (reduction over the batch) and the bias
//              gradients (row sums of d_l^T) in ONE grouped launch: a block owns a 32x32 tile
//              of one layer's dW, its 8 waves split the batch, partial tiles are reduced in LDS
//              and added once — deterministic, no atomics.
//
// Everything is branch-free in the load paths (clamped addresses + selects).
#include "optim_common.h"
#include "rows_common.h"

#include <cstdlib>

using namespace rk;

// 16-bit format of every activation / fragment / weight-gradient operand: bf16 (default) or, when
// this file is compiled with RK_LENET_H = 1 (the *_h.hip wrapper TU), IEEE fp16 for autocast fp16;
// the fp16 build's entry points carry an "_h" suffix.
#ifndef RK_LENET_H
#define RK_LENET_H 0
#endif
#if RK_LENET_H
#define RKL_NAME(n) n##_h
#else
#define RKL_NAME(n) n
#endif

namespace {

constexpr bool kH16 = RK_LENET_H;
__device__ __forceinline__ uint16_t c16(float v) { return kH16 ? f2h(v) : f2bf(v); }
__device__ __forceinline__ float d16(uint16_t v) { return kH16 ? h2f(v) : bf2f(v); }
__device__ __forceinline__ __bf16 e16(float v) { return __builtin_bit_cast(__bf16, c16(v)); }
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  typedef __attribute__((ext_vector_type(8))) _Float16 h8;
  if constexpr (kH16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

constexpr int ROWS = 16;
constexpr int MAXK = 512;
constexpr int LDSW = MAXK + 8;
constexpr int NW = 8;  // waves per block
constexpr int NT = 64 * NW;

// B fragment of a [N][K] fp32 row-major weight for output tile nt, k-step ks (forward: y = a W^T).
// K % 4 == 0 (checked on the host): two 16-byte loads, each all-in or all-out of range.
__device__ __forceinline__ bf16x8 wfrag_fwd(const float* W, int N, int K, int nt, int ks, int lane) {
  const int n = nt * 16 + (lane & 15), k0 = ks * 32 + 8 * (lane >> 4);
  const int nc = n < N ? n : N - 1;
  const int ka = k0 < K ? k0 : K - 4, kb = k0 + 4 < K ? k0 + 4 : K - 4;
  const float4 v0 = *(const float4*)(W + (int64_t)nc * K + ka);
  const float4 v1 = *(const float4*)(W + (int64_t)nc * K + kb);
  const bool oa = n < N && k0 < K, ob = n < N && k0 + 4 < K;
  bf16x8 b;
  b[0] = e16(oa ? v0.x : 0.f); b[1] = e16(oa ? v0.y : 0.f);
  b[2] = e16(oa ? v0.z : 0.f); b[3] = e16(oa ? v0.w : 0.f);
  b[4] = e16(ob ? v1.x : 0.f); b[5] = e16(ob ? v1.y : 0.f);
  b[6] = e16(ob ? v1.z : 0.f); b[7] = e16(ob ? v1.w : 0.f);
  return b;
}

// B fragment for the input gradient (dx = d W): B[k = n][col = c] = W[n][c].
__device__ __forceinline__ bf16x8 wfrag_bwd(const float* W, int N, int K, int ct, int ks, int lane) {
  const int c = ct * 16 + (lane & 15), n0 = ks * 32 + 8 * (lane >> 4);
  const int cc = c < K ? c : K - 1;
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = n0 + j;
    const float v = W[(int64_t)(n < N ? n : N - 1) * K + cc];
    b[j] = e16((c < K && n < N) ? v : 0.f);
  }
  return b;
}

__device__ __forceinline__ bf16x8 afrag(const uint16_t* act, int ks, int lane) {
  return *(const bf16x8*)(act + (lane & 15) * LDSW + ks * 32 + 8 * (lane >> 4));
}

// out = act(in . W^T + b) for the block's 16 rows; KS = k-steps (compile time: prefetch depth)
template <int KS>
__device__ __forceinline__ void layer_fwd(const uint16_t* in, int K, const float* W, const float* b, int N, bool relu,
                                          uint16_t* out, float* gout_f32, int64_t row0, int M) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ntiles = (N + 15) / 16;
  for (int nt = wv; nt < ntiles; nt += NW) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (KS > 0) {
      bf16x8 bf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) bf[ks] = wfrag_fwd(W, N, K, nt, ks, lane);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = mfma16(afrag(in, ks, lane), bf[ks], acc);
    } else {  // generic widths: prefetch 4 k-steps at a time
      for (int k0 = 0; k0 < (K + 31) / 32; k0 += 4) {
        bf16x8 bf[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) bf[q] = wfrag_fwd(W, N, K, nt, k0 + q, lane);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (k0 + q < (K + 31) / 32)  // uniform; never read LDS columns past the staged width
            acc = mfma16(afrag(in, k0 + q, lane), bf[q], acc);
      }
    }
    const int col = nt * 16 + (lane & 15);
    const float bias = b[col < N ? col : 0];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * (lane >> 4) + i;
      float v = acc[i] + bias;
      if (relu) v = fmaxf(v, 0.f);
      if (col < N) {
        if (out) out[r * LDSW + col] = c16(v);
        if (gout_f32 && row0 + r < M) gout_f32[(row0 + r) * N + col] = v;
      }
    }
  }
}

// dgrad: out[16][K] = (in[16][N] . W[N][K]) * [maskT > 0]; maskT is [K][M] (transposed activation)
template <int KS>
__device__ __forceinline__ void layer_dgrad(const uint16_t* in, int N, const float* W, int K, const uint16_t* maskT,
                                            uint16_t* out, uint16_t* gout_rows, int64_t row0, int M) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ctiles = (K + 15) / 16;
  for (int ct = wv; ct < ctiles; ct += NW) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (KS > 0) {
      bf16x8 bf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) bf[ks] = wfrag_bwd(W, N, K, ct, ks, lane);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = mfma16(afrag(in, ks, lane), bf[ks], acc);
    } else {
      for (int k0 = 0; k0 < (N + 31) / 32; k0 += 4) {
        bf16x8 bf[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) bf[q] = wfrag_bwd(W, N, K, ct, k0 + q, lane);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (k0 + q < (N + 31) / 32)
            acc = mfma16(afrag(in, k0 + q, lane), bf[q], acc);
      }
    }
    const int col = ct * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * (lane >> 4) + i;
      const bool rin = row0 + r < M;
      float v = acc[i];
      if (maskT) {
        const float mv = d16(maskT[(int64_t)(col < K ? col : 0) * M + (rin ? row0 + r : 0)]);
        v = mv > 0.f ? v : 0.f;
      }
      if (col < K) {
        if (out) out[r * LDSW + col] = c16(v);
        if (gout_rows && rin) gout_rows[(row0 + r) * K + col] = c16(v);
      }
    }
  }
}

__device__ void zero_pad(uint16_t* buf, int c0, int c1) {
  for (int i = threadIdx.x; i < ROWS * (c1 - c0); i += blockDim.x) {
    const int r = i / (c1 - c0), c = c0 + i % (c1 - c0);
    buf[r * LDSW + c] = 0;
  }
}

__device__ void stage_rows(uint16_t* dst, const void* src, int src_f32, int K, int64_t row0, int M) {
  const int Kp = (K + 31) / 32 * 32;
  for (int i = threadIdx.x; i < ROWS * Kp; i += blockDim.x) {
    const int r = i / Kp, c = i % Kp;
    const bool ok = c < K && row0 + r < M;
    const int64_t o = ok ? (row0 + r) * K + c : 0;
    const float v = src_f32 ? ((const float*)src)[o] : d16(((const uint16_t*)src)[o]);
    dst[r * LDSW + c] = c16(ok ? v : 0.f);
  }
}

// write the block's [16][C] LDS activation as columns of a transposed [C][M] global tensor
__device__ void store_transposed(uint16_t* __restrict__ gT, const uint16_t* buf, int C, int64_t row0, int M) {
  const bool full = row0 + ROWS <= M && (M & 7) == 0;
  for (int i = threadIdx.x; i < C * 2; i += blockDim.x) {
    const int c = i >> 1, h = i & 1;  // 8-row half h of column c
    if (full) {
      uint4 v;
      uint32_t* w = (uint32_t*)&v;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = (uint32_t)buf[(8 * h + 2 * k) * LDSW + c] | ((uint32_t)buf[(8 * h + 2 * k + 1) * LDSW + c] << 16);
      *(uint4*)(gT + (int64_t)c * M + row0 + 8 * h) = v;
    } else {
      for (int k = 0; k < 8; ++k)
        if (row0 + 8 * h + k < M) gT[(int64_t)c * M + row0 + 8 * h + k] = buf[(8 * h + k) * LDSW + c];
    }
  }
}

template <int KS1, int KS2, int KS3>
__global__ void __launch_bounds__(NT) mlp3_fwd_kernel(const uint16_t* __restrict__ x, int K0, const float* w1,
                                                      const float* b1, int N1, const float* w2, const float* b2, int N2,
                                                      const float* w3, const float* b3, int N3, uint16_t* xT,
                                                      uint16_t* h1T, uint16_t* h2T, float* y, int M) {
  __shared__ __attribute__((aligned(16))) uint16_t buf0[ROWS * LDSW];
  __shared__ __attribute__((aligned(16))) uint16_t buf1[ROWS * LDSW];
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;
  stage_rows(buf0, x, 0, K0, row0, M);
  zero_pad(buf1, N1, KS2 > 0 ? KS2 * 32 : (N1 + 31) / 32 * 32);
  __syncthreads();
  if (xT) store_transposed(xT, buf0, K0, row0, M);
  layer_fwd<KS1>(buf0, K0, w1, b1, N1, true, buf1, nullptr, row0, M);
  __syncthreads();
  store_transposed(h1T, buf1, N1, row0, M);
  zero_pad(buf0, N2, KS3 > 0 ? KS3 * 32 : (N2 + 31) / 32 * 32);
  __syncthreads();
  layer_fwd<KS2>(buf1, N1, w2, b2, N2, true, buf0, nullptr, row0, M);
  __syncthreads();
  store_transposed(h2T, buf0, N2, row0, M);
  layer_fwd<KS3>(buf0, N2, w3, b3, N3, false, nullptr, y, row0, M);
}

template <int KS3, int KS2, int KS1>
__global__ void __launch_bounds__(NT) mlp3_dgrad_kernel(const float* __restrict__ dy, int N3, const float* w3, int N2,
                                                        const uint16_t* h2T, const float* w2, int N1,
                                                        const uint16_t* h1T, const float* w1, int K0, uint16_t* dyT,
                                                        uint16_t* d2T, uint16_t* d1T, uint16_t* dx, int M) {
  __shared__ __attribute__((aligned(16))) uint16_t buf0[ROWS * LDSW];
  __shared__ __attribute__((aligned(16))) uint16_t buf1[ROWS * LDSW];
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;
  stage_rows(buf0, dy, 1, N3, row0, M);
  zero_pad(buf1, N2, KS2 > 0 ? KS2 * 32 : (N2 + 31) / 32 * 32);
  __syncthreads();
  store_transposed(dyT, buf0, N3, row0, M);
  layer_dgrad<KS3>(buf0, N3, w3, N2, h2T, buf1, nullptr, row0, M);
  __syncthreads();
  store_transposed(d2T, buf1, N2, row0, M);
  zero_pad(buf0, N1, KS1 > 0 ? KS1 * 32 : (N1 + 31) / 32 * 32);
  __syncthreads();
  layer_dgrad<KS2>(buf1, N2, w2, N1, h1T, buf0, nullptr, row0, M);
  __syncthreads();
  store_transposed(d1T, buf0, N1, row0, M);
  if (dx) layer_dgrad<KS1>(buf0, N1, w1, K0, nullptr, nullptr, dx, row0, M);
}

// ------------------------------------------------------------------ grouped weight gradient
struct WgradProb {
  const uint16_t* dT;  // [N][M]
  const uint16_t* xT;  // [K][M]
  float* dw;           // [N][K], accumulated
  float* db;           // [N], accumulated (may be null)
  int N, K, tiles_k, tile_begin;
};
// optional column reduction riding on the same launch: dst[c] += sum_r slab[r][c] over the
// [rows][width] slab of per-block partials (the fused LeNet backward's conv gradients); columns
// [bound[i], bound[i+1]) go to dst[i] (null = dropped).
struct SlabArgs {
  const float* slab;
  int rows, width, ncols, nblocks;
  float* dst[4];
  int bound[5];
};
// Batch-loss finalisation riding on the wgrad launch (the LeNet backward stores per-block CE
// partials and the valid count; one extra block here sums them and does the Loss capsule's
// accumulate / report-ring bookkeeping — no last-block ticket at the end of the backward).
struct LossFin {
  const float* partials;
  int nparts;
  float* loss_out;  // [2]: loss (written here), nvalid (written by the backward)
  float *acc, *ring;
  int64_t* slot;
  int ring_size;
  float acc_scale;
  int sync;
};
struct WgradArgs {
  int late_ticket;  // LDS-staged dW tile blocks take the optimizer-step ticket after their operand wait
  uint64_t* trace;  // optional phase stamps [blocks][8] (s_memrealtime): start, reduced, end, tile: old values in, main loop done
  float gscale;     // every produced gradient is scaled by this (the upstream gradient factor)
  // normalisation by a count the backward left unapplied (the fused LeNet cross-entropy's mean,
  // pre-scaled by 1 / M): gradients are also scaled by M / sum(cnt_parts[0..ncnt)), and the loss
  // block divides by that sum
  const float* cnt_parts;
  int ncnt;
  // deferred loader batch consumed by this step (runtime/data.py PendingRows): one extra block
  // advances the epoch cursor and stages the next batch's rows (rows_common.h), or null
  const int64_t* rn_table;
  int64_t* rn_meta;
  int64_t* rn_rows;
  int rn_cur, rn_bs, has_rows;
  WgradProb p[3];
  int nprob, M, tiles, nslab;
  SlabArgs sl;
  int has_loss;
  LossFin lf;
  // optional optimizer epilogue: records of the 3 dW / 3 db / 4 slab destinations' parameters
  rk_opt::AdamEpi epi;
  rk_opt::TensorRec rdw[3], rdb[3], rsl[4];
  // fp16 AMP (may be null): any non-finite gradient this launch writes sets *amp_found = 1 (the
  // loss scaler's found-inf slot), so the step needs no separate check launch
  float* amp_found;
};

__device__ __forceinline__ void flag_nonfinite(float* found, float v) {
  if (found && !__builtin_isfinite(v)) *found = 1.f;  // same value from any lane: benign race
}



// one slab block: SLC = 32 columns x all rows; 16 row groups per block, 16 independent loads per
// thread in flight, LDS reduce over the groups, one plain RMW per column (sole owner: deterministic).
// (32 columns, not 64: the LeNet launch then has > 200 workgroups, the slab part 81 of them.)
constexpr int SLC = 32, SLG = NT / SLC;
constexpr int kEpiGroups = 4;  // param groups the epilogue precomputes step constants for

// per-group Adam constants of this launch's step, written to LDS before the caller's barrier
struct StepFill {
  const WgradArgs* a;
  float cur;
  rk_opt::AdamStep* s_ks;
  float cpart;   // this thread's share of the count partials (loaded at kernel start)
  float* s_cnt;  // [NW] per-wave count sums
  rk_opt::AdamHyper hy;  // threads < kEpiGroups: their group's hyperparameters (loaded at kernel start)
  __device__ __forceinline__ void operator()() const {
    if (a->epi.on && threadIdx.x < kEpiGroups) s_ks[threadIdx.x] = rk_opt::adam_step(hy, cur + 1.f);
    if (a->cnt_parts) {
      const float c = wave_sum_dpp(cpart);  // (all lanes active; DPP, not six ds_bpermute round trips)
      if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = c;
    }
  }
  // after the caller's barrier: the gradient factor (gscale / count when normalising)
  __device__ __forceinline__ float count() const {
    float n = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) n += s_cnt[w];
    return n;
  }
  __device__ __forceinline__ float gs() const {
    if (!a->cnt_parts) return a->gscale;
    const float n = count();  // the backward pre-scaled by 1 / M (the batch): apply M / count
    return n > 0.f ? a->gscale * ((float)a->M / n) : 0.f;
  }
};

__device__ void loss_fin_block(const LossFin& f, float (*red)[32 * 32], const StepFill& sf) {
  float t = 0.f;
  for (int i = threadIdx.x; i < f.nparts; i += NT) t += f.partials[i];
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) t += __shfl_xor(t, k, 64);
  if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = t;
  sf();
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < NT / 64; ++w) s += red[0][w];  // fixed order: deterministic
    float nv;
    if (sf.a->cnt_parts) {
      nv = sf.count();
      f.loss_out[1] = nv;
    } else {
      nv = f.loss_out[1];
    }
    const float l = nv > 0.f ? s / nv : NAN;
    f.loss_out[0] = l;
    if (f.acc) {
      float v = f.acc[0] + l * f.acc_scale;
      if (f.sync) {
        const int64_t k = f.slot[0];
        f.ring[k] = v;
        f.slot[0] = (k + 1) % f.ring_size;
        v = 0.f;
      }
      f.acc[0] = v;
    }
  }
}

__device__ __forceinline__ void slab_reduce_block(const WgradArgs& a, int j, float (*red)[32 * 32],
                                                  const rk_opt::AdamStep* ks, const StepFill& sf) {
  const SlabArgs& s = a.sl;
  const int cl = threadIdx.x % SLC, rg = threadIdx.x / SLC;
  const int c = j * SLC + cl;
  const bool ok = c < s.ncols;
  const float* base = s.slab + (ok ? c : 0);
  // the destination value is read up front (this block is its only writer), and each thread keeps
  // its slab rows in flight at once: the launch is one memory round trip, not several
  float* dst = nullptr;
  float old = 0.f;
  int di = 0;
  rk_opt::EpiElem ee{};
  if (threadIdx.x < SLC && ok) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (c >= s.bound[i] && c < s.bound[i + 1] && s.dst[i]) {
        dst = s.dst[i] + (c - s.bound[i]);
        di = i;
      }
    if (dst) {
      old = *dst;
      if (ks) ee = rk_opt::epi_fetch(a.rsl[di], c - s.bound[di]);
    }
  }
  constexpr int U = 16;
  float acc = 0.f;
  int r = rg;
  for (; r + (U - 1) * SLG < s.rows; r += U * SLG) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base[(int64_t)(r + u * SLG) * s.width];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  for (; r < s.rows; r += SLG) acc += base[(int64_t)r * s.width];
  float* const redf = &red[0][0];
  redf[rg * SLC + cl] = acc;
  sf();
  __syncthreads();
  if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memrealtime();
  if (dst) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < SLG; ++g) t += redf[g * SLC + threadIdx.x];
    t *= sf.gs();
    if (ks) rk_opt::epi_apply(a.rsl[di], ks[a.rsl[di].group], c - s.bound[di], ee, old + t, a.epi.zero_grads);
    else *dst = old + t;
    flag_nonfinite(a.amp_found, old + t);
  }
}

// 8 consecutive batch elements m0.. of row r of a [R][M] bf16 tensor; zero when out of range
// (M % 8 == 0, so a group is all-in or all-out).
__device__ __forceinline__ bf16x8 rowfrag(const uint16_t* T, int R, int M, int r, int m0) {
  const bool ok = r < R && m0 < M;
  const uint4 v = *(const uint4*)(T + (int64_t)(r < R ? r : 0) * M + (ok ? m0 : 0));
  const uint4 z = make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(bf16x8, ok ? v : z);
}


// dW tile: WTN output features (rows of d^T) x 32 input features (rows of x^T).  16, not 32: the
// LeNet launch's 67 tiles become 131 (> 200 workgroups with the slab blocks), each block's chain of
// operand latency -> 8-wave LDS reduction -> optimizer epilogue half as long.
constexpr int WTN = 16, WNI = WTN / 16, WEPT = WTN * 32 / NT;
static_assert(WEPT >= 1 && WTN * 32 % NT == 0, "tile elements per thread");

template <bool LDSV>
__device__ void wgrad_tile(const WgradArgs& a, float (*red)[32 * 32], float (*rsum)[32], const rk_opt::AdamStep* ks,
                           const StepFill& sf, char* stage, unsigned* ticket);

// LDSV: the tiles' operands arrive by LDS-DMA in whole 256-B row segments (16 KiB per wave: its 32 rows
// of d^T and x^T over its 128 batch elements) and the MFMA fragments are read back from LDS, instead of
// fragment-shaped global loads (16 rows x 64 B per instruction: half cache lines).  M % 512 == 0.
template <bool LDSV>
__global__ void __launch_bounds__(NT) mlp3_wgrad_kernel(WgradArgs a) {
  if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x * 8] = __builtin_amdgcn_s_memrealtime();
  __shared__ __attribute__((aligned(1024))) char stage[LDSV ? NW * 16384 : NW * 32 * 32 * 4];
  float (*red)[32 * 32] = (float (*)[32 * 32])stage;  // (LDSV: reused once the staged operands are read)
  __shared__ float rsum[NW][32];
  __shared__ rk_opt::AdamStep s_ks[kEpiGroups];
  __shared__ float s_cnt[NW];
  // optimizer epilogue: the step counter is loaded now but consumed only where each block type
  // already synchronises (its LDS reduction), so its memory round trip overlaps the gradient loads
  // instead of preceding them; likewise the count partials of a normalising launch
  const float cur = a.epi.on ? a.epi.step[0] : 0.f;
  // the optimizer step counter's ticket, taken when the block STARTS: the block that arrives last
  // advances the counter at its end (rk_opt::advance_step takes it at the end, so every block's
  // tail waited one agent-scope atomic round trip).  Every block has read `cur` long before: the
  // last block's store comes after its whole tile, microseconds after all tickets (and the loads
  // issued before them) were taken.
  // (an LDS-staged dW tile block takes it later, right after its operands landed: taken here, the
  // atomic's round trip on the one contended counter sat inside that block's operand wait)
  unsigned ticket = 0;
  const bool late_ticket = LDSV && a.late_ticket && !(a.has_rows && (int)blockIdx.x == (int)gridDim.x - 1) && (int)blockIdx.x < a.tiles;
  if (a.epi.on && threadIdx.x == 0 && !late_ticket)
    ticket = __hip_atomic_fetch_add(a.epi.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float cpart = 0.f;
  if (a.cnt_parts)
    for (int i = threadIdx.x; i < a.ncnt; i += NT) cpart += a.cnt_parts[i];
  // the hyperparameters too: read here, their latency hides under the tile's loads (read in sf(),
  // after the MFMA loop, they were one more memory round trip on every block's tail)
  rk_opt::AdamHyper hy{};
  if (a.epi.on && threadIdx.x < kEpiGroups) hy = a.epi.hyper[threadIdx.x < a.epi.on ? threadIdx.x : 0];
  const StepFill sf{&a, cur, s_ks, cpart, s_cnt, hy};
  const rk_opt::AdamStep* ks = a.epi.on ? s_ks : nullptr;
  if (a.has_rows && (int)blockIdx.x == (int)gridDim.x - 1) {
    // the step's batch cursor (no gradient work; still takes the optimizer step's ticket below)
    rows_next_block(a.rn_table, a.rn_meta, a.rn_rows, a.rn_cur, a.rn_bs);
  } else if ((int)blockIdx.x >= a.tiles) {
    if ((int)blockIdx.x - a.tiles < a.nslab) slab_reduce_block(a, blockIdx.x - a.tiles, red, ks, sf);
    else loss_fin_block(a.lf, red, sf);
  } else {
    wgrad_tile<LDSV>(a, red, rsum, ks, sf, stage, late_ticket ? &ticket : nullptr);
  }
  if (a.epi.on && threadIdx.x == 0 && ticket == gridDim.x - 1) {
    a.epi.step[0] = cur + 1.f;
    __hip_atomic_store(a.epi.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x * 8 + 2] = __builtin_amdgcn_s_memrealtime();
}

template <bool LDSV>
__device__ void wgrad_tile(const WgradArgs& a, float (*red)[32 * 32], float (*rsum)[32], const rk_opt::AdamStep* ks,
                           const StepFill& sf, char* stage, unsigned* ticket) {
  int pi = 0;
#pragma unroll
  for (int i = 1; i < 3; ++i)
    if (i < a.nprob && (int)blockIdx.x >= a.p[i].tile_begin) pi = i;
  const WgradProb P = a.p[pi];
  const int t = blockIdx.x - P.tile_begin;
  const int n0 = (t / P.tiles_k) * WTN, k0 = (t % P.tiles_k) * 32;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, lo = lane & 15, hi = lane >> 4;
  const int per = ((a.M + NW * 64 - 1) / (NW * 64)) * 64;  // batch range per wave, multiple of 64
  const int mb = wv * per, me = min(a.M, mb + per);
  // this block is the only writer of its dW tile / db rows: read their old values up front so the
  // final accumulate does not wait on a memory round trip
  float dw_old[WEPT];
  rk_opt::EpiElem ew[WEPT], eb{};
#pragma unroll
  for (int q = 0; q < WEPT; ++q) {
    const int e = threadIdx.x + q * NT, r = e >> 5, c = e & 31;
    const bool in = n0 + r < P.N && k0 + c < P.K;
    dw_old[q] = in ? P.dw[(int64_t)(n0 + r) * P.K + k0 + c] : 0.f;
    if (ks && in) ew[q] = rk_opt::epi_fetch(a.rdw[pi], (int64_t)(n0 + r) * P.K + k0 + c);
  }
  if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x * 8 + 3] = __builtin_amdgcn_s_memrealtime() + (uint64_t)(dw_old[0] == 12345.f);
  const bool has_db = k0 == 0 && P.db && threadIdx.x < WTN && n0 + (int)threadIdx.x < P.N;
  const float db_old = has_db ? P.db[n0 + threadIdx.x] : 0.f;
  if (ks && has_db) eb = rk_opt::epi_fetch(a.rdb[pi], n0 + threadIdx.x);
  f32x4 acc[WNI][2];
  float rs[WNI];
#pragma unroll
  for (int i = 0; i < WNI; ++i) {
    rs[i] = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (LDSV) {
#if defined(__HIP_DEVICE_COMPILE__)
    // wave region: [WTN d rows][256 B] then [32 x rows][256 B]; row r's 16-B chunk c at c ^ (r & 15)
    // (the 16 rows a ds_read_b128 lane group reads hit 16 different bank slots); the LDS-DMA image
    // is lane-linear, so the swizzle is applied to each lane's SOURCE chunk
    char* const wst = stage + wv * 16384;
    constexpr int QD = WTN / 4;  // 1-KiB pieces of d rows
#pragma unroll
    for (int q = 0; q < QD + 8; ++q) {  // 1 KiB each: 4 rows x 256 B
      const int r = 4 * (q < QD ? q : q - QD) + (lane >> 4), c = lane & 15;
      const uint16_t* T = q < QD ? P.dT : P.xT;
      const int R = q < QD ? P.N : P.K, r0 = q < QD ? n0 : k0;
      const int gr = min(r0 + r, R - 1);  // rows past the edge: any valid row (their outputs are not stored)
      const uint16_t* src = T + (int64_t)gr * a.M + mb + 8 * (c ^ (r & 15));
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(wst + q * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" ::: "memory");
    // the optimizer step's ticket (see the kernel): its round trip overlaps the MFMAs and the
    // reduction; the value is needed only at the block's end
    if (ticket && a.epi.on && threadIdx.x == 0)
      *ticket = __hip_atomic_fetch_add(a.epi.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      bf16x8 af[WNI], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ra = 16 * i + lo;
        if (i < WNI) af[i] = *(const bf16x8*)(wst + ra * 256 + (((4 * s4 + hi) ^ (ra & 15)) * 16));
        bf[i] = *(const bf16x8*)(wst + WTN * 256 + ra * 256 + (((4 * s4 + hi) ^ (ra & 15)) * 16));
      }
#pragma unroll
      for (int i = 0; i < WNI; ++i) {
        const bool rin = n0 + 16 * i + lo < P.N;  // clamped rows must not enter the row sums
        const uint4 aw = __builtin_bit_cast(uint4, af[i]);
        const uint32_t awd[4] = {aw.x, aw.y, aw.z, aw.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rs[i] += rin ? d16((uint16_t)(awd[j] & 0xffffu)) + d16((uint16_t)(awd[j] >> 16)) : 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
      }
    }
    __syncthreads();  // every wave done with its staged operands: `red` (aliased) may be written
#endif
  } else
  for (int m = mb; m < me; m += 128) {  // four k-steps per iteration, all loads issued first
    bf16x8 af[4][WNI], bf[4][2];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int mk = m + 32 * s + 8 * hi;
      const int mm = mk < me ? mk : a.M;  // a.M -> zero fragment
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i < WNI) af[s][i] = rowfrag(P.dT, P.N, a.M, n0 + 16 * i + lo, mm);
        bf[s][i] = rowfrag(P.xT, P.K, a.M, k0 + 16 * i + lo, mm);
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int i = 0; i < WNI; ++i) {
        // (the fragment's elements via its dwords: a per-element __bf16 -> uint16_t bit_cast of
        // the vector's lanes miscompiles under -O3 to element 0 eight times)
        const uint4 aw = __builtin_bit_cast(uint4, af[s][i]);
        const uint32_t awd[4] = {aw.x, aw.y, aw.z, aw.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rs[i] += d16((uint16_t)(awd[j] & 0xffffu)) + d16((uint16_t)(awd[j] >> 16));
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[s][i], bf[s][j], acc[i][j]);
      }
    }
  }
  if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x * 8 + 4] = __builtin_amdgcn_s_memrealtime() + (uint64_t)(acc[0][0][0] == 12345.f);
  // reduce the 8 waves' partial tiles in LDS; C element (row 16i + 4hi + r, col 16j + lo)
#pragma unroll
  for (int i = 0; i < WNI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wv][(16 * i + 4 * hi + r) * 32 + 16 * j + lo] = acc[i][j][r];
  // row sums of d^T (bias gradient): lanes lo, lo+16, lo+32, lo+48 hold parts of row 16i + lo
#pragma unroll
  for (int i = 0; i < WNI; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
    if (hi == 0) rsum[wv][16 * i + lo] = rs[i];
  }
  sf();
  __syncthreads();
  if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memrealtime();
  const float gsc = sf.gs();
#pragma unroll
  for (int q = 0; q < WEPT; ++q) {
    const int e = threadIdx.x + q * NT, r = e >> 5, c = e & 31;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][e];
    v *= gsc;
    if (n0 + r < P.N && k0 + c < P.K) {
      const int64_t i = (int64_t)(n0 + r) * P.K + k0 + c;
      if (ks) rk_opt::epi_apply(a.rdw[pi], ks[a.rdw[pi].group], i, ew[q], dw_old[q] + v, a.epi.zero_grads);
      else P.dw[i] = dw_old[q] + v;
      flag_nonfinite(a.amp_found, dw_old[q] + v);
    }
  }
  if (has_db) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += rsum[w][threadIdx.x];
    v *= gsc;
    if (ks) rk_opt::epi_apply(a.rdb[pi], ks[a.rdb[pi].group], n0 + threadIdx.x, eb, db_old + v, a.epi.zero_grads);
    else P.db[n0 + threadIdx.x] = db_old + v;
    flag_nonfinite(a.amp_found, db_old + v);
  }
}

}  // namespace

// The NEXT rk_mlp3_wgrad_loss on this thread also advances a deferred loader batch's cursor and
// stages the next batch's rows (one extra block; rows_common.h): the step that consumed the batch
// ends with its cursor step instead of a launch of its own.
struct RowsReq {
  const int64_t* table;
  int64_t* meta;
  int64_t* rows;
  int n_cur, bs;
};
static thread_local RowsReq g_rows{};
// Likewise the NEXT rk_mlp3_wgrad_loss flags non-finite gradients into *found (WgradArgs::amp_found).
static thread_local float* g_amp_found = nullptr;
RK_API int RKL_NAME(rk_mlp3_set_amp_found)(float* found) {
  g_amp_found = found;
  return 0;
}
RK_API int RKL_NAME(rk_mlp3_set_rows)(const int64_t* table, int64_t* meta, int64_t* rows, int n_cur, int bs) {
  if (!table || !meta || !rows || n_cur < 0 || bs < 1) return (int)hipErrorInvalidValue;
  g_rows = RowsReq{table, meta, rows, n_cur, bs};
  return 0;
}

// Diagnostics: per-block phase stamps of the grouped weight-gradient launch ([blocks][8] u64, or
// null = off): start, operands reduced (after the block's LDS barrier), end; tiles also: old values
// loaded, main loop done.
#if RK_LENET_H
extern uint64_t* g_wgrad_trace;
#else
uint64_t* g_wgrad_trace = nullptr;
RK_API void rk_mlp3_set_trace(void* tr) { g_wgrad_trace = (uint64_t*)tr; }
#endif

// K0, N1, N2 must be multiples of 4 (16-byte weight rows); widths <= 512.
RK_API int RKL_NAME(rk_mlp3_fwd)(const void* x, int K0, const float* w1, const float* b1, int N1, const float* w2,
                       const float* b2, int N2, const float* w3, const float* b3, int N3, void* xT, void* h1T,
                       void* h2T, float* y, int M, hipStream_t s) {
  if (K0 > MAXK || N1 > MAXK || N2 > MAXK || N3 > MAXK) return (int)hipErrorInvalidValue;
  if ((K0 & 3) || (N1 & 3) || (N2 & 3)) return (int)hipErrorInvalidValue;
  const int grid = (M + ROWS - 1) / ROWS;
  const int k1 = (K0 + 31) / 32, k2 = (N1 + 31) / 32, k3 = (N2 + 31) / 32;
#define RK_F(A, B, C) mlp3_fwd_kernel<A, B, C><<<grid, NT, 0, s>>>((const uint16_t*)x, K0, w1, b1, N1, w2, b2, N2, w3, b3, N3, (uint16_t*)xT, (uint16_t*)h1T, (uint16_t*)h2T, y, M)
  if (k1 == 13 && k2 == 4 && k3 == 3) RK_F(13, 4, 3);  // LeNet 400-120-84-10
  else RK_F(0, 0, 0);
#undef RK_F
  return (int)hipGetLastError();
}

RK_API int RKL_NAME(rk_mlp3_dgrad)(const float* dy, int N3, const float* w3, int N2, const void* h2T, const float* w2, int N1,
                         const void* h1T, const float* w1, int K0, void* dyT, void* d2T, void* d1T, void* dx, int M,
                         hipStream_t s) {
  if (K0 > MAXK || N1 > MAXK || N2 > MAXK || N3 > MAXK) return (int)hipErrorInvalidValue;
  const int grid = (M + ROWS - 1) / ROWS;
  const int k3 = (N3 + 31) / 32, k2 = (N2 + 31) / 32, k1 = (N1 + 31) / 32;
#define RK_D(A, B, C) mlp3_dgrad_kernel<A, B, C><<<grid, NT, 0, s>>>(dy, N3, w3, N2, (const uint16_t*)h2T, w2, N1, (const uint16_t*)h1T, w1, K0, (uint16_t*)dyT, (uint16_t*)d2T, (uint16_t*)d1T, (uint16_t*)dx, M)
  if (k3 == 1 && k2 == 3 && k1 == 4) RK_D(1, 3, 4);
  else RK_D(0, 0, 0);
#undef RK_D
  return (int)hipGetLastError();
}

// Grouped dW_l += dT_l . xT_l^T, db_l += rowsum(dT_l) for up to 3 layers. M % 8 == 0.
// slab (may be null): also dst[i][c - bound[i]] += sum over the slab_rows rows of slab[r][c] for
// c in [bound[i], bound[i+1]), bound[0] = 0, c < bound[4] <= slab_width.
// Host description of the optimizer epilogue (see rk_opt::AdamEpi): records of the parameters
// whose gradients the launch produces, in the order dW[3], db[3] (the problems) and slab dst[4].
struct WgradEpi {
  const void* hyper;  // AdamHyper[ngroups]
  float* step;
  unsigned* counter;
  int ngroups, zero_grads;
  rk_opt::TensorRec rdw[3], rdb[3], rsl[4];
};

// loss (may be null): also finalise a batch loss from per-block partials (see LossFin).
// epi (may be null): apply the Adam/AdamW update to every produced gradient element (the step's
// optimizer launch is then skipped by the caller).  Every dW/db/slab destination needs a record.
// gscale: factor on every produced gradient (1 unless the backward inputs were formed for a unit
// upstream gradient, e.g. by the fused LeNet step kernel ahead of the loss scaling).
// norm_by_count: the backward scaled by 1 / M instead of the loss's 1 / (valid count) and stored
// per-block valid counts after its loss partials (loss->partials[nparts ..]): gradients are scaled
// by M / their sum, the loss divided by it.
RK_API int RKL_NAME(rk_mlp3_wgrad_loss)(int nprob, const void* const* dT, const void* const* xT, float* const* dw,
                              float* const* db, const int* Ns, const int* Ks, int M, const float* slab, int slab_rows,
                              int slab_width, float* const* slab_dst, const int* slab_bound, const LossFin* loss,
                              const WgradEpi* epi, float gscale, int norm_by_count, hipStream_t s) {
  // the staged rows request (rk_mlp3_set_rows) belongs to THIS call whatever happens: taken and
  // cleared first, so an argument error below cannot leave it attached to a later launch
  const RowsReq rows_req = g_rows;
  g_rows = RowsReq{};
  float* const amp_found = g_amp_found;
  g_amp_found = nullptr;
  if (nprob < 1 || nprob > 3 || (M & 7)) return (int)hipErrorInvalidValue;
  WgradArgs a{};
  a.trace = g_wgrad_trace;
  static const int late_env = getenv("ROCKET_WGRAD_LATE_TICKET") ? atoi(getenv("ROCKET_WGRAD_LATE_TICKET")) : 1;
  a.late_ticket = late_env;
  a.gscale = gscale;
  a.amp_found = amp_found;
  if (norm_by_count) {  // count partials follow the loss partials: partials[nparts .. 2 nparts)
    if (!loss) return (int)hipErrorInvalidValue;
    a.cnt_parts = loss->partials + loss->nparts;
    a.ncnt = loss->nparts;
  }
  a.nprob = nprob;
  a.M = M;
  int tiles = 0;
  for (int i = 0; i < 3; ++i) {
    const int j = i < nprob ? i : nprob - 1;
    a.p[i].dT = (const uint16_t*)dT[j];
    a.p[i].xT = (const uint16_t*)xT[j];
    a.p[i].dw = dw[j];
    a.p[i].db = db[j];
    a.p[i].N = Ns[j];
    a.p[i].K = Ks[j];
    a.p[i].tiles_k = (Ks[j] + 31) / 32;
    a.p[i].tile_begin = tiles;
    if (i < nprob) tiles += ((Ns[j] + WTN - 1) / WTN) * a.p[i].tiles_k;
  }
  a.tiles = tiles;
  int extra = 0;
  if (slab) {
    if (slab_rows < 1 || slab_bound[0] != 0 || slab_bound[4] > slab_width) return (int)hipErrorInvalidValue;
    a.sl.slab = slab;
    a.sl.rows = slab_rows;
    a.sl.width = slab_width;
    a.sl.ncols = slab_bound[4];
    for (int i = 0; i < 4; ++i) a.sl.dst[i] = slab_dst[i];
    for (int i = 0; i < 5; ++i) a.sl.bound[i] = slab_bound[i];
    extra = (a.sl.ncols + SLC - 1) / SLC;
  }
  a.nslab = extra;
  if (loss) {
    if (!loss->partials || !loss->loss_out || loss->nparts < 1 || (loss->acc && (!loss->ring || !loss->slot || loss->ring_size < 1)))
      return (int)hipErrorInvalidValue;
    a.has_loss = 1;
    a.lf = *loss;
    extra += 1;
  }
  if (epi) {
    if (!epi->hyper || !epi->step || !epi->counter || epi->ngroups < 1 || epi->ngroups > kEpiGroups || nprob != 3 ||
        !slab)
      return (int)hipErrorInvalidValue;
    a.epi.hyper = (const rk_opt::AdamHyper*)epi->hyper;
    a.epi.step = epi->step;
    a.epi.counter = epi->counter;
    a.epi.on = epi->ngroups;
    a.epi.zero_grads = epi->zero_grads;
    for (int i = 0; i < 3; ++i) {
      a.rdw[i] = epi->rdw[i];
      a.rdb[i] = epi->rdb[i];
      // each record must describe the very gradient buffer this launch writes
      if ((float*)a.rdw[i].g != dw[i] || (float*)a.rdb[i].g != db[i] || a.rdw[i].group >= epi->ngroups ||
          a.rdb[i].group >= epi->ngroups)
        return (int)hipErrorInvalidValue;
    }
    for (int i = 0; i < 4; ++i) {
      a.rsl[i] = epi->rsl[i];
      if ((float*)a.rsl[i].g != slab_dst[i] || a.rsl[i].group >= epi->ngroups) return (int)hipErrorInvalidValue;
    }
  }
  if (rows_req.table) {  // the staged rows request: one more block of this launch
    a.rn_table = rows_req.table;
    a.rn_meta = rows_req.meta;
    a.rn_rows = rows_req.rows;
    a.rn_cur = rows_req.n_cur;
    a.rn_bs = rows_req.bs;
    a.has_rows = 1;
    extra += 1;
  }
  // LDS-staged tile operands (mlp3_wgrad_kernel<true>) when every wave's batch range is 128 rows;
  // ROCKET_WGRAD_LDS=0 keeps the fragment-shaped global loads
  static const int lds_env = getenv("ROCKET_WGRAD_LDS") ? atoi(getenv("ROCKET_WGRAD_LDS")) : 1;
  if (lds_env && M == NW * 128) mlp3_wgrad_kernel<true><<<tiles + extra, NT, 0, s>>>(a);
  else mlp3_wgrad_kernel<false><<<tiles + extra, NT, 0, s>>>(a);
  return (int)hipGetLastError();
}

RK_API int RKL_NAME(rk_mlp3_wgrad)(int nprob, const void* const* dT, const void* const* xT, float* const* dw, float* const* db,
                         const int* Ns, const int* Ks, int M, const float* slab, int slab_rows, int slab_width,
                         float* const* slab_dst, const int* slab_bound, hipStream_t s) {
  return RKL_NAME(rk_mlp3_wgrad_loss)(nprob, dT, xT, dw, db, Ns, Ks, M, slab, slab_rows, slab_width, slab_dst, slab_bound,
                            nullptr, nullptr, 1.f, 0, s);
}
