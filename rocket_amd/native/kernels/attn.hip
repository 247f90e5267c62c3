// Fused multi-head attention for short sequences (ViT: L = 197 tokens, head dim 64), bf16 in/out,
// fp32 accumulation on v_mfma_f32_16x16x32_bf16 (BASELINE ViT-B/16 config).
//
// Layout: q/k/v are read straight from the QKV projection output [B*L, 3*H*D] (token-major,
// per-head column blocks) and the output / input gradients are written in the same token-major
// layout — the head split/merge permutes of the composite path never materialise.
//
// Whole-row softmax: a key sequence of <= 224 tokens fits in one tile row, so every kernel keeps
// all keys of a head in LDS and needs no online-softmax rescaling:
//   attn_fwd   block = (head, batch): K/V staged once, the 4 waves loop over 16-query tiles.  S = Q K^T (13 MFMA tiles
//              in registers), row max/sum by 16-lane shuffles, P (bf16) through a wave-private LDS
//              tile into O = P V; writes O and the row log-sum-exp (log2 domain).
//   attn_bwd_q same decomposition: recompute P from the saved LSE, dP = dO V^T, dS = P (dP - delta) * scale,
//              dQ = dS K; also writes delta = rowsum(dO * O) for attn_bwd_kv.
//   attn_bwd_kv block = (head, batch), waves loop over 16-key tiles: S^T = K Q^T and dP^T = V dO^T over
//              all queries, dV = P^T dO, then dK = dS^T Q (P^T / dS^T reuse one LDS tile).
// All operand fragments are 16-byte LDS reads (row-major copies for "consecutive d" operands,
// transposed copies for "consecutive token" operands; row strides 72 / 232 bf16 keep the 16 rows
// of a fragment on distinct banks).
#include "rk_common.h"

using namespace rk;

namespace {

constexpr int D = 64;
constexpr int LMAX = 224;        // max tokens (K-dim padded to 32)
constexpr int RS = D + 8;        // row-major stride (72)
constexpr int TS = LMAX + 8;     // transposed stride (232)
constexpr int NTH = 256;         // 4 waves
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const uint16_t* q;   // token-major, row stride ld (elements), head h at column h*D
  const uint16_t* k;
  const uint16_t* v;
  const uint16_t* o;   // forward output (bwd), row stride ldo
  const uint16_t* dout;
  uint16_t* out;       // fwd: O;  bwd: dQ / dK / dV base (row stride ldg)
  uint16_t* dq;
  uint16_t* dk;
  uint16_t* dv;
  float* lse;          // [B*H][L], log2 domain
  float* delta;        // [B*H][L]
  int ld, ldo, ldg;
  int L, H;
  float scale;         // softmax scale (1/sqrt(D))
};

__device__ __forceinline__ bf16x8 ld16(const uint16_t* p) { return *(const bf16x8*)p; }
__device__ __forceinline__ bf16x8 zero8() { return bf16x8{}; }

// global token row r of head h (clamped + selected: branch-free, always a valid address)
__device__ __forceinline__ bf16x8 gload_row(const uint16_t* base, int ld, int b, int L, int r, int h, int c) {
  const int rc = r < L ? r : L - 1;
  const bf16x8 v = ld16(base + ((int64_t)b * L + rc) * ld + h * D + c);
  return r < L ? v : zero8();
}

// stage [LMAX][RS] row-major copy of a head's tokens (zero rows >= L)
__device__ __forceinline__ void stage_rows(uint16_t* dst, const uint16_t* src, int ld, int b, int L, int h) {
  for (int i = threadIdx.x; i < LMAX * (D / 8); i += NTH) {
    const int r = i >> 3, c = (i & 7) * 8;
    *(bf16x8*)(dst + r * RS + c) = gload_row(src, ld, b, L, r, h, c);
  }
}

// stage [D][TS] transposed copy (token index contiguous), zero tokens >= L
__device__ __forceinline__ void stage_trans(uint16_t* dst, const uint16_t* src, int ld, int b, int L, int h) {
  for (int i = threadIdx.x; i < LMAX * (D / 8); i += NTH) {
    const int r = i >> 3, c = (i & 7) * 8;
    const int rc = r < L ? r : L - 1;
    uint4 u = *(const uint4*)(src + ((int64_t)b * L + rc) * ld + h * D + c);
    if (r >= L) u = make_uint4(0, 0, 0, 0);
    const uint32_t wds[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      dst[(c + 2 * e) * TS + r] = (uint16_t)(wds[e] & 0xffffu);
      dst[(c + 2 * e + 1) * TS + r] = (uint16_t)(wds[e] >> 16);
    }
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float red16_max(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float red16_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int NT = LMAX / 16;  // 14 key tiles max

// --------------------------------------------------------------------------------- forward
__global__ void __launch_bounds__(NTH) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[D * TS];
  __shared__ __attribute__((aligned(16))) uint16_t Ps[4][16 * TS];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lo = lane & 15, hi = lane >> 4;
  const int L = a.L;
  const int ntile = (L + 15) / 16;
  stage_rows(Ks, a.k, a.ld, b, L, h);
  stage_trans(Vt, a.v, a.ld, b, L, h);
  for (int i = lane; i < 16 * TS; i += 64) Ps[w][i] = 0;  // zero pads (cols >= 16*ntile)
  __syncthreads();

  const float sl = a.scale * LOG2E;
  // the block owns every query tile of its (batch, head): K/V are staged once per head
  for (int qt = w; qt < ntile; qt += 4) {
  const int q0 = 16 * qt;
  bf16x8 qa[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) qa[ks] = gload_row(a.q, a.ld, b, L, q0 + lo, h, 32 * ks + 8 * hi);
  f32x4 s[NT];
  float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t < ntile) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], ld16(Ks + (16 * t + lo) * RS + 32 * ks + 8 * hi), s[t], 0, 0, 0);
      const bool valid = 16 * t + lo < L;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[t][i] = valid ? s[t][i] * sl : -INFINITY;
        m[i] = fmaxf(m[i], s[t][i]);
      }
    }
  }
  float sum[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m[i] = red16_max(m[i]);
    sum[i] = 0.f;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t < ntile) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = exp2f(s[t][i] - m[i]);
        sum[i] += p;
        Ps[w][(4 * hi + i) * TS + 16 * t + lo] = f2bf(p);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) sum[i] = red16_sum(sum[i]);
  wave_lds_sync();

  const int kst = (16 * ntile + 31) / 32;
  f32x4 o[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) o[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < kst; ++ks) {
    const bf16x8 pa = ld16(&Ps[w][lo * TS + 32 * ks + 8 * hi]);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      o[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, ld16(Vt + (16 * nt + lo) * TS + 32 * ks + 8 * hi), o[nt], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = q0 + 4 * hi + i;
    if (r < L) {
      const float inv = 1.f / sum[i];
      uint16_t* orow = a.out + ((int64_t)b * L + r) * a.ldo + h * D;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) orow[16 * nt + lo] = f2bf(o[nt][i] * inv);
      if (lo == 0) a.lse[((int64_t)b * a.H + h) * L + r] = m[i] + log2f(sum[i]);
    }
  }
  wave_lds_sync();  // P of this tile fully consumed before the next tile overwrites it
  }
}

// ------------------------------------------------------------------------------- backward: dQ
__global__ void __launch_bounds__(NTH) attn_bwd_q_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Kt[D * TS];
  __shared__ __attribute__((aligned(16))) uint16_t Ss[4][16 * TS];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lo = lane & 15, hi = lane >> 4;
  const int L = a.L;
  const int ntile = (L + 15) / 16;
  stage_rows(Ks, a.k, a.ld, b, L, h);
  stage_rows(Vs, a.v, a.ld, b, L, h);
  stage_trans(Kt, a.k, a.ld, b, L, h);
  for (int i = lane; i < 16 * TS; i += 64) Ss[w][i] = 0;
  __syncthreads();

  for (int qt = w; qt < ntile; qt += 4) {
  const int q0 = 16 * qt;
  bf16x8 qa[2], ga[2];
  float dot = 0.f;  // partial rowsum(dO * O) of row q0 + lo over this lane's 16 d values
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    qa[ks] = gload_row(a.q, a.ld, b, L, q0 + lo, h, 32 * ks + 8 * hi);
    ga[ks] = gload_row(a.dout, a.ldo, b, L, q0 + lo, h, 32 * ks + 8 * hi);
    const bf16x8 ov = gload_row(a.o, a.ldo, b, L, q0 + lo, h, 32 * ks + 8 * hi);
    const uint4 gu = __builtin_bit_cast(uint4, ga[ks]), ou = __builtin_bit_cast(uint4, ov);
    const uint32_t gw[4] = {gu.x, gu.y, gu.z, gu.w}, ow[4] = {ou.x, ou.y, ou.z, ou.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      dot += __uint_as_float(gw[e] << 16) * __uint_as_float(ow[e] << 16) +
             __uint_as_float(gw[e] & 0xffff0000u) * __uint_as_float(ow[e] & 0xffff0000u);
  }
  dot += __shfl_xor(dot, 16, 64);
  dot += __shfl_xor(dot, 32, 64);  // every lane with this lo holds delta(row q0 + lo)
  const int64_t bh = (int64_t)b * a.H + h;
  if (hi == 0 && q0 + lo < L) a.delta[bh * L + q0 + lo] = dot;
  // per C-layout row r = 4hi + i: delta and lse of query q0 + r
  float dl[4], ls[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dl[i] = __shfl(dot, 4 * hi + i, 64);
    const int r = q0 + 4 * hi + i;
    ls[i] = a.lse[bh * L + (r < L ? r : L - 1)];
  }
  const float sl = a.scale * LOG2E;
#pragma unroll 2
  for (int t = 0; t < ntile; ++t) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], ld16(Ks + (16 * t + lo) * RS + 32 * ks + 8 * hi), s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga[ks], ld16(Vs + (16 * t + lo) * RS + 32 * ks + 8 * hi), dp, 0, 0, 0);
    }
    const bool valid = 16 * t + lo < L;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = valid ? exp2f(s[i] * sl - ls[i]) : 0.f;
      Ss[w][(4 * hi + i) * TS + 16 * t + lo] = f2bf(p * (dp[i] - dl[i]) * a.scale);
    }
  }
  wave_lds_sync();
  const int kst = (16 * ntile + 31) / 32;
  f32x4 dq[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) dq[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < kst; ++ks) {
    const bf16x8 sa = ld16(&Ss[w][lo * TS + 32 * ks + 8 * hi]);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      dq[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, ld16(Kt + (16 * nt + lo) * TS + 32 * ks + 8 * hi), dq[nt], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = q0 + 4 * hi + i;
    if (r < L) {
      uint16_t* row = a.dq + ((int64_t)b * L + r) * a.ldg + h * D;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) row[16 * nt + lo] = f2bf(dq[nt][i]);
    }
  }
  wave_lds_sync();
  }
}

// --------------------------------------------------------------------------- backward: dK, dV
__global__ void __launch_bounds__(NTH) attn_bwd_kv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Qs[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Gs[LMAX * RS];  // dO row-major
  __shared__ __attribute__((aligned(16))) uint16_t Qt[D * TS];
  __shared__ __attribute__((aligned(16))) uint16_t Gt[D * TS];     // dO transposed
  __shared__ __attribute__((aligned(16))) uint16_t Ts[4][16 * TS]; // P^T, then dS^T
  __shared__ float lse_s[LMAX], del_s[LMAX];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lo = lane & 15, hi = lane >> 4;
  const int L = a.L;
  const int ntile = (L + 15) / 16;
  const int64_t bh = (int64_t)b * a.H + h;
  stage_rows(Qs, a.q, a.ld, b, L, h);
  stage_rows(Gs, a.dout, a.ldo, b, L, h);
  stage_trans(Qt, a.q, a.ld, b, L, h);
  stage_trans(Gt, a.dout, a.ldo, b, L, h);
  for (int i = threadIdx.x; i < LMAX; i += NTH) {
    lse_s[i] = i < L ? a.lse[bh * L + i] : 0.f;
    del_s[i] = i < L ? a.delta[bh * L + i] : 0.f;
  }
  for (int i = lane; i < 16 * TS; i += 64) Ts[w][i] = 0;
  __syncthreads();

  const float sl = a.scale * LOG2E;
  for (int kt = w; kt < ntile; kt += 4) {
  const int k0 = 16 * kt;
  bf16x8 ka[2], va[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    ka[ks] = gload_row(a.k, a.ld, b, L, k0 + lo, h, 32 * ks + 8 * hi);
    va[ks] = gload_row(a.v, a.ld, b, L, k0 + lo, h, 32 * ks + 8 * hi);
  }
  const int kst = (16 * ntile + 31) / 32;
  // pass 1: P^T (rows = keys 4hi+i, cols = queries) -> dV = P^T dO
#pragma unroll 2
  for (int t = 0; t < ntile; ++t) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[ks], ld16(Qs + (16 * t + lo) * RS + 32 * ks + 8 * hi), s, 0, 0, 0);
    const int qi = 16 * t + lo;
    const float lq = lse_s[qi];
#pragma unroll
    for (int i = 0; i < 4; ++i) Ts[w][(4 * hi + i) * TS + qi] = f2bf(qi < L ? exp2f(s[i] * sl - lq) : 0.f);
  }
  wave_lds_sync();
  f32x4 acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < kst; ++ks) {
    const bf16x8 pa = ld16(&Ts[w][lo * TS + 32 * ks + 8 * hi]);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, ld16(Gt + (16 * nt + lo) * TS + 32 * ks + 8 * hi), acc[nt], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = k0 + 4 * hi + i;
    if (r < L) {
      uint16_t* row = a.dv + ((int64_t)b * L + r) * a.ldg + h * D;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) row[16 * nt + lo] = f2bf(acc[nt][i]);
    }
  }
  wave_lds_sync();  // every lane finished reading P^T before it is overwritten with dS^T
  // pass 2: dS^T = P^T (dP^T - delta) * scale, dP^T = V dO^T -> dK = dS^T Q
#pragma unroll 2
  for (int t = 0; t < ntile; ++t) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[ks], ld16(Qs + (16 * t + lo) * RS + 32 * ks + 8 * hi), s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va[ks], ld16(Gs + (16 * t + lo) * RS + 32 * ks + 8 * hi), dp, 0, 0, 0);
    }
    const int qi = 16 * t + lo;
    const float lq = lse_s[qi], dq = del_s[qi];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = qi < L ? exp2f(s[i] * sl - lq) : 0.f;
      Ts[w][(4 * hi + i) * TS + qi] = f2bf(p * (dp[i] - dq) * a.scale);
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < kst; ++ks) {
    const bf16x8 sa = ld16(&Ts[w][lo * TS + 32 * ks + 8 * hi]);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, ld16(Qt + (16 * nt + lo) * TS + 32 * ks + 8 * hi), acc[nt], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = k0 + 4 * hi + i;
    if (r < L) {
      uint16_t* row = a.dk + ((int64_t)b * L + r) * a.ldg + h * D;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) row[16 * nt + lo] = f2bf(acc[nt][i]);
    }
  }
  wave_lds_sync();
  }
}

}  // namespace

RK_API int rk_attn_max_len() { return LMAX; }

// q/k/v: bf16 token-major (row stride ld elements), out: [B*L][ldo] with head h at column h*64;
// lse: [B*H][L] f32.  head dim 64, L <= 224.
RK_API int rk_attn_fwd(const void* q, const void* k, const void* v, int ld, void* out, int ldo, float* lse, int B,
                       int L, int H, float scale, hipStream_t s) {
  if (L < 1 || L > LMAX || B < 1 || H < 1) return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = (const uint16_t*)q; a.k = (const uint16_t*)k; a.v = (const uint16_t*)v;
  a.out = (uint16_t*)out; a.lse = lse; a.ld = ld; a.ldo = ldo; a.L = L; a.H = H; a.scale = scale;
  dim3 grid(1, H, B);  // one block per (batch, head)
  attn_fwd_kernel<<<grid, NTH, 0, s>>>(a);
  return (int)hipGetLastError();
}

// gradients dq/dk/dv written token-major with row stride ldg (e.g. into one [B*L][3*H*64] buffer);
// delta: [B*H][L] f32 scratch.
RK_API int rk_attn_bwd(const void* q, const void* k, const void* v, int ld, const void* o, const void* dout, int ldo,
                       const float* lse, float* delta, void* dq, void* dk, void* dv, int ldg, int B, int L, int H,
                       float scale, hipStream_t s) {
  if (L < 1 || L > LMAX || B < 1 || H < 1) return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = (const uint16_t*)q; a.k = (const uint16_t*)k; a.v = (const uint16_t*)v;
  a.o = (const uint16_t*)o; a.dout = (const uint16_t*)dout;
  a.dq = (uint16_t*)dq; a.dk = (uint16_t*)dk; a.dv = (uint16_t*)dv;
  a.lse = (float*)lse; a.delta = delta;
  a.ld = ld; a.ldo = ldo; a.ldg = ldg; a.L = L; a.H = H; a.scale = scale;
  dim3 grid(1, H, B);
  attn_bwd_q_kernel<<<grid, NTH, 0, s>>>(a);
  attn_bwd_kv_kernel<<<grid, NTH, 0, s>>>(a);
  return (int)hipGetLastError();
}
