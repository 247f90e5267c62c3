// Fused multi-head attention for short sequences (ViT: L = 197 tokens, head dim 64), bf16 in/out,
// fp32 accumulation on v_mfma_f32_16x16x32_bf16 (BASELINE ViT-B/16 config).
//
// Layout: q/k/v are read straight from the QKV projection output [B*L, 3*H*D] (token-major,
// per-head column blocks) and the output / input gradients are written in the same token-major
// layout — the head split/merge permutes of the composite path never materialise.
//
// Whole-row softmax: a key sequence of <= 224 tokens fits in one tile row, so no online-softmax
// rescaling.  Every kernel is "operand-on-the-lane": the score tile is computed with the token
// whose softmax/reduction axis is NOT summed next on the MFMA lane, so the accumulator of one
// product is already (lane-locally) the operand of the next:
//   S^T = K Q^T puts the query on the lane (C[row = key 4hi+i][col = query lo]); for a 32-key
//   k-step built from key tiles t0, t1 the lane's 8 k-values are keys {16t0+4hi+i, 16t1+4hi+i} —
//   the MFMA reduction order is free, so the P^T B-operand of O^T = V^T P^T is just the packed
//   accumulators.  The matching V^T A-operand is read from the ROW-MAJOR V image with the gfx950
//   transpose read ds_read_b64_tr_b16 (4 keys x 16 d per 16-lane group), so no transposed copy is
//   staged and P never touches LDS.
//   attn_fwd    block = (head, batch), K/V row-major in LDS (64 KB: 2 blocks per CU), the 4 waves
//               loop over 16-query tiles; writes O and the row log-sum-exp (log2 domain).
//   attn_bwd_q  same shape: S^T, dP^T = V dO^T (query on the lane), dS^T = P^T (dP^T - delta),
//               dQ = dS K with dS^T's accumulators as the A operand and K^T by transpose reads;
//               also writes delta = rowsum(dO * O) for attn_bwd_kv.
//   attn_bwd_kv block = (head, batch), Q/dO row-major in LDS, waves loop over 16-key tiles: S and
//               dP with the KEY on the lane, so P^T / dS^T are the A operands of dV = P^T dO and
//               dK = dS^T Q, with dO and Q read transposed.
// LDS images are unpadded 128-B rows (64 bf16) whose 16-B chunks are XOR-swizzled per row pair,
// chunk' = chunk ^ (((row >> 1) & 3) << 1): both access kinds are then bank-conflict free --
//  * ds_read_b128 fragment reads (16 rows, chunk 4ks + hi): each of the instruction's four 16-lane
//    groups is 8 rows at one chunk + the other 8 rows at the next chunk, landing on 16 distinct
//    16-B slots of the 256-B bank row (two rows per bank row);
//  * ds_read_b64_tr_b16 transpose reads (per 32-lane half: 8 consecutive rows x 2 chunks).
// (The round-2 layout, 144-B padded rows, put 2 lanes of every b128 group on one slot: 39-47 %
// SQ_LDS_BANK_CONFLICT, profiles/r2_pmc_vit_b16.md.)
#include "rk_common.h"

using namespace rk;

namespace {

constexpr int D = 64;
constexpr int LMAX = 224;        // max tokens: 14 tiles of 16 (7 k-steps of 32)
constexpr int NT = LMAX / 16;    // 14
constexpr int NKS = NT / 2;      // 7
constexpr int RS = D;            // row-major LDS stride (64 bf16 = 128 B), chunk-swizzled (eoff)
// threads per block (template parameter NTH of each kernel): 4 or 8 waves looping over the head's
// 16-row tiles (13 at L = 197: 8 waves finish in 2 rounds instead of 4); rk_attn_set_waves
int g_waves[3] = {8, 82, 82};  // fwd, bwd_q, bwd_kv (82: 8 waves bounded to 128 VGPRs, 2 blocks/CU)
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const uint16_t* q;   // token-major, row stride ld (elements), head h at column h*D
  const uint16_t* k;
  const uint16_t* v;
  const uint16_t* o;   // forward output (bwd), row stride ldo
  const uint16_t* dout;
  uint16_t* out;       // fwd: O
  uint16_t* dq;        // bwd: gradients, row stride ldg
  uint16_t* dk;
  uint16_t* dv;
  float* lse;          // [B*H][L], log2 domain
  float* delta;        // [B*H][L]
  float* stamps;       // fused backward diagnostics: [B*H][4] phase times, or null (rk_attn_set_stamps)
  int ld, ldo, ldg;
  int L, H;
  float scale;         // softmax scale (1/sqrt(D))
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ bf16x8 ld16(const uint16_t* p) { return *(const bf16x8*)p; }
__device__ __forceinline__ bf16x8 zero8() { return bf16x8{}; }

// global token row r of head h, 8 d-values from column c (clamped + selected: branch-free)
__device__ __forceinline__ bf16x8 gload_row(const uint16_t* base, int ld, int b, int L, int r, int h, int c) {
  const int rc = r < L ? r : L - 1;
  const bf16x8 v = ld16(base + ((int64_t)b * L + rc) * ld + h * D + c);
  return r < L ? v : zero8();
}

// element offset of 8-element chunk ch of row r in a swizzled [LMAX][64] image (header comment)
__device__ __forceinline__ int eoff(int r, int ch) { return r * RS + ((ch ^ (((r >> 1) & 3) << 1)) << 3); }

// stage a head's tokens of two tensors row-major into [LMAX][RS] images (zero rows >= L): every
// thread issues all of its 16-byte loads before its first LDS write, so the block waits for one
// memory round trip instead of one per loop iteration
template <int NTH>
__device__ __forceinline__ void stage_rows2(uint16_t* d0, const uint16_t* s0, int ld0, uint16_t* d1,
                                            const uint16_t* s1, int ld1, int b, int L, int h) {
  constexpr int N = LMAX * (D / 8), IT = (N + NTH - 1) / NTH;
  bf16x8 v0[IT], v1[IT];
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = min((int)threadIdx.x + u * NTH, N - 1);
    v0[u] = gload_row(s0, ld0, b, L, i >> 3, h, (i & 7) * 8);
    v1[u] = gload_row(s1, ld1, b, L, i >> 3, h, (i & 7) * 8);
  }
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = (int)threadIdx.x + u * NTH;
    if (i < N) {
      *(bf16x8*)(d0 + eoff(i >> 3, i & 7)) = v0[u];
      *(bf16x8*)(d1 + eoff(i >> 3, i & 7)) = v1[u];
    }
  }
}

// fragment row read: 8 d-values (chunk ch) of row r
__device__ __forceinline__ bf16x8 frag(const uint16_t* img, int r, int ch) { return ld16(img + eoff(r, ch)); }

// Transpose read of a row-major [.][RS] bf16 image: the calling 16-lane group (lanes 16g..16g+15)
// gets rows r0..r0+3 (r0 = this group's first row), columns c0..c0+15: lane lo receives column
// c0 + lo, element q = row r0 + q.  Every lane of the wave must execute it (EXEC all ones).
__device__ __forceinline__ uint2 tr4(const uint16_t* img, int r0, int c0, int lo) {
  const int c = c0 + 4 * (lo & 3);
  const uint16_t* p = img + eoff(r0 + (lo >> 2), c >> 3) + (c & 7);
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  return __builtin_bit_cast(uint2, v);
}

// 16x16x32 operand whose 8 k-values are rows {r0a..r0a+3, r0b..r0b+3} of a row-major image at
// columns c0 + lo (the "k = keys of tiles t0, t1" order of the accumulator hand-off)
__device__ __forceinline__ bf16x8 tr_operand(const uint16_t* img, int r0a, int r0b, int c0, int lo) {
  const uint2 a = tr4(img, r0a, c0, lo), b = tr4(img, r0b, c0, lo);
  return __builtin_bit_cast(bf16x8, make_uint4(a.x, a.y, b.x, b.y));
}

// transposed read of the fused backward's [key][32-query] dS chunk image (64-B rows): the 16-lane
// group gets keys r0..r0+3, queries c0..c0+15; lane lo receives query c0 + lo, element j = key r0 + j
template <int P = 32>  // row pitch (elements)
__device__ __forceinline__ uint2 tr4dsc(const uint16_t* img, int r0, int c0, int lo) {
  const uint16_t* p = img + (r0 + (lo >> 2)) * P + c0 + 4 * (lo & 3);
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  return __builtin_bit_cast(uint2, v);
}

// 16-bit element format of a kernel instance: H = fp16 (autocast fp16), else bf16.  Operands
// travel as bf16x8 bit patterns either way; only the MFMA opcode and the conversions differ.
template <bool H = false>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return pack16t<H>(a, b);
}
template <bool H = false>
__device__ __forceinline__ uint16_t cvt16(float a) {
  return H ? f2h(a) : f2bf(a);
}
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
template <bool H = false>
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (H)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// accumulators of tiles t0 (k 0..3) and t1 (k 4..7) -> one 16-bit x 8 operand
template <bool H = false>
__device__ __forceinline__ bf16x8 pack_operand(const f32x4& x, const f32x4& y) {
  return __builtin_bit_cast(bf16x8, make_uint4(pack2<H>(x[0], x[1]), pack2<H>(x[2], x[3]), pack2<H>(y[0], y[1]),
                                               pack2<H>(y[2], y[3])));
}

__device__ __forceinline__ float red4_max(float v) {  // over the 4 lanes sharing lo (hi = 0..3)
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float red4_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// --------------------------------------------------------------------------------- forward
template <int NTH, int MINW = 1, bool H = false>  // MINW: minimum waves per SIMD (launch_bounds)
__global__ void __launch_bounds__(NTH, MINW) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[LMAX * RS];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lo = lane & 15, hi = lane >> 4;
  const int L = a.L;
  const int ntile = (L + 15) / 16;
  bf16x8 qn[2];  // this wave's first query tile, loaded with the K/V staging
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) qn[ks] = gload_row(a.q, a.ld, b, L, 16 * w + lo, h, 32 * ks + 8 * hi);
  stage_rows2<NTH>(Ks, a.k, a.ld, Vs, a.v, a.ld, b, L, h);
  __syncthreads();

  const float sl = a.scale * LOG2E;
  const int64_t bh = (int64_t)b * a.H + h;
  for (int qt = w; qt < ntile; qt += NTH / 64) {
    const int q0 = 16 * qt;
    bf16x8 qb[2];  // B operand of S^T = K Q^T: n = query q0 + lo, k = d 32ks + 8hi + j
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qb[ks] = qn[ks];
    if (qt + NTH / 64 < ntile) {  // the next tile's Q: in flight under this tile's products
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) qn[ks] = gload_row(a.q, a.ld, b, L, q0 + 16 * (NTH / 64) + lo, h, 32 * ks + 8 * hi);
    }
    f32x4 s[NT];
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      s[t] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      if (t < ntile) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc = mfma16<H>(frag(Ks, 16 * t + lo, 4 * ks + hi), qb[ks], acc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // C[row = key 16t + 4hi + i][col = query lo]
          s[t][i] = 16 * t + 4 * hi + i < L ? acc[i] * sl : -INFINITY;
          m = fmaxf(m, s[t][i]);
        }
      }
    }
    m = red4_max(m);
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[t][i] = __builtin_amdgcn_exp2f(s[t][i] - m);  // masked / absent keys: exp2(-inf) = 0
        sum += s[t][i];
      }
    sum = red4_sum(sum);
    f32x4 o[4];  // O^T: C[row = d 16nt + 4hi + i][col = query lo]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) o[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (32 * ks < 16 * ntile) {  // uniform
        const bf16x8 pb = pack_operand<H>(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          o[nt] = mfma16<H>(
              tr_operand(Vs, 32 * ks + 4 * hi, 32 * ks + 16 + 4 * hi, 16 * nt, lo), pb, o[nt]);
      }
    }
    const int r = q0 + lo;
    if (r < L) {
      const float inv = 1.f / sum;
      uint16_t* orow = a.out + ((int64_t)b * L + r) * a.ldo + h * D;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        *(uint2*)(orow + 16 * nt + 4 * hi) = make_uint2(pack2<H>(o[nt][0] * inv, o[nt][1] * inv),
                                                        pack2<H>(o[nt][2] * inv, o[nt][3] * inv));
      if (hi == 0) a.lse[bh * L + r] = m + log2f(sum);
    }
  }
}

// ------------------------------------------------------------------------------- backward: dQ
template <int NTH, int MINW = 1>  // MINW: minimum waves per SIMD (launch_bounds)
__global__ void __launch_bounds__(NTH, MINW) attn_bwd_q_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[LMAX * RS];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lo = lane & 15, hi = lane >> 4;
  const int L = a.L;
  const int ntile = (L + 15) / 16;
  stage_rows2<NTH>(Ks, a.k, a.ld, Vs, a.v, a.ld, b, L, h);
  __syncthreads();

  const float sl = a.scale * LOG2E;
  const int64_t bh = (int64_t)b * a.H + h;
  for (int qt = w; qt < ntile; qt += NTH / 64) {
    const int q0 = 16 * qt;
    bf16x8 qb[2], gb[2];  // B operands: n = query q0 + lo, k = d
    float dot = 0.f;      // partial rowsum(dO * O) of query q0 + lo over this lane's 16 d values
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qb[ks] = gload_row(a.q, a.ld, b, L, q0 + lo, h, 32 * ks + 8 * hi);
      gb[ks] = gload_row(a.dout, a.ldo, b, L, q0 + lo, h, 32 * ks + 8 * hi);
      const bf16x8 ov = gload_row(a.o, a.ldo, b, L, q0 + lo, h, 32 * ks + 8 * hi);
      const uint4 gu = __builtin_bit_cast(uint4, gb[ks]), ou = __builtin_bit_cast(uint4, ov);
      const uint32_t gw[4] = {gu.x, gu.y, gu.z, gu.w}, ow[4] = {ou.x, ou.y, ou.z, ou.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        dot += __uint_as_float(gw[e] << 16) * __uint_as_float(ow[e] << 16) +
               __uint_as_float(gw[e] & 0xffff0000u) * __uint_as_float(ow[e] & 0xffff0000u);
    }
    const float delta = red4_sum(dot);  // every lane with this lo holds delta(query q0 + lo)
    const int rq = q0 + lo;
    if (hi == 0 && rq < L) a.delta[bh * L + rq] = delta;
    const float lq = a.lse[bh * L + (rq < L ? rq : L - 1)];
    f32x4 ds[NT];  // dS^T: C[row = key 16t + 4hi + i][col = query lo]
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      ds[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t < ntile) {
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(Ks, 16 * t + lo, 4 * ks + hi), qb[ks], s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(Vs, 16 * t + lo, 4 * ks + hi), gb[ks], dp, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = 16 * t + 4 * hi + i < L ? exp2f(s[i] * sl - lq) : 0.f;
          ds[t][i] = p * (dp[i] - delta) * a.scale;
        }
      }
    }
    f32x4 dq[4];  // dQ: C[row = query 4hi + i][col = d 16nt + lo]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dq[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (32 * ks < 16 * ntile) {
        const bf16x8 sa = pack_operand(ds[2 * ks], ds[2 * ks + 1]);  // A: row = query lo, k = keys
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          dq[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              sa, tr_operand(Ks, 32 * ks + 4 * hi, 32 * ks + 16 + 4 * hi, 16 * nt, lo), dq[nt], 0, 0, 0);
      }
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
  }
}

// --------------------------------------------------------------------------- backward: dK, dV
template <int NTH, int MINW = 1>  // MINW: minimum waves per SIMD (launch_bounds)
__global__ void __launch_bounds__(NTH, MINW) attn_bwd_kv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Qs[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Gs[LMAX * RS];  // dO row-major
  __shared__ float lse_s[LMAX], del_s[LMAX];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lo = lane & 15, hi = lane >> 4;
  const int L = a.L;
  const int ntile = (L + 15) / 16;
  const int64_t bh = (int64_t)b * a.H + h;
  stage_rows2<NTH>(Qs, a.q, a.ld, Gs, a.dout, a.ldo, b, L, h);
  for (int i = threadIdx.x; i < LMAX; i += NTH) {
    lse_s[i] = i < L ? a.lse[bh * L + i] : 0.f;
    del_s[i] = i < L ? a.delta[bh * L + i] : 0.f;
  }
  __syncthreads();

  const float sl = a.scale * LOG2E;
  for (int kt = w; kt < ntile; kt += NTH / 64) {
    const int k0 = 16 * kt;
    bf16x8 kb[2], vb[2];  // B operands of S = Q K^T and dP = dO V^T: n = key k0 + lo, k = d
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kb[ks] = gload_row(a.k, a.ld, b, L, k0 + lo, h, 32 * ks + 8 * hi);
      vb[ks] = gload_row(a.v, a.ld, b, L, k0 + lo, h, 32 * ks + 8 * hi);
    }
    f32x4 dk[4], dv[4];  // C[row = key 4hi + i][col = d 16nt + lo]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dk[nt] = dv[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < NKS; ++ks) {
      if (32 * ks >= 16 * ntile) break;  // uniform
      f32x4 p2[2], ds2[2];  // query tiles 2ks, 2ks+1: C[row = query 16qt + 4hi + i][col = key lo]
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * ks + u;
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
        if (qt < ntile) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(Qs, 16 * qt + lo, 4 * kk + hi), kb[kk], s, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(Gs, 16 * qt + lo, 4 * kk + hi), vb[kk], dp, 0, 0, 0);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qi = 16 * qt + 4 * hi + i;
          const float p = qi < L ? exp2f(s[i] * sl - lse_s[qi]) : 0.f;
          p2[u][i] = p;
          ds2[u][i] = p * (dp[i] - del_s[qi]) * a.scale;
        }
      }
      // A operands: row = key lo, k = queries {32ks + 4hi + i, 32ks + 16 + 4hi + i}
      const bf16x8 pa = pack_operand(p2[0], p2[1]);
      const bf16x8 sa = pack_operand(ds2[0], ds2[1]);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        dv[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            pa, tr_operand(Gs, 32 * ks + 4 * hi, 32 * ks + 16 + 4 * hi, 16 * nt, lo), dv[nt], 0, 0, 0);
        dk[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            sa, tr_operand(Qs, 32 * ks + 4 * hi, 32 * ks + 16 + 4 * hi, 16 * nt, lo), dk[nt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = k0 + 4 * hi + i;
      if (r < L) {
        uint16_t* rk = a.dk + ((int64_t)b * L + r) * a.ldg + h * D;
        uint16_t* rv = a.dv + ((int64_t)b * L + r) * a.ldg + h * D;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          rk[16 * nt + lo] = f2bf(dk[nt][i]);
          rv[16 * nt + lo] = f2bf(dv[nt][i]);
        }
      }
    }
  }
}

// ------------------------------------------------------------- backward: fused dQ, dK, dV
// One block per (head, batch) with ONE WAVE PER 16-KEY TILE (ntile <= 14 waves); Q, dO and K are
// staged once (swizzled row images).  The queries are walked in 32-row chunks; per chunk:
//  A (every wave, its key tile): S = Q K^T and dP = dO V^T with the key on the lane (computed
//    ONCE; the split kernels compute both twice), P and dS; dV += P^T dO and dK += dS^T Q stay in
//    the wave's registers; dS goes to the chunk's shared [key][32-query] bf16 image;
//  B (one barrier later, waves 0..7): one 16-query x 16-d tile of dQ each = dS_chunk K over all
//    keys (A operand = the dS image read transposed: query on the lane; B = K image read
//    transposed), complete in one wave -> stored straight to dQ (no cross-wave reduction).
// The dS image is double-buffered, so a chunk costs one barrier.  delta = rowsum(dO * O) is
// formed while dO is staged.  LDS: 3 x 28 KiB images + 2 x 14 KiB dS chunks + lse / delta.
// (A first version reduced dQ over the key-tile waves with LDS float atomics: 5x slower than the
// split kernels, its chunk loop ~20 us per iteration; bench/attn_probe.py phase stamps.)
constexpr int FUSED_MAXW = LMAX / 16;
constexpr int DSC = 32;  // queries per chunk
// dS image: 64-byte rows [key][32 queries], the 8-byte query groups (4 queries) XOR-swizzled per
// row, g -> g ^ dsw(row) with dsw = row bits {2, 1} in place and bit 3 moved to bit 0.  Both
// accesses are then conflict-free (tools/lds_banks.py): the writer's 16 lanes (16 consecutive
// key rows, one group) cover 32 distinct banks because dsw is a bijection over the 8 rows of a
// parity, and a transpose-read half wave (8 consecutive rows x 4 groups) puts rows r and r + 4
// (the same 16-dword segment of the 256-byte bank row) into opposite 4-group halves via bit 2.
// (The unswizzled 96-byte pitch it replaces: 4-way store conflicts, 37 % of the kernel's LDS cycles.)
constexpr int DSP = 32;
__device__ __forceinline__ int dsw(int row) { return (row & 6) | ((row >> 3) & 1); }
// element offset of query group g (queries 4g..4g+3) of key row `row`
__device__ __forceinline__ int dsoff(int row, int g) { return row * DSP + 4 * (g ^ dsw(row)); }
__device__ __forceinline__ uint2 tr4dsz(const uint16_t* img, int r0, int c0, int lo) {
  const int row = r0 + (lo >> 2);
  const uint16_t* p = img + dsoff(row, (c0 >> 2) + (lo & 3));
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  return __builtin_bit_cast(uint2, v);
}

template <bool H = false>
__global__ void __launch_bounds__(64 * FUSED_MAXW) attn_bwd_fused_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Qs[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Gs[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Ks[LMAX * RS];
  __shared__ __attribute__((aligned(16))) uint16_t dSs[2][LMAX * DSP];  // [key][query of the chunk]
  __shared__ __attribute__((aligned(16))) float lse_s[LMAX];
  __shared__ __attribute__((aligned(16))) float del_s[LMAX];
  const int b = blockIdx.z, h = blockIdx.y;
  const int nthr = blockDim.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lo = lane & 15, hi = lane >> 4;
  const int L = a.L;
  const int ntile = (L + 15) / 16;
  const int64_t bh = (int64_t)b * a.H + h;
  // diagnostics (rk_attn_set_stamps): thread 0 stamps s_memrealtime at phase boundaries into
  // stamps[block * 4 + 1..3] (staged, chunk loop done, end; bench/attn_probe.py)
  float* stamp = (a.stamps != nullptr && threadIdx.x == 0) ? a.stamps + (int64_t)bh * 4 : nullptr;
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  const int k0 = 16 * w;  // this wave's key tile (blockDim = 64 * ntile: every wave has one)
  // its V fragments, loaded with the staging (retired by the staging barrier: no memory wait in
  // the chunk loop, whose only memory operations are then the dQ stores)
  bf16x8 vb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) vb[ks] = gload_row(a.v, a.ld, b, L, k0 + lo, h, 32 * ks + 8 * hi);
  // 8 consecutive threads = one row; a pass issues the 16-byte loads of SU rows-chunks per thread
  // (Q, K, dO, O) before any LDS write: one memory round trip per pass (one pass at L = 197)
  constexpr int SU = 3;
  for (int i0 = threadIdx.x; i0 < LMAX * (D / 8); i0 += SU * nthr) {
    bf16x8 qv[SU], kv[SU], gv[SU], ov[SU];
    float lv[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int i = min(i0 + u * nthr, LMAX * (D / 8) - 1);
      const int r = i >> 3, c = (i & 7) * 8;
      lv[u] = a.lse[bh * L + min(r, L - 1)];
      qv[u] = gload_row(a.q, a.ld, b, L, r, h, c);
      kv[u] = gload_row(a.k, a.ld, b, L, r, h, c);
      gv[u] = gload_row(a.dout, a.ldo, b, L, r, h, c);
      ov[u] = gload_row(a.o, a.ldo, b, L, r, h, c);
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int i = i0 + u * nthr;
      const int r = i >> 3, ch = i & 7;
      const bool in = i < LMAX * (D / 8);  // uniform per 8-thread row group (nthr % 64 == 0)
      if (in) {
        *(bf16x8*)(Qs + eoff(r, ch)) = qv[u];
        *(bf16x8*)(Ks + eoff(r, ch)) = kv[u];
        *(bf16x8*)(Gs + eoff(r, ch)) = gv[u];
      }
      const uint4 gu = __builtin_bit_cast(uint4, gv[u]), ou = __builtin_bit_cast(uint4, ov[u]);
      const uint32_t gw[4] = {gu.x, gu.y, gu.z, gu.w}, ow[4] = {ou.x, ou.y, ou.z, ou.w};
      float dot = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        dot += lo16t<H>(gw[e]) * lo16t<H>(ow[e]) + hi16t<H>(gw[e]) * hi16t<H>(ow[e]);
      dot += __shfl_xor(dot, 1, 64);
      dot += __shfl_xor(dot, 2, 64);
      dot += __shfl_xor(dot, 4, 64);
      if (in && ch == 0) {
        del_s[r] = dot;
        lse_s[r] = r < L ? lv[u] : 0.f;
      }
    }
  }
  // the dS rows of a key tile without a wave (odd ntile: the last 32-key step's upper half) are
  // read by the dQ products: keep them zero (uninitialised LDS could hold NaN patterns)
  for (int i = threadIdx.x; i < 2 * LMAX * DSP / 8; i += nthr) *(uint4*)(&dSs[0][0] + 8 * i) = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  if (stamp) stamp[1] = (float)(__builtin_amdgcn_s_memrealtime() - t_start);

  const float sl = a.scale * LOG2E;
  bf16x8 kb[2];  // B operands of S = Q K^T / dP = dO V^T: n = key k0 + lo, k = d
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) kb[ks] = frag(Ks, k0 + lo, 4 * ks + hi);
  f32x4 dk[4], dv[4];  // C[row = key 4hi + i][col = d 16nt + lo]
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) dk[nt] = dv[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkey32 = (ntile + 1) / 2;  // 32-key k-steps of the dQ products
  // phase B of chunk kc (reads dS buffer kc & 1): the chunk's 8 dQ tiles (16 queries qh x 16 d nt)
  // = sum over keys of dS[q][k] K[k][d], tile t on wave t % nwaves (fewer than 8 waves when L <= 112)
  auto phase_b = [&](int kc) {
    const uint16_t* dsc = dSs[kc & 1];
    for (int t = w; t < 8; t += nthr / 64) {
      const int qh = t >> 2, nt = t & 3;
      if (32 * kc + 16 * qh >= L) continue;  // wave-uniform
      f32x4 dq = {0.f, 0.f, 0.f, 0.f};
      for (int kq = 0; kq < nkey32; ++kq) {
        // A: row = query 16qh + lo, k = keys 32kq + {4hi + j, 16 + 4hi + j} (transposed reads of the
        // [key][query] image); B: k = the same keys, n = d 16nt + lo (transposed reads of K)
        const uint2 a0 = tr4dsz(dsc, 32 * kq + 4 * hi, 16 * qh, lo), a1 = tr4dsz(dsc, 32 * kq + 16 + 4 * hi, 16 * qh, lo);
        const bf16x8 av = __builtin_bit_cast(bf16x8, make_uint4(a0.x, a0.y, a1.x, a1.y));
        dq = mfma16<H>(
            av, tr_operand(Ks, 32 * kq + 4 * hi, 32 * kq + 16 + 4 * hi, 16 * nt, lo), dq);
      }
      const int r0 = 32 * kc + 16 * qh + 4 * hi;  // C[row = query r0 + i][col = d lo]
      uint16_t* dqp = a.dq + ((int64_t)b * L + r0) * a.ldg + h * D + 16 * nt + lo;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (r0 + i < L) dqp[(int64_t)i * a.ldg] = cvt16<H>(dq[i]);
    }
  };
  int nchunks = 0;
  for (int ks = 0; ks < NKS; ++ks) {
    if (32 * ks >= 16 * ntile) break;  // uniform
    nchunks = ks + 1;
    uint16_t* dsc = dSs[ks & 1];
    // ---- A: this wave's key tile x the chunk's 32 queries
    f32x4 p2[2], ds2[2];  // query tiles 2ks, 2ks+1: C[row = query 16qt + 4hi + i][col = key lo]
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qt = 2 * ks + u;
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      if (qt < ntile) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          sv = mfma16<H>(frag(Qs, 16 * qt + lo, 4 * kk + hi), kb[kk], sv);
          dp = mfma16<H>(frag(Gs, 16 * qt + lo, 4 * kk + hi), vb[kk], dp);
        }
      }
      // the 4 queries' lse / delta as one 16-byte LDS read each (entries >= L are zero), the exp
      // unconditional and masked by a select: no branch, no per-element LDS round trip
      const int q4 = 16 * qt + 4 * hi;
      const f32x4 lq = *(const f32x4*)(lse_s + q4), dq4 = *(const f32x4*)(del_s + q4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = q4 + i < L && k0 + lo < L;
        const float e = __builtin_amdgcn_exp2f(sv[i] * sl - lq[i]);
        const float p = ok ? e : 0.f;
        p2[u][i] = p;
        ds2[u][i] = p * (dp[i] - dq4[i]) * a.scale;
      }
    }
    const bf16x8 pa = pack_operand<H>(p2[0], p2[1]);  // A: row = key lo, k = the chunk's queries
    const bf16x8 sa = pack_operand<H>(ds2[0], ds2[1]);
    // dS -> the chunk image first (the barrier below waits for it): row = key k0 + lo, 4
    // consecutive queries 16u + 4hi .. +3
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *(uint2*)(dsc + dsoff(k0 + lo, 4 * u + hi)) =
          make_uint2(pack2<H>(ds2[u][0], ds2[u][1]), pack2<H>(ds2[u][2], ds2[u][3]));
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      dv[nt] = mfma16<H>(
          pa, tr_operand(Gs, 32 * ks + 4 * hi, 32 * ks + 16 + 4 * hi, 16 * nt, lo), dv[nt]);
      dk[nt] = mfma16<H>(
          sa, tr_operand(Qs, 32 * ks + 4 * hi, 32 * ks + 16 + 4 * hi, 16 * nt, lo), dk[nt]);
    }
    // ---- B of the PREVIOUS chunk in the same barrier interval (its buffer was completed before
    // the previous barrier; the next chunk's A rewrites it only after the barrier below)
    if (ks > 0) phase_b(ks - 1);
    // chunk ks's dS rows of every key tile are in: wait for this wave's LDS traffic only, then the
    // raw barrier — __syncthreads() would also wait (vmcnt(0)) for the dQ stores just issued, a
    // memory round trip per chunk that nothing here depends on
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (nchunks > 0) phase_b(nchunks - 1);
  if (stamp) stamp[2] = (float)(__builtin_amdgcn_s_memrealtime() - t_start);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = k0 + 4 * hi + i;
    if (r < L) {
      uint16_t* rk = a.dk + ((int64_t)b * L + r) * a.ldg + h * D;
      uint16_t* rv = a.dv + ((int64_t)b * L + r) * a.ldg + h * D;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        rk[16 * nt + lo] = cvt16<H>(dk[nt][i]);
        rv[16 * nt + lo] = cvt16<H>(dv[nt][i]);
      }
    }
  }
  if (stamp) stamp[3] = (float)(__builtin_amdgcn_s_memrealtime() - t_start);
}


// ------------------------------------------------ backward: fused dQ, dK, dV, streamed queries
// As attn_bwd_fused_kernel (one block per (head, batch), a wave per 16-key tile, 32-query chunks,
// dS through a double-buffered image, the previous chunk's dQ in the same barrier interval), but
// only K is staged whole: the chunk's Q / dO / O rows (3 x 4 KiB) arrive by LDS-DMA into a 2-slot
// ring, issued one chunk ahead by waves 0..11 (one 1-KiB piece each, source-side swizzle so the
// lane-linear DMA image matches eoff), so the loads of chunk ks+1 run under chunk ks's products
// instead of a whole-block staging phase in front of them.  delta = rowsum(dO * O) of the chunk's
// rows is formed by every wave from the slot (32 rows x 64 d), then shuffled to the lanes that
// need it.  Every dQ store is issued (rows >= L go to a sink), so the number of VMEM operations a
// wave issues after its DMA piece is known (nst) and the end-of-chunk wait is vmcnt(nst): the
// stores are never waited for.  All LDS is one array (hipcc otherwise waits vmcnt(0) before LDS
// reads next to an LDS-DMA destination).
// Transpose reads as inline asm: the ds_read_tr16_b64 intrinsic carries no alias information, so
// after an LDS-DMA into the same array hipcc puts s_waitcnt vmcnt(0) in front of it (the DMA of
// the next chunk would then be waited for mid-chunk).  The caller waits lgkmcnt(0) + sched_barrier
// before using the results (hipcc does not track inline-asm LDS reads).
__device__ __forceinline__ uint2 tr_raw(const uint16_t* p) {
  uint2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(const lds_void*)p));
  return v;
}
__device__ __forceinline__ uint2 tr4_raw(const uint16_t* img, int r0, int c0, int lo) {
  const int c = c0 + 4 * (lo & 3);
  return tr_raw(img + eoff(r0 + (lo >> 2), c >> 3) + (c & 7));
}
__device__ __forceinline__ bf16x8 tr_operand_raw(const uint16_t* img, int r0a, int r0b, int c0, int lo) {
  const uint2 a = tr4_raw(img, r0a, c0, lo), b = tr4_raw(img, r0b, c0, lo);
  return __builtin_bit_cast(bf16x8, make_uint4(a.x, a.y, b.x, b.y));
}
__device__ __forceinline__ uint2 tr4dsc_raw(const uint16_t* img, int r0, int c0, int lo) {
  return tr_raw(img + (r0 + (lo >> 2)) * 32 + c0 + 4 * (lo & 3));
}
__device__ __forceinline__ void lds_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __attribute__((aligned(16))) uint4 g_attn_zero[1];
__device__ uint16_t g_attn_sink[64];

constexpr int SB_K = 0;                          // K image [LMAX][64], eoff-swizzled
constexpr int SB_Q = SB_K + LMAX * RS * 2;       // Q ring: 2 slots x [32][64]
constexpr int SB_G = SB_Q + 2 * DSC * RS * 2;    // dO ring
constexpr int SB_O = SB_G + 2 * DSC * RS * 2;    // O ring (delta only)
constexpr int SB_S = SB_O + 2 * DSC * RS * 2;    // dS: 2 x [LMAX][32]
constexpr int SB_L = SB_S + 2 * LMAX * DSC * 2;  // lse [LMAX] f32
constexpr int SB_END = SB_L + LMAX * 4;

__global__ void __launch_bounds__(64 * FUSED_MAXW) attn_bwd_stream_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[SB_END];
  uint16_t* Ks = (uint16_t*)(smem + SB_K);
  float* lse_s = (float*)(smem + SB_L);
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, lo = lane & 15, hi = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar) wave index
  const int nthr = blockDim.x;
  const int L = a.L;
  const int ntile = (L + 15) / 16;
  const int nchunks = (ntile + 1) / 2;
  const int64_t bh = (int64_t)b * a.H + h;
  float* stamp = (a.stamps != nullptr && threadIdx.x == 0) ? a.stamps + (int64_t)bh * 4 : nullptr;
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  const int k0 = 16 * w;

  // a chunk is 12 pieces of 1 KiB (tensor pc / 4: Q, dO, O; rows 8 (pc % 4) .. + 7), piece pc on
  // wave pc % nw (one each at L = 197, up to 12 on a 1-wave block)
  const int nw = nthr / 64;
  const bool stager = w < 12;
  const int srow0 = lane >> 3;
  // per-tensor sources (kernel arguments read once, outside the chunk loop)
  const uint16_t* const srcs[3] = {a.q, a.dout, a.o};
  const int lds_[3] = {a.ld, a.ldo, a.ldo};
  auto stage_chunk = [&](int c, int slot) {
    for (int pc = w; pc < 12; pc += nw) {  // scalar loop
      const int tsel = pc >> 2, piece = pc & 3;
      const int srow = 8 * piece + srow0;
      const int lch = (lane & 7) ^ (((srow >> 1) & 3) << 1);  // logical chunk landing at this lane's slot
      const uint16_t* sbase = tsel == 0 ? srcs[0] : tsel == 1 ? srcs[1] : srcs[2];
      const int sld = tsel == 0 ? lds_[0] : lds_[1];
      const int sbyte = (tsel == 0 ? SB_Q : tsel == 1 ? SB_G : SB_O) + piece * 1024;
      const int r = 32 * c + srow;
      const char* src = r < L ? (const char*)(sbase + ((int64_t)b * L + r) * sld + h * D + lch * 8)
                              : (const char*)g_attn_zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(smem + sbyte + slot * DSC * RS * 2), 16, 0, 0);
    }
  };
  stage_chunk(0, 0);  // in flight under the K staging
  bf16x8 vb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) vb[ks] = gload_row(a.v, a.ld, b, L, k0 + lo, h, 32 * ks + 8 * hi);
  {  // K image + lse, every load issued before the first LDS write
    constexpr int N = LMAX * (D / 8), SU = 3;
    for (int i0 = threadIdx.x; i0 < N; i0 += SU * nthr) {
      bf16x8 kv[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int i = min(i0 + u * nthr, N - 1);
        kv[u] = gload_row(a.k, a.ld, b, L, i >> 3, h, (i & 7) * 8);
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int i = i0 + u * nthr;
        if (i < N) *(bf16x8*)(Ks + eoff(i >> 3, i & 7)) = kv[u];
      }
    }
    for (int r = threadIdx.x; r < LMAX; r += nthr) lse_s[r] = r < L ? a.lse[bh * L + r] : 0.f;
  }
  {  // dS rows of key tiles without a wave stay zero (read by the dQ products)
    uint16_t* d0 = (uint16_t*)(smem + SB_S);
    for (int i = threadIdx.x; i < 2 * LMAX * DSC / 8; i += nthr) *(uint4*)(d0 + 8 * i) = make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();  // K, lse, dS zeros and chunk 0's DMA (every wave waited vmcnt(0) here)
  if (stamp) stamp[1] = (float)(__builtin_amdgcn_s_memrealtime() - t_start);

  const float sl = a.scale * LOG2E;
  bf16x8 kb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) kb[ks] = frag(Ks, k0 + lo, 4 * ks + hi);
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) dk[nt] = dv[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkey32 = (ntile + 1) / 2;
  // phase B of chunk kc: the chunk's 8 dQ tiles, tile t on wave t % nw; returns the number of VMEM
  // stores this wave issued (wave-uniform)
  auto phase_b = [&](int kc) -> int {
    int nst = 0;
    const uint16_t* dsc = (const uint16_t*)(smem + SB_S) + (kc & 1) * LMAX * DSC;
    for (int t = w; t < 8; t += nw) {
    const int qh = t >> 2, nt = t & 3;
    if (32 * kc + 16 * qh >= L) continue;  // wave-uniform
    f32x4 dq = {0.f, 0.f, 0.f, 0.f};
    for (int kq = 0; kq < nkey32; ++kq) {
      const uint2 a0 = tr4dsc_raw(dsc, 32 * kq + 4 * hi, 16 * qh, lo), a1 = tr4dsc_raw(dsc, 32 * kq + 16 + 4 * hi, 16 * qh, lo);
      const bf16x8 bv = tr_operand_raw(Ks, 32 * kq + 4 * hi, 32 * kq + 16 + 4 * hi, 16 * nt, lo);
      lds_wait();
      const bf16x8 av = __builtin_bit_cast(bf16x8, make_uint4(a0.x, a0.y, a1.x, a1.y));
      dq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, dq, 0, 0, 0);
    }
    const int r0 = 32 * kc + 16 * qh + 4 * hi;
    uint16_t* dqp = a.dq + ((int64_t)b * L + r0) * a.ldg + h * D + 16 * nt + lo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // every store issued (rows >= L into the sink): a known count
      uint16_t* p = r0 + i < L ? dqp + (int64_t)i * a.ldg : g_attn_sink + lane;
      *p = f2bf(dq[i]);
    }
    nst += 4;
    }
    return nst;
  };
  for (int ks = 0; ks < nchunks; ++ks) {
    const int slot = ks & 1;
    const bool ahead = ks + 1 < nchunks;
    if (ahead) stage_chunk(ks + 1, slot ^ 1);  // that slot was last read before the previous barrier
    const uint16_t* Qc = (const uint16_t*)(smem + SB_Q) + slot * DSC * RS;
    const uint16_t* Gc = (const uint16_t*)(smem + SB_G) + slot * DSC * RS;
    const uint16_t* Oc = (const uint16_t*)(smem + SB_O) + slot * DSC * RS;
    uint16_t* dsc = (uint16_t*)(smem + SB_S) + slot * LMAX * DSC;
    // delta of the chunk's rows: lane = row (lane & 31), d half (lane >> 5)
    float dl;
    {
      const int r = lane & 31, hf = lane >> 5;
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4 gu = __builtin_bit_cast(uint4, frag(Gc, r, 4 * hf + j));
        const uint4 ou = __builtin_bit_cast(uint4, frag(Oc, r, 4 * hf + j));
        const uint32_t gw[4] = {gu.x, gu.y, gu.z, gu.w}, ow[4] = {ou.x, ou.y, ou.z, ou.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          t += __uint_as_float(gw[e] << 16) * __uint_as_float(ow[e] << 16) +
               __uint_as_float(gw[e] & 0xffff0000u) * __uint_as_float(ow[e] & 0xffff0000u);
      }
      dl = t + __shfl_xor(t, 32, 64);
    }
    f32x4 p2[2], ds2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qt = 2 * ks + u;
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      if (qt < ntile) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(Qc, 16 * u + lo, 4 * kk + hi), kb[kk], sv, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(Gc, 16 * u + lo, 4 * kk + hi), vb[kk], dp, 0, 0, 0);
        }
      }
      const int q4 = 16 * qt + 4 * hi;
      const f32x4 lq = *(const f32x4*)(lse_s + q4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dqi = __shfl(dl, 16 * u + 4 * hi + i, 64);
        const bool ok = q4 + i < L && k0 + lo < L;
        const float e = __builtin_amdgcn_exp2f(sv[i] * sl - lq[i]);
        const float p = ok ? e : 0.f;
        p2[u][i] = p;
        ds2[u][i] = p * (dp[i] - dqi) * a.scale;
      }
    }
    const bf16x8 pa = pack_operand(p2[0], p2[1]);
    const bf16x8 sa = pack_operand(ds2[0], ds2[1]);
    {  // dS row of this lane's key, 4 queries per u, as inline-asm LDS stores (a plain store after an
       // LDS-DMA into the same array gets a vmcnt(0) wait from hipcc; the barrier's lgkmcnt(0)
       // retires these)
      const uint32_t da = (uint32_t)(uintptr_t)(lds_void*)(dsc + (k0 + lo) * DSC + 4 * hi);
      const uint2 v0 = make_uint2(pack2(ds2[0][0], ds2[0][1]), pack2(ds2[0][2], ds2[0][3]));
      const uint2 v1 = make_uint2(pack2(ds2[1][0], ds2[1][1]), pack2(ds2[1][2], ds2[1][3]));
      asm volatile("ds_write_b64 %0, %1\n\tds_write_b64 %0, %2 offset:32" ::"v"(da), "v"(v0), "v"(v1) : "memory");
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {  // two d-halves: 8 transpose reads in flight, then 4 MFMAs
      bf16x8 gv[2], qv[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        gv[j] = tr_operand_raw(Gc, 4 * hi, 16 + 4 * hi, 16 * (2 * hh + j), lo);
        qv[j] = tr_operand_raw(Qc, 4 * hi, 16 + 4 * hi, 16 * (2 * hh + j), lo);
      }
      lds_wait();
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        dv[2 * hh + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, gv[j], dv[2 * hh + j], 0, 0, 0);
        dk[2 * hh + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, qv[j], dk[2 * hh + j], 0, 0, 0);
      }
    }
    const int nst = ks > 0 ? phase_b(ks - 1) : 0;
    // this wave's DMA piece of chunk ks+1 has landed once at most the nst dQ stores issued after it
    // are outstanding; then LDS traffic, then the raw barrier (no wait for the stores themselves)
    if (ahead && stager) {
      if (nst == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (nst == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (0 stores; or many: wait for all)
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (nchunks > 0) phase_b(nchunks - 1);
  if (stamp) stamp[2] = (float)(__builtin_amdgcn_s_memrealtime() - t_start);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = k0 + 4 * hi + i;
    if (r < L) {
      uint16_t* rk = a.dk + ((int64_t)b * L + r) * a.ldg + h * D;
      uint16_t* rv = a.dv + ((int64_t)b * L + r) * a.ldg + h * D;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        rk[16 * nt + lo] = f2bf(dk[nt][i]);
        rv[16 * nt + lo] = f2bf(dv[nt][i]);
      }
    }
  }
  if (stamp) stamp[3] = (float)(__builtin_amdgcn_s_memrealtime() - t_start);
}

}  // namespace

int g_bwd_fused = 1;         // rk_attn_set_bwd_fused
float* g_stamps = nullptr;   // rk_attn_set_stamps

RK_API int rk_attn_max_len() { return LMAX; }

// 2: the fused kernel with streamed query chunks (attn_bwd_stream_kernel); 1 (default): one fused
// dQ/dK/dV kernel with whole-head staging; 0: the dQ and dK/dV kernels (A/B, ROCKET_ATTN_BWD)
RK_API int rk_attn_set_bwd_fused(int mode) {
  if (mode < 0 || mode > 2) return (int)hipErrorInvalidValue;
  g_bwd_fused = mode;
  return 0;
}

// diagnostics: the fused backward writes per-block phase stamps ([B*H][4] f32, 100 MHz ticks)
// into `p` on its following launches; null turns them off
RK_API int rk_attn_set_stamps(float* p) {
  g_stamps = p;
  return 0;
}

// waves per block (4 or 8) of the forward, dQ and dK/dV kernels (A/B switch: ROCKET_ATTN_WAVES)
RK_API int rk_attn_set_waves(int fwd, int bwd_q, int bwd_kv) {
  const int w[3] = {fwd, bwd_q, bwd_kv};
  for (int i = 0; i < 3; ++i) {
    if (w[i] != 4 && w[i] != 8 && w[i] != 82) return (int)hipErrorInvalidValue;  // 82: 8 waves, >= 4 waves per SIMD (2 blocks/CU)
    g_waves[i] = w[i];
  }
  return 0;
}

// q/k/v: 16-bit token-major (row stride ld elements; h = 1: fp16, 0: bf16), out: [B*L][ldo] with
// head h at column h*64; lse: [B*H][L] f32.  head dim 64, L <= 224.
RK_API int rk_attn_fwd16(int hf, const void* q, const void* k, const void* v, int ld, void* out, int ldo, float* lse,
                         int B, int L, int H, float scale, hipStream_t s) {
  if (L < 1 || L > LMAX || B < 1 || H < 1) return (int)hipErrorInvalidValue;
  if (ldo % 4 != 0 || (uintptr_t)out % 8 != 0) return (int)hipErrorInvalidValue;  // 8-byte O row pieces
  AttnArgs a{};
  a.q = (const uint16_t*)q; a.k = (const uint16_t*)k; a.v = (const uint16_t*)v;
  a.out = (uint16_t*)out; a.lse = lse; a.ld = ld; a.ldo = ldo; a.L = L; a.H = H; a.scale = scale;
  dim3 grid(1, H, B);  // one block per (batch, head)
  if (hf) {
    if (g_waves[0] == 82) attn_fwd_kernel<512, 4, true><<<grid, 512, 0, s>>>(a);
    else if (g_waves[0] == 8) attn_fwd_kernel<512, 1, true><<<grid, 512, 0, s>>>(a);
    else attn_fwd_kernel<256, 1, true><<<grid, 256, 0, s>>>(a);
  } else if (g_waves[0] == 82) attn_fwd_kernel<512, 4><<<grid, 512, 0, s>>>(a);
  else if (g_waves[0] == 8) attn_fwd_kernel<512><<<grid, 512, 0, s>>>(a);
  else attn_fwd_kernel<256><<<grid, 256, 0, s>>>(a);
  return (int)hipGetLastError();
}
RK_API int rk_attn_fwd(const void* q, const void* k, const void* v, int ld, void* out, int ldo, float* lse, int B,
                       int L, int H, float scale, hipStream_t s) {
  return rk_attn_fwd16(0, q, k, v, ld, out, ldo, lse, B, L, H, scale, s);
}

// gradients dq/dk/dv written token-major with row stride ldg (e.g. into one [B*L][3*H*64] buffer);
// delta: [B*H][L] f32 scratch.  fp16 (hf = 1): the fused backward only.
RK_API int rk_attn_bwd16(int hf, const void* q, const void* k, const void* v, int ld, const void* o, const void* dout,
                         int ldo, const float* lse, float* delta, void* dq, void* dk, void* dv, int ldg, int B, int L,
                         int H, float scale, hipStream_t s) {
  if (L < 1 || L > LMAX || B < 1 || H < 1) return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = (const uint16_t*)q; a.k = (const uint16_t*)k; a.v = (const uint16_t*)v;
  a.o = (const uint16_t*)o; a.dout = (const uint16_t*)dout;
  a.dq = (uint16_t*)dq; a.dk = (uint16_t*)dk; a.dv = (uint16_t*)dv;
  a.lse = (float*)lse; a.delta = delta; a.stamps = g_stamps;
  a.ld = ld; a.ldo = ldo; a.ldg = ldg; a.L = L; a.H = H; a.scale = scale;
  dim3 grid(1, H, B);
  if (hf) {
    if (g_bwd_fused != 1) return (int)hipErrorInvalidValue;
    attn_bwd_fused_kernel<true><<<grid, 64 * ((L + 15) / 16), 0, s>>>(a);
    return (int)hipGetLastError();
  }
  if (g_bwd_fused == 2) {
    attn_bwd_stream_kernel<<<grid, 64 * ((L + 15) / 16), 0, s>>>(a);
    return (int)hipGetLastError();
  }
  if (g_bwd_fused) {
    attn_bwd_fused_kernel<<<grid, 64 * ((L + 15) / 16), 0, s>>>(a);
    return (int)hipGetLastError();
  }
  if (delta == nullptr) return (int)hipErrorInvalidValue;  // the split kernels pass delta between them
  if (g_waves[1] == 82) attn_bwd_q_kernel<512, 4><<<grid, 512, 0, s>>>(a);
  else if (g_waves[1] == 8) attn_bwd_q_kernel<512><<<grid, 512, 0, s>>>(a);
  else attn_bwd_q_kernel<256><<<grid, 256, 0, s>>>(a);
  if (g_waves[2] == 82) attn_bwd_kv_kernel<512, 4><<<grid, 512, 0, s>>>(a);
  else if (g_waves[2] == 8) attn_bwd_kv_kernel<512><<<grid, 512, 0, s>>>(a);
  else attn_bwd_kv_kernel<256><<<grid, 256, 0, s>>>(a);
  return (int)hipGetLastError();
}
RK_API int rk_attn_bwd(const void* q, const void* k, const void* v, int ld, const void* o, const void* dout, int ldo,
                       const float* lse, float* delta, void* dq, void* dk, void* dv, int ldg, int B, int L, int H,
                       float scale, hipStream_t s) {
  return rk_attn_bwd16(0, q, k, v, ld, o, dout, ldo, lse, delta, dq, dk, dv, ldg, B, L, H, scale, s);
}
