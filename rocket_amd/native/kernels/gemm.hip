// MFMA bf16 GEMM with fused prologue/epilogue for the linear layers.
//
//   C[M,N] (+)= act( A[M,K] · B[K,N] + bias[N] )
//
// * A, B: fp32 or bf16 in global memory, either layout (``trans`` flags), converted
//   to bf16 while staging through LDS; f32 accumulation in the MFMA accumulators
//   (v_mfma_f32_16x16x32_bf16, wave64: each wave owns a 32x32 output tile = 2x2
//   MFMA fragments).
// * A prologue: optional activation-gradient mask read from the saved forward
//   activation (ReLU: y>0, GELU: gelu'(z)) so dgrad/wgrad consume dY⊙act'(·)
//   without a separate threshold_backward kernel (K9).
// * Epilogue: bias, ReLU / GELU(erf), optional pre-activation side output (for the
//   GELU backward), output dtype f32 / bf16, accumulate into C (persistent
//   fp32 grads), optional row-sum of the masked A into ``rowsum`` (the bias
//   gradient of a wgrad, fused: no separate column-sum kernel).
// * Split-K across blocks with f32 atomics when the tile grid is too small to
//   fill 256 CUs (only for linear epilogues into f32 accumulators).
// * Block ids are remapped XCD-aware (tiles sharing an A panel share an L2).
#include "rk_common.h"

using namespace rk;

namespace {

constexpr int BK = 32;
constexpr int PAD = 8;  // bf16 elements of row padding in LDS (80-byte rows)
constexpr int LDS_ROW = BK + PAD;

struct GemmArgs {
  const void* a;
  const void* a_mask;
  const void* b;
  void* c;
  void* c_pre;  // optional pre-activation output (same layout/dtype as C)
  const float* bias;
  float* rowsum;
  int64_t lda, ldb, ldc, ld_mask;
  int M, N, K;
  int a_dt, b_dt, c_dt, mask_dt;
  int a_trans, b_trans;
  int mask_mode;  // 0 none, 1 relu'(m) = m>0, 2 gelu'(m)
  int act;        // 0 none, 1 relu, 2 gelu(erf)
  int accumulate; // C += result
  int splitk;     // >1: atomics into f32 C
  int k_per_split;
};

__device__ __forceinline__ float load_any(const void* p, int dt, int64_t i) {
  return dt == BF16 ? bf2f(((const uint16_t*)p)[i]) : ((const float*)p)[i];
}

__device__ __forceinline__ float apply_mask(float v, float m, int mode) {
  if (mode == 1) return m > 0.f ? v : 0.f;
  if (mode == 2) return v * gelu_grad(m);
  return v;
}

// Load 8 consecutive elements (contiguous in memory) as f32; element i is valid when i < valid.
// Branch-free (clamped address + select): a conditional load makes hipcc branch and wait per
// element.  With vec_ok (uniform) the caller guarantees valid is 0 or 8 for every lane.
__device__ __forceinline__ void load8(const void* p, int dt, int64_t base, int valid, bool vec_ok, float out[8]) {
  if (vec_ok) {
    const int64_t o = valid > 0 ? base : 0;
    if (dt == BF16) {
      const uint4 v = *(const uint4*)((const uint16_t*)p + o);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        out[2 * i] = valid > 0 ? __uint_as_float(w[i] << 16) : 0.f;
        out[2 * i + 1] = valid > 0 ? __uint_as_float(w[i] & 0xffff0000u) : 0.f;
      }
    } else {
      const float4 v0 = *(const float4*)((const float*)p + o);
      const float4 v1 = *(const float4*)((const float*)p + o + 4);
      const float t[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) out[i] = valid > 0 ? t[i] : 0.f;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = load_any(p, dt, i < valid ? base + i : 0);
      out[i] = i < valid ? v : 0.f;
    }
  }
}

// Stage a ROWS x BK tile of a logical [rows, K] operand into LDS as [row][k] bf16.
// trans == 0: element (r, k) at ptr[r*ld + k]; trans == 1: at ptr[k*ld + r].
// With a mask (A operand only) the same addressing applies to the mask tensor.
// Returns this thread's contribution to the row sums of the staged (masked) values
// via `rs` (only meaningful when rowsum is requested).
template <int ROWS, int NT>
__device__ __forceinline__ void stage(uint16_t* lds, const void* p, int dt, int64_t ld, int trans, int row0, int nrows,
                                      int k0, int K, const void* mask, int mdt, int64_t ldm, int mmode, bool vec_p,
                                      bool vec_m, float* rowacc) {
  const int tid = threadIdx.x;
  for (int e = tid * 8; e < ROWS * BK; e += NT * 8) {
    float v[8], m[8];
    if (!trans) {
      const int r = e / BK, kk = e % BK;
      const int gr = row0 + r, gk = k0 + kk;
      const int valid = (gr < nrows) ? max(0, min(8, K - gk)) : 0;
      const int64_t off = (int64_t)gr * ld + gk;
      load8(p, dt, off, valid, vec_p, v);
      if (mmode) {
        load8(mask, mdt, (int64_t)gr * ldm + gk, valid, vec_m, m);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = apply_mask(v[i], m[i], mmode);
      }
      uint4 packed;
      uint32_t* w = (uint32_t*)&packed;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
      *(uint4*)(lds + r * LDS_ROW + kk) = packed;
      if (rowacc) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[i];
        rowacc[0] += s;  // caller maps e -> row
      }
    } else {
      const int kk = e / ROWS, r = e % ROWS;
      const int gr = row0 + r, gk = k0 + kk;
      const int valid = (gk < K) ? max(0, min(8, nrows - gr)) : 0;
      const int64_t off = (int64_t)gk * ld + gr;
      load8(p, dt, off, valid, vec_p, v);
      if (mmode) {
        load8(mask, mdt, (int64_t)gk * ldm + gr, valid, vec_m, m);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = apply_mask(v[i], m[i], mmode);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) lds[(r + i) * LDS_ROW + kk] = f2bf(v[i]);
    }
  }
}

template <int WM, int WN>
__global__ void __launch_bounds__(64 * WM * WN) gemm_kernel(GemmArgs g) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BM = 32 * WM, BN = 32 * WN;
  __shared__ __attribute__((aligned(16))) uint16_t As[BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BN * LDS_ROW];
  __shared__ float rows_lds[BM];

  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / ntiles;
  const int tile = lin % ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int kb = split * g.k_per_split, ke = min(g.K, kb + g.k_per_split);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // vector staging needs 16-byte alignment AND all-or-nothing 8-element groups (extent % 8 == 0)
  const bool vec_a = ((uintptr_t)g.a % 16 == 0) && ((g.lda * (g.a_dt == BF16 ? 2 : 4)) % 16 == 0) &&
                     ((g.a_trans ? g.M : g.K) % 8 == 0);
  const bool vec_b = ((uintptr_t)g.b % 16 == 0) && ((g.ldb * (g.b_dt == BF16 ? 2 : 4)) % 16 == 0) &&
                     ((g.b_trans ? g.N : g.K) % 8 == 0);
  const bool vec_m = g.a_mask && vec_a && ((uintptr_t)g.a_mask % 16 == 0) &&
                     ((g.ld_mask * (g.mask_dt == BF16 ? 2 : 4)) % 16 == 0);
  const bool want_rows = g.rowsum != nullptr && tn == 0 && !g.a_trans;
  const bool want_rows_t = g.rowsum != nullptr && tn == 0 && g.a_trans;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float rowacc = 0.f;
  if (want_rows_t)
    for (int i = threadIdx.x; i < BM; i += NT) rows_lds[i] = 0.f;

  for (int k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();
    stage<BM, NT>(As, g.a, g.a_dt, g.lda, g.a_trans, row0, g.M, k0, ke, g.a_mask, g.mask_dt, g.ld_mask, g.mask_mode,
                  vec_a, vec_m, want_rows ? &rowacc : nullptr);
    stage<BN, NT>(Bs, g.b, g.b_dt, g.ldb, g.b_trans, col0, g.N, k0, ke, nullptr, 0, 0, 0, vec_b, false, nullptr);
    __syncthreads();
    if (want_rows_t) {  // row sums of a transposed A tile: read back from LDS
      for (int r = threadIdx.x; r < BM; r += NT) {
        float s = 0.f;
        for (int kk = 0; kk < BK; ++kk) s += bf2f(As[r * LDS_ROW + kk]);
        rows_lds[r] += s;
      }
    }
    const int fr = lane & 15, fk = (lane >> 4) * 8;
    bf16x8 af[2], bfg[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = *(const bf16x8*)(As + (wm * 32 + i * 16 + fr) * LDS_ROW + fk);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfg[j] = *(const bf16x8*)(Bs + (wn * 32 + j * 16 + fr) * LDS_ROW + fk);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
  }

  // ---- bias-gradient row sums (blocks of the first N tile only) ----
  if (want_rows) {
    // stage(): thread t handled groups e = t*8 + n*NT*8 -> row e/BK; with NT*8 % BK == 0 the row
    // index advances by NT*8/BK per iteration, so each thread's groups map to rows r0 + n*step.
    // We accumulated all of them into one scalar, which is only valid when each thread maps to a
    // single row: true when BM*BK <= NT*8 (one iteration).  Guarded on the host.
    __syncthreads();
    for (int i = threadIdx.x; i < BM; i += NT) rows_lds[i] = 0.f;
    __syncthreads();
    const int r = (threadIdx.x * 8) / BK;
    if (r < BM) atomicAdd(&rows_lds[r], rowacc);
    __syncthreads();
  }
  if (want_rows || want_rows_t) {
    __syncthreads();
    for (int r = threadIdx.x; r < BM; r += NT)
      if (row0 + r < g.M) atomicAdd(g.rowsum + row0 + r, rows_lds[r]);
  }

  // ---- epilogue ----
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = col0 + wn * 32 + j * 16 + fr;
      if (col >= g.N) continue;
      const float bias = (g.bias && split == 0) ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * 32 + i * 16 + fq * 4 + r;
        if (row >= g.M) continue;
        float v = acc[i][j][r] + bias;
        const int64_t off = (int64_t)row * g.ldc + col;
        if (g.splitk > 1) {
          atomicAdd((float*)g.c + off, v);
          continue;
        }
        if (g.c_pre) {
          if (g.c_dt == BF16) ((uint16_t*)g.c_pre)[off] = f2bf(v);
          else ((float*)g.c_pre)[off] = v;
        }
        if (g.act == 1) v = fmaxf(v, 0.f);
        else if (g.act == 2) v = 0.5f * v * (1.f + erff(v * 0.7071067811865476f));
        if (g.c_dt == BF16) {
          uint16_t* c = (uint16_t*)g.c;
          if (g.accumulate) v += bf2f(c[off]);
          c[off] = f2bf(v);
        } else {
          float* c = (float*)g.c;
          if (g.accumulate) v += c[off];
          c[off] = v;
        }
      }
    }
  }
}

}  // namespace

RK_API int rk_gemm(const void* a, int a_dt, int64_t lda, int a_trans, const void* a_mask, int mask_dt, int64_t ld_mask,
                   int mask_mode, const void* b, int b_dt, int64_t ldb, int b_trans, void* c, int c_dt, int64_t ldc,
                   void* c_pre, const float* bias, int act, int accumulate, float* rowsum, int M, int N, int K,
                   int splitk, int cfg, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  // operands are bf16 or f32 (anything else would be read with the wrong element size)
  auto dt_ok = [](int d) { return d == F32 || d == BF16; };
  if (!dt_ok(a_dt) || !dt_ok(b_dt) || !dt_ok(c_dt)) return (int)hipErrorInvalidValue;
  GemmArgs g;
  g.a = a; g.a_mask = a_mask; g.b = b; g.c = c; g.c_pre = c_pre; g.bias = bias; g.rowsum = rowsum;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ld_mask = ld_mask;
  g.M = M; g.N = N; g.K = K;
  g.a_dt = a_dt; g.b_dt = b_dt; g.c_dt = c_dt; g.mask_dt = mask_dt;
  g.a_trans = a_trans; g.b_trans = b_trans; g.mask_mode = a_mask ? mask_mode : 0;
  g.act = act; g.accumulate = accumulate;
  if (splitk < 1) splitk = 1;
  if (splitk > 1 && (c_dt != F32 || act != 0 || c_pre)) return (int)hipErrorInvalidValue;
  int kps = (K + splitk - 1) / splitk;
  kps = ((kps + BK - 1) / BK) * BK;
  splitk = (K + kps - 1) / kps;
  g.splitk = splitk;
  g.k_per_split = kps;
  if (cfg == 0) {  // 64x64 tile, 4 waves
    if (rowsum && !a_trans && 64 * BK > 256 * 8) return (int)hipErrorInvalidValue;
    const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
    gemm_kernel<2, 2><<<tiles * splitk, 256, 0, s>>>(g);
  } else {  // 32x32 tile, 1 wave
    if (rowsum && !a_trans) return (int)hipErrorInvalidValue;  // 32*32 > 64*8: multi-row per thread
    const int tiles = ((M + 31) / 32) * ((N + 31) / 32);
    gemm_kernel<1, 1><<<tiles * splitk, 64, 0, s>>>(g);
  }
  return (int)hipGetLastError();
}
