// Large bf16 MFMA GEMM for the transformer projections (ViT-B/16 qkv, proj, fc1,
// fc2 in all three directions) and, through the same core, anything else shaped like them.
//
//   C[M,N] (op)= epi( sum_k A(m,k) * B(n,k) )           bf16 operands, f32 accumulation
//
// Operand layouts (per operand, template flag):
//   row   ("K-contiguous")  A(m,k) = a[m*lda + k]   e.g. activations X[M,K], nn.Linear W[N,K]
//   kmaj  ("K-major")       A(m,k) = a[k*lda + m]   e.g. W read as [K_out][K_in] for the dgrad,
//                                                     dY / X read token-major for the wgrad
// so forward (row,row), dgrad (row,kmaj) and wgrad (kmaj,kmaj) all run without a transpose pass.
//
// Design for gfx950 (cdna guide §5):
// * 512 threads = 8 waves as 2 (M) x 4 (N); block tile BM x BN x 64 (256x256, 256x128, 128x128);
//   each wave owns (BM/2) x (BN/4) as 16x16 fragments of v_mfma_f32_16x16x32_bf16.
// * Global -> LDS by global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip, 1 KiB per wave
//   instruction), double-buffered: the DMA of k-tile t+1 is in flight while tile t is consumed;
//   one barrier per k-tile.
// * LDS images are lane-linear (the DMA writes base + 16*lane), so the bank-conflict swizzles
//   are applied to the per-lane SOURCE address and undone on the read (guide rule 21):
//     row image  [rows][64 k] (128-B rows):  16-B slot ^= (row >> 1) & 7
//                -> every 16-lane ds_read_b128 group covers all 16 slots of a bank row;
//     kmaj image [64 k][R cols] (2R-B rows): 16-B slot ^= ((k & 3) | ((k >> 1) & 4)) << 1
//                -> the two ds_read_b64_tr_b16 (hardware transpose) reads of a fragment hit
//                   16 distinct slots per 32-lane half.
// * MFMA operands swapped (B fragment as the A operand) so every lane holds 4 CONSECUTIVE output
//   columns: 8-byte bf16 / 16-byte f32 epilogue stores.
// * Epilogue: + bias[n]; GELU (optionally also storing the pre-activation for the backward) or
//   ReLU; or multiply by gelu'(aux[m][n]) / relu'(aux) (the dgrad of an activation fused into the
//   GEMM that produces its input gradient); f32 or bf16 out; C += (persistent f32 grads);
//   split-K over blocks with f32 atomics (weight gradients: few output tiles, long K).
// * Optional row sums of A (bias gradient of a wgrad: db[m] = sum_k dY(m,k)) from extra MFMAs
//   against a ones fragment, spread over the 4 N-waves of the blocks in tile column 0.
// * Block ids remapped XCD-aware (consecutive tiles sharing an A panel share an L2).
#include "mgemm_core.h"

using namespace rk;

namespace {

template <int BM, int BN, int BK, int NS, int WM, int WN, int OCC, bool AK, bool BKM>
__global__ void __launch_bounds__(64 * WM * WN, OCC * WM * WN / 4) mgemm_kernel(MArgs g) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;  // per-wave tile
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int KK = BK / 32;                // MFMA k-steps per k-tile
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NL = (BM + BN) * BK / (512 * NW);  // LDS-DMA instructions per wave per k-tile
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE_BYTES];

  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / ntiles;
  const int tile = lin % ntiles;
  int tm, tn;
  grouped_tile(tile, tiles_m, tiles_n, g.tgroup, tm, tn);
  const int row0 = tm * BM, col0 = tn * BN;
  const int kb = split * g.k_per_split;
  const int ke = min(g.K, kb + g.k_per_split);
  const int nt = (ke - kb + BK - 1) / BK;  // the last k-tile may be partial (K % BK != 0)
  const int klast = (ke - kb) - (nt - 1) * BK;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // bias-gradient row sums: tile column 0 only; wave wn sums A fragments i = wn, wn+WN, ...
  const bool want_rows = g.rowsum != nullptr && tn == 0;
  constexpr int FR = (FM + WN - 1) / WN;
  f32x4 racc[FR];
#pragma unroll
  for (int i = 0; i < FR; ++i) racc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  Stager<BM, BK, AK, NW> sa;
  Stager<BN, BK, BKM, NW> sb;
  sa.init(g.lda, row0, g.M, wid, lane);
  sb.init(g.ldb, col0, g.N, wid, lane);
  // byte step of one k-tile: row image BK elements along the row, kmaj image BK rows
  const int64_t a_step = AK ? (int64_t)BK * g.lda * 2 : BK * 2;
  const int64_t b_step = BKM ? (int64_t)BK * g.ldb * 2 : BK * 2;
  const char* a_k0 = (const char*)g.a + (AK ? (int64_t)kb * g.lda * 2 : (int64_t)kb * 2);
  const char* b_k0 = (const char*)g.b + (BKM ? (int64_t)kb * g.ldb * 2 : (int64_t)kb * 2);
  auto issue = [&](int t) {
    char* buf = smem + (t % NS) * STAGE_BYTES;
    if (t + 1 < nt || klast == BK) {
      sa.issue(a_k0 + t * a_step, buf, wid);
      sb.issue(b_k0 + t * b_step, buf + A_BYTES, wid);
    } else {
      const char* zero = (const char*)g_mgemm_zero;
      sa.issue_tail(a_k0 + t * a_step, buf, wid, lane, klast, zero);
      sb.issue_tail(b_k0 + t * b_step, buf + A_BYTES, wid, lane, klast, zero);
    }
  };
  FragReader<BM, BK, AK, FM> ra;
  FragReader<BN, BK, BKM, FN> rb;
  ra.init(wm * TM, lane);
  rb.init(wn * TN, lane);
  // side inputs of the epilogue (gelu'/relu' operand, or the old bf16 C of an accumulate), loaded
  // now so their latency hides under the main loop instead of serialising the epilogue
  uint2 side[FM][FN];
  {
    const uint16_t* src = (g.epi == kMulGeluGrad || g.epi == kMulReluGrad) ? g.aux
                          : (g.accumulate && g.c_dt == BF16 && g.splitk == 1) ? (const uint16_t*)g.c : nullptr;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int m = min(row0 + wm * TM + i * 16 + (lane & 15), g.M - 1);
        const int n = min(col0 + wn * TN + j * 16 + 4 * (lane >> 4), g.N - 4);
        side[i][j] = src ? *(const uint2*)(src + (int64_t)m * g.ldc + n) : make_uint2(0u, 0u);
      }
  }

  // prologue: NS-1 k-tiles in flight
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nt) issue(t);

  for (int t = 0; t < nt; ++t) {
    // tile t has landed once at most the tiles issued after it (up to t+NS-2) are outstanding
    wait_vm((min(nt - 1, t + NS - 2) - t) * NL);
    // every wave's share of tile t is in LDS, and every wave has consumed tile t-1 (its
    // fragments fed MFMAs before the wave got here): refill tile t-1's slot with tile t+NS-1
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < nt) issue(t + NS - 1);
    const char* As = smem + (t % NS) * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = rb.get(Bs, j, kk);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = ra.get(As, i, kk);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      if (want_rows) {  // static fragment index, wave-uniform condition (no runtime-indexed arrays)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          if (i % WN == wn) racc[i / WN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[i], racc[i / WN], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: lane holds C[m][n..n+3], m = .. + (lane & 15), n = .. + 4 * (lane >> 4) ----
  if (want_rows && lane < 16) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = row0 + wm * TM + i * 16 + lane;
      if (i % WN == wn && m < g.M) atomicAdd(g.rowsum + m, racc[i / WN][0]);
    }
  }
  store_tile<FM, FN, true>(g, acc, side, row0 + wm * TM, col0 + wn * TN, lane, split);
}

// Large-tile kernel (one block per CU, 8 waves): BM x BN x 64 k-tiles in a 2-slot LDS ring, the
// k-tile consumed in 4 phases (k-half x M-half of the wave's fragments).  Each phase issues the
// LDS reads of the NEXT phase's operands, then its 8..16 MFMAs, so fragment reads run under the
// matrix cores instead of in front of them (operands in 4 named register sets: B of the current /
// next k-half, A of the current / next phase).  One barrier per k-tile, in its last phase: wait for
// tile t+1's DMA, then refill tile t's slot with tile t+2 and read tile t+1's first operands.
// Per-wave tile (BM/WM) x (BN/WN): with 128 x 64 the LDS reads per MFMA are half those of the
// 64 x 32 wave tile of the 2-blocks-per-CU kernel, whose LDS port the MFMAs otherwise wait on.
template <int BM, int BN, int WM, int WN, bool AK, bool BKM>
__global__ void __launch_bounds__(64 * WM * WN, WM * WN / 4) mgemm_phase_kernel(MArgs g) {
  constexpr int BK = 64, NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16, FH = FM / 2;
  static_assert(FM % 2 == 0, "phases split the wave's A fragments in halves");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES];

  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin / tiles_n, tn = lin % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int nt = (g.K + BK - 1) / BK;
  const int klast = g.K - (nt - 1) * BK;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stager<BM, BK, AK, NW> sa;
  Stager<BN, BK, BKM, NW> sb;
  sa.init(g.lda, row0, g.M, wid, lane);
  sb.init(g.ldb, col0, g.N, wid, lane);
  constexpr int NL = (BM + BN) * BK / (512 * NW);
  const int64_t a_step = AK ? (int64_t)BK * g.lda * 2 : BK * 2;
  const int64_t b_step = BKM ? (int64_t)BK * g.ldb * 2 : BK * 2;
  auto issue = [&](int t) {
    char* buf = smem + (t & 1) * STAGE_BYTES;
    if (t + 1 < nt || klast == BK) {
      sa.issue((const char*)g.a + t * a_step, buf, wid);
      sb.issue((const char*)g.b + t * b_step, buf + A_BYTES, wid);
    } else {
      const char* zero = (const char*)g_mgemm_zero;
      sa.issue_tail((const char*)g.a + t * a_step, buf, wid, lane, klast, zero);
      sb.issue_tail((const char*)g.b + t * b_step, buf + A_BYTES, wid, lane, klast, zero);
    }
  };
  FragReader<BM, BK, AK, FM> ra;
  FragReader<BN, BK, BKM, FN> rb;
  ra.init(wm * TM, lane);
  rb.init(wn * TN, lane);

  bf16x8 Ba[FN], Bb[FN], Aa[FH], Ab[FH];
  auto readB = [&](bf16x8 (&dst)[FN], int t, int kk) {
    const char* Bs = smem + (t & 1) * STAGE_BYTES + A_BYTES;
#pragma unroll
    for (int j = 0; j < FN; ++j) dst[j] = rb.get(Bs, j, kk);
  };
  auto readA = [&](bf16x8 (&dst)[FH], int t, int kk, int mh) {
    const char* As = smem + (t & 1) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < FH; ++i) dst[i] = ra.get(As, mh * FH + i, kk);
  };
  // MFMAs of fragments i in [i0, i1) of an M-half; sched_barrier keeps the LDS reads placed between
  // two such groups where they are written: after the first MFMAs (whose operands arrived during
  // the previous phase, so hipcc's lgkmcnt wait in front of them costs nothing) and before the rest
  auto mma = [&](const bf16x8 (&B)[FN], const bf16x8 (&A)[FH], int mh, int i0, int i1) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < FH; ++i)
      if (i >= i0 && i < i1)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[mh * FH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[j], A[i], acc[mh * FH + i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int I0 = 1;  // MFMA rows issued ahead of each phase's prefetch

  issue(0);
  if (nt > 1) issue(1);
  if (nt > 1) wait_vm(NL); else wait_vm(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  readB(Ba, 0, 0);
  readA(Aa, 0, 0, 0);

  for (int t = 0; t < nt; ++t) {
    // phase 1: (k-half 0, M-half 0); prefetch A(0, 1)
    mma(Ba, Aa, 0, 0, I0);
    readA(Ab, t, 0, 1);
    mma(Ba, Aa, 0, I0, FH);
    // phase 2: (0, 1); prefetch B(1), A(1, 0)
    mma(Ba, Ab, 1, 0, I0);
    readB(Bb, t, 1);
    readA(Aa, t, 1, 0);
    mma(Ba, Ab, 1, I0, FH);
    // phase 3: (1, 0); prefetch A(1, 1)
    mma(Bb, Aa, 0, 0, I0);
    readA(Ab, t, 1, 1);
    mma(Bb, Aa, 0, I0, FH);
    // phase 4: (1, 1); cross into tile t+1
    mma(Bb, Ab, 1, 0, I0);
    if (t + 1 < nt) {
      wait_vm(0);  // this wave's share of tile t+1 (nothing younger is in flight)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of tile t are done
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (t + 2 < nt) issue(t + 2);  // into tile t's slot
      readB(Ba, t + 1, 0);
      readA(Aa, t + 1, 0, 0);
    }
    mma(Bb, Ab, 1, I0, FH);
  }

  const uint2 nos[FM][FN] = {};
  store_tile<FM, FN, false>(g, acc, nos, row0 + wm * TM, col0 + wn * TN, lane, 0);
}

// Deep-ring large-tile kernel: BM x BN x 32 k-tiles in a 4-slot LDS ring (3 tiles of DMA in
// flight behind the one being consumed: the L2-miss latency of the panel slices that other XCDs
// have not fetched yet is hidden ~3000 cycles deep), one block per CU, 8 waves.  Each k-tile is
// consumed in 2 phases (the wave's A fragments in halves); a phase issues the LDS reads of the
// next phase after its first MFMA row, so fragment reads run under the matrix cores.  B fragments
// alternate between two register sets by tile parity (loop unrolled by 2 tiles).
template <int BM, int BN, int WM, int WN, bool AK, bool BKM>
__global__ void __launch_bounds__(64 * WM * WN, WM * WN / 4) mgemm_deep_kernel(MArgs g) {
  constexpr int BK = 32, NS = 4, NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16, FH = FM / 2;
  static_assert(FM % 2 == 0, "phases split the wave's A fragments in halves");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NL = (BM + BN) * BK / (512 * NW);
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE_BYTES];

  const int tiles_n = (g.N + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin / tiles_n, tn = lin % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int nt = (g.K + BK - 1) / BK;
  const int klast = g.K - (nt - 1) * BK;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stager<BM, BK, AK, NW> sa;
  Stager<BN, BK, BKM, NW> sb;
  sa.init(g.lda, row0, g.M, wid, lane);
  sb.init(g.ldb, col0, g.N, wid, lane);
  const int64_t a_step = AK ? (int64_t)BK * g.lda * 2 : BK * 2;
  const int64_t b_step = BKM ? (int64_t)BK * g.ldb * 2 : BK * 2;
  auto issue = [&](int t) {
    char* buf = smem + (t % NS) * STAGE_BYTES;
    if (t + 1 < nt || klast == BK) {
      sa.issue((const char*)g.a + t * a_step, buf, wid);
      sb.issue((const char*)g.b + t * b_step, buf + A_BYTES, wid);
    } else {
      const char* zero = (const char*)g_mgemm_zero;
      sa.issue_tail((const char*)g.a + t * a_step, buf, wid, lane, klast, zero);
      sb.issue_tail((const char*)g.b + t * b_step, buf + A_BYTES, wid, lane, klast, zero);
    }
  };
  FragReader<BM, BK, AK, FM> ra;
  FragReader<BN, BK, BKM, FN> rb;
  ra.init(wm * TM, lane);
  rb.init(wn * TN, lane);

  bf16x8 Ba[FN], Bb[FN], Alo[FH], Ahi[FH];
  auto readB = [&](bf16x8 (&dst)[FN], int t) {
    const char* Bs = smem + (t % NS) * STAGE_BYTES + A_BYTES;
#pragma unroll
    for (int j = 0; j < FN; ++j) dst[j] = rb.get(Bs, j, 0);
  };
  auto readA = [&](bf16x8 (&dst)[FH], int t, int mh) {
    const char* As = smem + (t % NS) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < FH; ++i) dst[i] = ra.get(As, mh * FH + i, 0);
  };
  auto mma = [&](const bf16x8 (&B)[FN], const bf16x8 (&A)[FH], int mh, int i0, int i1) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < FH; ++i)
      if (i >= i0 && i < i1)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[mh * FH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[j], A[i], acc[mh * FH + i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  // the boundary into tile u: its DMA landed (tiles up to u+NS-2 may stay in flight) in every
  // wave, every wave finished reading tile u-1: refill u-1's slot with tile u+NS-1
  auto boundary = [&](int u) {
    wait_vm((min(nt - 1, u + NS - 2) - u) * NL);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (u + NS - 1 < nt) issue(u + NS - 1);
  };
  // one k-tile: phase 1 (B, Alo) prefetching Ahi; phase 2 (B, Ahi) crossing into tile t+1 and
  // prefetching its B (into BN) and Alo.  A macro, not a lambda taking array references: every
  // fragment array is then a distinct named register block (no copies between them).
#define RK_DEEP_TILE(t, B, BN)                        \
  do {                                                \
    mma(B, Alo, 0, 0, 1);                             \
    readA(Ahi, (t), 1);                               \
    mma(B, Alo, 0, 1, FH);                            \
    mma(B, Ahi, 1, 0, 1);                             \
    if ((t) + 1 < nt) {                               \
      boundary((t) + 1);                              \
      readB(BN, (t) + 1);                             \
      readA(Alo, (t) + 1, 0);                         \
    }                                                 \
    mma(B, Ahi, 1, 1, FH);                            \
  } while (0)

#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nt) issue(t);
  wait_vm((min(nt - 1, NS - 2)) * NL);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (NS - 1 < nt) issue(NS - 1);  // the ring's last slot (the boundaries refill from tile NS on)
  readB(Ba, 0);
  readA(Alo, 0, 0);
  for (int t = 0; t < nt; t += 2) {
    RK_DEEP_TILE(t, Ba, Bb);
    if (t + 1 < nt) RK_DEEP_TILE(t + 1, Bb, Ba);
  }
#undef RK_DEEP_TILE

  const uint2 nos[FM][FN] = {};
  store_tile<FM, FN, false>(g, acc, nos, row0 + wm * TM, col0 + wn * TN, lane, 0);
}

// Ping-pong kernel (tile 10; cdna guide §5 "256² 8-phase template", T1-T5): 256 x 256 x 64
// k-tiles, one PERSISTENT block per CU, 8 waves in two GROUPS of 4 (group wr owns output rows
// wr*128..+127 of a tile, wave wc of a group columns wc*64..+63).  Group 1 runs one barrier
// behind group 0, so on every SIMD (one wave of each group) one wave issues MFMAs while the other
// issues its LDS reads and LDS-DMAs: the matrix core does not wait on the LDS port or on staging.
// A k-tile is 4 phases; a phase = [R: fragment reads + one half-tile DMA, lgkmcnt(0)] barrier
// [M: 16 MFMAs = one 64 x 32 quadrant x K 64] barrier.  Quadrant order (mq,nq): 00 01 11 10, so
// each operand fragment is read once per k-tile: B (both nq) + A(mq 0) in phase 0, A(mq 1) in
// phase 2 (16 / 0 / 8 / 0 ds_read_b128 per wave; a 12 / 4 / 8 / 0 split measured slower).
// Persistence: block b owns output tiles pos(b), pos(b) + grid, ... (pos XCD-aware: the blocks
// of one XCD run neighbouring tiles) and consumes their k-tiles as ONE stream, so the DMA of the
// next tile's first k-tiles runs under the current tile's last MFMAs and the epilogue stores of a
// tile overlap the next tile's loads (no per-tile pipeline fill / drain, no lock-step store bursts).
// LDS: 2 stream-slot buffers x [A0 | A1 | B0 | B1] half-tiles of 128 rows x 64 k (16 KiB each,
// the swizzled lane-linear images of the other kernels).  Staging schedule, stream k-tile s read
// from buffer s&1: phase 0 DMAs A1 of s+1; phases 1-3 DMA B0, B1, A0 of s+2 into buffer s&1 --
// each only after every wave has retired (lgkmcnt(0) before a barrier) its last read of that
// half: B in phase 0, A0 in phase 2 (group 0), A1 in phase 2 (group 1, one barrier later), s+2's
// A1 then following in s+1's phase 0.  Phase 3 waits vmcnt(6) (the 3 half-tiles of s+2 stay in
// flight; loads retire in order, so older epilogue stores cannot satisfy the count early),
// retiring this wave's share of s+1; the two barriers that follow publish it to both groups.
template <bool KMAJ>
struct PStager {  // one 128-row (row image) / 128-column (kmaj image) half of a 64-deep k-tile
  uint32_t u[2], v[2];  // row: u = row in the half, v = k of the chunk; kmaj: u = k row, v = column
  __device__ __forceinline__ void init(int wid, int lane) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = (wid * 2 + i) * 64 + lane;  // 16-byte chunk of the lane-linear image
      if constexpr (!KMAJ) {
        const int r = q >> 3;
        u[i] = r;
        v[i] = ((q & 7) ^ rswz<64>(r)) * 8;
      } else {
        const int k = q >> 4;
        u[i] = k;
        v[i] = ((q & 15) ^ kswz<128>(k)) * 8;
      }
    }
  }
  // rows (cols) r0.. of k-tile kt; chunks at k >= kvalid come from the zero page.  (Addresses are
  // recomputed per DMA -- min, multiply-add, select -- which measured faster than precomputed
  // per-lane offsets plus a block-uniform edge branch.)
  __device__ __forceinline__ void issue(const uint16_t* base, int64_t ld, int r0, int rdim, int kt, int kvalid,
                                        char* lds, int wid) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint16_t* src;
      int kpos;
      if constexpr (!KMAJ) {
        const int gr = min(r0 + (int)u[i], rdim - 1);
        src = base + (int64_t)gr * ld + kt * 64 + v[i];
        kpos = v[i];
      } else {
        const int gc = min(r0 + (int)v[i], rdim - 8);
        src = base + (int64_t)(kt * 64 + (int)u[i]) * ld + gc;
        kpos = u[i];
      }
      if (kpos >= kvalid) src = (const uint16_t*)g_mgemm_zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (wid * 2 + i) * 1024), 16, 0, 0);
    }
  }
};

struct PCursor {  // one position of a block's k-tile stream
  int i, kt, r0, c0;
};

template <bool BKM>
__global__ void __launch_bounds__(512, 2) mgemm_pp_kernel(MArgs g) {
  constexpr int NW = 8;
  constexpr int HB = 128 * 64 * 2;  // half-tile bytes
  constexpr int BUF = 4 * HB;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF + 3 * 1024];  // + 3 tile-bias buffers
  (void)NW;
  float* const bias_lds = (float*)(smem + 2 * BUF);

  const int tiles_n = (g.N + 255) / 256;
  const int ntiles = ((g.M + 255) / 256) * tiles_n;
  const int grid = gridDim.x;
  const int pos = xcd_remap(blockIdx.x, grid);
  const int my_tiles = (ntiles - pos + grid - 1) / grid;
  const int nt = (g.K + 63) / 64;
  const int klast = g.K - (nt - 1) * 64;
  const int S = my_tiles * nt;  // k-tiles in this block's stream

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  PStager<false> sa;
  PStager<BKM> sb;
  sa.init(wid, lane);
  sb.init(wid, lane);
  auto place = [&](PCursor& c) {
    const int lin = pos + c.i * grid;
    const int tm = lin / tiles_n;
    c.r0 = tm * 256;
    c.c0 = (lin - tm * tiles_n) * 256;
  };
  auto advance = [&](PCursor c) {
    if (++c.kt == nt) {
      c.kt = 0;
      ++c.i;
      if (c.i < my_tiles) place(c);
    }
    return c;
  };
  // half h (0 = A0, 1 = A1, 2 = B0, 3 = B1; a constant at every call site) of stream slot s at c
  auto stage = [&](const PCursor& c, int s, int h) {
    char* dst = smem + (s & 1) * BUF + h * HB;
    const int kvalid = c.kt + 1 == nt ? klast : 64;
    if (h < 2) sa.issue(g.a, g.lda, c.r0 + h * 128, g.M, c.kt, kvalid, dst, wid);
    else sb.issue(g.b, g.ldb, c.c0 + (h - 2) * 128, g.N, c.kt, kvalid, dst, wid);
  };
  FragReader<128, 64, false, 8> ra;
  FragReader<128, 64, BKM, 4> rb;
  ra.init(0, lane);
  rb.init((wc & 1) * 64, lane);
  const int a_half = wr * HB, b_half = (2 + (wc >> 1)) * HB;

  bf16x8 Bf[2][2][2];  // [nq][fragment][k-step]
  bf16x8 Af[4][2];     // [fragment][k-step] of the current M quadrant
  auto readB = [&](const char* buf, int q) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) Bf[q][f][kk] = rb.get(buf + b_half, q * 2 + f, kk);
  };
  auto readA = [&](const char* buf, int mq) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) Af[f][kk] = ra.get(buf + a_half, mq * 4 + f, kk);
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto lds_done = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // M part of a phase: quadrant (mq, nq), K = 64
  auto mma = [&](int mq, int nq) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mq * 4 + f][nq * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(Bf[nq][j][kk], Af[f][kk], acc[mq * 4 + f][nq * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // bias[c0 .. c0+255] of tile i -> bias buffer i%3 (three: with one k-tile per tile, group 1
  // still reads tile i-1's bias while group 0 issues tile i+1's; waves 0-3, one 4-byte DMA per lane; counted
  // by those waves' vmcnt like the half-tiles it is issued with, and older than every half-tile
  // the phase-3 wait leaves in flight)
  auto stage_bias = [&](const PCursor& c) {
    if (g.bias != nullptr && wid < 4) {
      const int n = min(c.c0 + wid * 64 + lane, g.N - 1);
      __builtin_amdgcn_global_load_lds((const void*)(g.bias + n),
                                       (lds_void*)(smem + 2 * BUF + (c.i % 3) * 1024 + wid * 256), 4, 0, 0);
    }
  };
  // epilogue of tile c: + bias (from LDS), ReLU / GELU (pre-activation side output optional),
  // bf16 or f32 stores -- no global loads, so no vmcnt wait drains the next tile's DMAs
  auto epilogue = [&](const PCursor& c) {
    // the tile's bias by inline-asm LDS reads: a plain read of an LDS array that DMAs write makes
    // hipcc wait vmcnt(0) first, draining the next tile's half-tiles
    f32x4 b4[4];
    if (g.bias) {
      const uint32_t base = (uint32_t)(uintptr_t)(const lds_void*)(bias_lds + (c.i % 3) * 256 + wc * 64 + 4 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(b4[j]) : "v"(base), "i"(j * 64));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) b4[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int mbase = c.r0 + wr * 128;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = c.c0 + wc * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = mbase + i * 16 + (lane & 15);
        if (m >= g.M) continue;
        const int64_t off = (int64_t)m * g.ldc + n;
        float v[4] = {acc[i][j][0] + b4[j][0], acc[i][j][1] + b4[j][1], acc[i][j][2] + b4[j][2],
                      acc[i][j][3] + b4[j][3]};
        if (g.epi != kNone) {
          if (g.c_pre) {
            if (g.c_dt == BF16)
              *(uint2*)((uint16_t*)g.c_pre + off) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                                               (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
            else
              *(float4*)((float*)g.c_pre + off) = make_float4(v[0], v[1], v[2], v[3]);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = g.epi == kGelu ? gelu_f(v[e]) : fmaxf(v[e], 0.f);
        }
        if (g.c_dt == BF16)
          *(uint2*)((uint16_t*)g.c + off) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                                       (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
        else
          *(float4*)((float*)g.c + off) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };

  // prologue: slot 0 whole, slot 1's B0, B1, A0 (the loop's first phase 0 adds its A1)
  PCursor c0{0, 0, 0, 0};
  place(c0);
  PCursor c1 = advance(c0);
  PCursor c2 = advance(c1);
  stage_bias(c0);
  stage(c0, 0, 2); stage(c0, 0, 3); stage(c0, 0, 0); stage(c0, 0, 1);
  if (S > 1) {
    stage(c1, 1, 2); stage(c1, 1, 3); stage(c1, 1, 0);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  if (wr == 1) bar();  // group 1 runs one barrier behind

  for (int s = 0; s < S; ++s) {
    const char* buf = smem + (s & 1) * BUF;
    const bool more1 = s + 1 < S, more2 = s + 2 < S;
    // phase 0: quadrant (0, 0)
    readB(buf, 0);
    readB(buf, 1);
    readA(buf, 0);
    if (more1) {
      if (c1.kt == 0) stage_bias(c1);
      stage(c1, s + 1, 1);
    }
    lds_done();
    bar();
    mma(0, 0);
    bar();
    // phase 1: quadrant (0, 1)
    if (more2) stage(c2, s + 2, 2);
    bar();
    mma(0, 1);
    bar();
    // phase 2: quadrant (1, 1)
    readA(buf, 1);
    if (more2) stage(c2, s + 2, 3);
    lds_done();
    bar();
    mma(1, 1);
    bar();
    // phase 3: quadrant (1, 0); retire this wave's share of s+1
    if (more2) {
      stage(c2, s + 2, 0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    mma(1, 0);
    bar();
    if (c0.kt + 1 == nt) {  // the tile is complete: epilogue under the next tile's DMAs
      epilogue(c0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    c0 = c1;
    c1 = c2;
    c2 = advance(c2);
  }
  if (wr == 0) bar();  // equal barrier counts in both groups
}

template <int BM, int BN, int BK, int NS, int WM, int WN, int OCC>
int launch_tile(const MArgs& g, int a_kmaj, int b_kmaj, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  const dim3 grid(tiles * g.splitk), block(64 * WM * WN);
  if (!a_kmaj && !b_kmaj) mgemm_kernel<BM, BN, BK, NS, WM, WN, OCC, false, false><<<grid, block, 0, s>>>(g);
  else if (!a_kmaj && b_kmaj) mgemm_kernel<BM, BN, BK, NS, WM, WN, OCC, false, true><<<grid, block, 0, s>>>(g);
  else if (a_kmaj && b_kmaj) mgemm_kernel<BM, BN, BK, NS, WM, WN, OCC, true, true><<<grid, block, 0, s>>>(g);
  else return (int)hipErrorInvalidValue;  // (kmaj, row) has no user
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN>
int launch_deep(const MArgs& g, int a_kmaj, int b_kmaj, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  const dim3 grid(tiles), block(64 * WM * WN);
  if (!a_kmaj && !b_kmaj) mgemm_deep_kernel<BM, BN, WM, WN, false, false><<<grid, block, 0, s>>>(g);
  else if (!a_kmaj && b_kmaj) mgemm_deep_kernel<BM, BN, WM, WN, false, true><<<grid, block, 0, s>>>(g);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN>
int launch_phase(const MArgs& g, int a_kmaj, int b_kmaj, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  const dim3 grid(tiles), block(64 * WM * WN);
  if (!a_kmaj && !b_kmaj) mgemm_phase_kernel<BM, BN, WM, WN, false, false><<<grid, block, 0, s>>>(g);
  else if (!a_kmaj && b_kmaj) mgemm_phase_kernel<BM, BN, WM, WN, false, true><<<grid, block, 0, s>>>(g);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// compute units of the current device (cached; the persistent kernels size their grid by it)
int rk_num_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cus[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

int launch_pp(const MArgs& g, int a_kmaj, int b_kmaj, hipStream_t s) {
  const int tiles = ((g.M + 255) / 256) * ((g.N + 255) / 256);
  if (a_kmaj || g.accumulate || g.epi > kGelu) return (int)hipErrorInvalidValue;
  const int grid = std::min(tiles, rk_num_cus());  // persistent: one block per CU
  if (b_kmaj) mgemm_pp_kernel<true><<<grid, 512, 0, s>>>(g);
  else mgemm_pp_kernel<false><<<grid, 512, 0, s>>>(g);
  return (int)hipGetLastError();
}

// k-tile depth of each tile config (the K granularity a caller must respect)
constexpr int kTileBK[] = {32, 64, 64, 64, 64, 32};

// dst[i] (+)= sum_s part[s][i]: the combine of a library split-K weight gradient (strided-batched
// partial products, bf16 / fp16 or f32) straight into the fp32 weight.grad — one pass instead of a
// reduction launch, a temporary and an accumulation launch.  8 elements per thread, all split
// loads issued before the first add.  DT: 0 f32, 1 bf16, 2 fp16 (the _lib dtype codes).
template <int DT>
__device__ __forceinline__ void slab_add16(float (&acc)[8], const uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if constexpr (DT == 1) {
      acc[2 * k] += __uint_as_float(w[k] << 16);
      acc[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
    } else {
      acc[2 * k] += h2f((uint16_t)(w[k] & 0xffffu));
      acc[2 * k + 1] += h2f((uint16_t)(w[k] >> 16));
    }
  }
}

template <int DT>
__global__ void __launch_bounds__(256) slab_acc_kernel(const void* __restrict__ part, int splits, int64_t count,
                                                       float* __restrict__ dst, int accumulate) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= count) return;
  float acc[8];
  if (accumulate) {
    const float4 d0 = *(const float4*)(dst + i), d1 = *(const float4*)(dst + i + 4);
    acc[0] = d0.x; acc[1] = d0.y; acc[2] = d0.z; acc[3] = d0.w;
    acc[4] = d1.x; acc[5] = d1.y; acc[6] = d1.z; acc[7] = d1.w;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  }
  int s = 0;
  for (; s + 4 <= splits; s += 4) {
    if constexpr (DT != 0) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const uint4*)((const uint16_t*)part + (int64_t)(s + u) * count + i);
#pragma unroll
      for (int u = 0; u < 4; ++u) slab_add16<DT>(acc, v[u]);
    } else {
      float4 v[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* p = (const float*)part + (int64_t)(s + u) * count + i;
        v[u][0] = *(const float4*)p;
        v[u][1] = *(const float4*)(p + 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc[0] += v[u][0].x; acc[1] += v[u][0].y; acc[2] += v[u][0].z; acc[3] += v[u][0].w;
        acc[4] += v[u][1].x; acc[5] += v[u][1].y; acc[6] += v[u][1].z; acc[7] += v[u][1].w;
      }
    }
  }
  for (; s < splits; ++s) {
    if constexpr (DT != 0) {
      slab_add16<DT>(acc, *(const uint4*)((const uint16_t*)part + (int64_t)s * count + i));
    } else {
      const float* p = (const float*)part + (int64_t)s * count + i;
      const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
      acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
      acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
    }
  }
  *(float4*)(dst + i) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *(float4*)(dst + i + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

}  // namespace

// dst[count] (+)= sum over `splits` partial arrays part[s][count] (dt 0 f32 / 1 bf16 / 2 fp16); count % 8 == 0,
// 16-byte aligned pointers.
RK_API int rk_slab_acc(const void* part, int dt, int splits, int64_t count, float* dst, int accumulate,
                       hipStream_t s) {
  if (count <= 0) return 0;
  if (count % 8 || splits < 1 || dt < 0 || dt > 2 || ((uintptr_t)part | (uintptr_t)dst) % 16)
    return (int)hipErrorInvalidValue;
  const int64_t blocks = (count / 8 + 255) / 256;
  if (dt == 1) slab_acc_kernel<1><<<(unsigned)blocks, 256, 0, s>>>(part, splits, count, dst, accumulate);
  else if (dt == 2) slab_acc_kernel<2><<<(unsigned)blocks, 256, 0, s>>>(part, splits, count, dst, accumulate);
  else slab_acc_kernel<0><<<(unsigned)blocks, 256, 0, s>>>(part, splits, count, dst, accumulate);
  return (int)hipGetLastError();
}

// Tile configs (BM x BN x BK, LDS ring depth, waves, resident blocks per CU):
//   0: 128x128x64 ring 2, 2x4 waves, 2/CU (64 KiB)    4: 128x128x64 ring 2, 2x2 waves, 2/CU (64 KiB)
//   5: 128x128x32 ring 4, 2x4 waves, 2/CU (64 KiB)
//   6: 256x256x64 phase-pipelined, 2x4 waves, 1/CU (128 KiB)   7: 256x128x64 phase, 4x2 waves (96 KiB)
//   8: 256x256x32 4-slot ring, 2x4 waves, 1/CU (128 KiB)      9: 256x128x32 4-slot ring, 4x2 (96 KiB)
//     10: 256x256x64 ping-pong (two staggered wave groups, 4 phases per k-tile), 1/CU (128 KiB)
//      (6-10: row x row and row x kmaj only; no split-K / row sums)
// (256x256, 256x128 and 128x256 tiles with 1-2 blocks per CU and 2-4 deep rings measured slower
// at every ViT shape on this loop structure: bench/mgemm_probe.py, profiles/r2_mgemm_probe.md)
// Requirements (hipErrorInvalidValue otherwise; the caller falls back): K % 8 == 0 (unless both
// operands are kmaj), N % 8 == 0,
// 16-byte aligned operands / leading dimensions, a kmaj operand's extent % 8 == 0.  splitk > 1
// needs `slab` = splitk*M*N f32 scratch: the partial tiles are summed (+bias, +C) by a second launch.
RK_API int rk_mgemm(const void* a, int64_t lda, int a_kmaj, const void* b, int64_t ldb, int b_kmaj, void* c, int c_dt,
                    int64_t ldc, void* c_pre, const float* bias, const void* aux, int epi, int accumulate,
                    float* rowsum, int M, int N, int K, int splitk, int tile, float* slab, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (tile != 0 && (tile < 4 || tile > 10)) return (int)hipErrorInvalidValue;
  if (tile >= 6 && (splitk > 1 || rowsum != nullptr || (a_kmaj && b_kmaj))) return (int)hipErrorInvalidValue;
  // a row-layout operand moves K in 16-byte chunks (K % 8); a kmaj one in whole k-rows (any K)
  if (K <= 0 || ((!a_kmaj || !b_kmaj) && K % 8) || N % 8 || (a_kmaj && M % 8) || ldc % 4) return (int)hipErrorInvalidValue;
  if (((uintptr_t)a | (uintptr_t)b) % 16 || (lda * 2) % 16 || (ldb * 2) % 16) return (int)hipErrorInvalidValue;
  if ((epi == kMulGeluGrad || epi == kMulReluGrad) && aux == nullptr) return (int)hipErrorInvalidValue;
  MArgs g;
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c; g.c_pre = c_pre; g.bias = bias;
  g.aux = (const uint16_t*)aux; g.rowsum = rowsum; g.slab = slab;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.c_dt = c_dt; g.epi = epi; g.accumulate = accumulate;
  g.lds_epi = 0;
  g.tgroup = 4;  // grouped tile walk (rk_common.h)
  g.dbg = 0;
  if (splitk < 1) splitk = 1;
  const int kq = 64;  // split boundaries on 64 (a multiple of every config's BK)
  int kps = ((K + kq - 1) / kq + splitk - 1) / splitk * kq;
  splitk = (K + kps - 1) / kps;
  if (splitk > 1 && (slab == nullptr || epi != kNone || c_pre)) return (int)hipErrorInvalidValue;
  g.splitk = splitk;
  g.k_per_split = kps;
  int rc;
  switch (tile) {
    case 0: rc = launch_tile<128, 128, 64, 2, 2, 4, 2>(g, a_kmaj, b_kmaj, s); break;
    case 4: rc = launch_tile<128, 128, 64, 2, 2, 2, 2>(g, a_kmaj, b_kmaj, s); break;
    case 6: rc = launch_phase<256, 256, 2, 4>(g, a_kmaj, b_kmaj, s); break;
    case 7: rc = launch_phase<256, 128, 4, 2>(g, a_kmaj, b_kmaj, s); break;
    case 8: rc = launch_deep<256, 256, 2, 4>(g, a_kmaj, b_kmaj, s); break;
    case 9: rc = launch_deep<256, 128, 4, 2>(g, a_kmaj, b_kmaj, s); break;
    case 10: rc = launch_pp(g, a_kmaj, b_kmaj, s); break;
    default: rc = launch_tile<128, 128, 32, 4, 2, 4, 2>(g, a_kmaj, b_kmaj, s); break;
  }
  if (rc || splitk == 1) return rc;
  launch_mgemm_reduce(slab, splitk, M, N, bias, c, c_dt, ldc, accumulate, s);
  return (int)hipGetLastError();
}
