// Persistent 256x256 GEMM with the output tile drained under the next tile's main loop
// (forward layout: A [M][K], B [N][K], both K-contiguous; C = A B^T [+ bias], 16-bit C).
//
// Why a new kernel: the one-wave-per-SIMD 256x256 tile (xgemm4.hip) runs its K = 768 main loop at
// ~20 us per tile but then spends ~8 us storing the tile, with every CU storing at once (32 MiB in
// one burst, HBM-write bound), plus a 2 us pipeline fill per tile and wave quantisation
// (profiles/r5_x4_trace.md).  Here:
//
// * persistent: one block per CU walks its tiles pos, pos + G, ... (XCD-aware remap + grouped
//   order); the LDS-DMA k-tile stream runs ACROSS tiles, so the next tile's first two k-tiles are
//   already landing while the current one finishes (no per-tile prologue);
// * 32x32x16 MFMAs: a 128x128 wave tile is 4 x 4 accumulators of 16 f32 (all 256 accumulator
//   registers) and one k16 step needs only 8 fragments (32 VGPRs); two fragment sets = 64 VGPRs,
//   which leaves room for the finished tile PACKED to bf16 in 128 VGPRs;
// * epilogue = pack only (accumulators + bias -> bf16, lane pairs swapped with permlane32 so every
//   store is 16 B per lane, T21): the 32 store instructions per wave are issued 4 per k-tile over
//   the next tile's first 8 k-tiles, as raw buffer stores (out-of-range lanes get an offset past
//   the buffer, so every store instruction is issued and the vmcnt counts below stay exact).  The
//   chip's store traffic is then spread over the whole kernel instead of one burst per tile.
//
// Per k-tile (64 deep, 2-stage LDS ring, 64 KiB per stage, image as xgemm4: [256][64] bf16 per
// operand, 16-byte chunk c of row r at c ^ ((r >> 1) & 7)):
//   step s = 0, 1, 2: 16 MFMAs on fragment set s & 1  ||  8 reads of step s + 1 into the other set
//                     (+ this k-tile's share of the previous tile's stores);
//   boundary        : lgkmcnt(0); vmcnt(#stores issued since) = k-tile q + 1 landed; ONE barrier;
//                     DMA of k-tile q + 2 into this k-tile's stage (everyone finished reading it);
//   step 3          : 16 MFMAs on set 1  ||  reads of step 0 of k-tile q + 1 into set 0.
// vmcnt counts rely on vector-memory ops completing in issue order (DMA loads and stores alike).
#include "mgemm_core.h"

#include <type_traits>

using namespace rk;

namespace {

constexpr int X5_BM = 256, X5_BN = 256, X5_BK = 64, X5_NT = 256;
constexpr int X5_ROWB = X5_BK * 2;        // 128-byte image rows
constexpr int X5_OPB = X5_BM * X5_ROWB;   // 32 KiB per operand per stage
constexpr int X5_STAGE = 2 * X5_OPB;      // A + B
constexpr int X5_NI = X5_OPB / (1024 * 4);  // 8 DMA instructions per operand per wave
constexpr int X5_NST = 32;                // packed 16-byte stores per wave per tile
constexpr int X5_NIM = 16;                // of which issued right at the epilogue (row blocks i = 0, 1)
constexpr int X5_NPK = X5_NST - X5_NIM;   // kept packed in VGPRs and issued under the next tile

template <int I>
using ic = std::integral_constant<int, I>;
template <bool B>
using bc = std::integral_constant<bool, B>;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;

__device__ __forceinline__ void mfma32(f32x16& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma32_0(f32x16& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}

// two f32 -> one packed 16-bit pair (one v_cvt_pk_bf16_f32 for bf16; RNE either way)
template <int CDT>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  if constexpr (CDT == BF16) {
    typedef __attribute__((ext_vector_type(2))) float f2_t;
    typedef __attribute__((ext_vector_type(2))) __bf16 b2_t;
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2_t{a, b}, b2_t));
  } else {
    return pack16(a, b, F16);
  }
}

struct X5Args {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const float* bias;
  int64_t lda, ldb, ldc;
  int M, N, K, c_dt;
};

template <int CDT, bool HASB>
__global__ void __launch_bounds__(X5_NT, 1) xgemm5_kernel(X5Args g) {
  // 2-stage ring + one 1-KiB bias row per wave (one __shared__ object: see the guide's trap 4(a))
  __shared__ __attribute__((aligned(1024))) char smem[2 * X5_STAGE + 4 * 1024];
  const int tiles_m = (g.M + X5_BM - 1) / X5_BM, tiles_n = (g.N + X5_BN - 1) / X5_BN;
  const int total = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int pos = xcd_remap(blockIdx.x, G);
  const int my = pos < total ? (total - pos + G - 1) / G : 0;
  const int U = g.K / X5_BK;
  const int S = my * U;  // k-tiles in this block's stream
  const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;

  // ---- DMA (xgemm4's lane pattern): lane l of a 1-KiB piece lands at image row l/8, slot l%8
  uint32_t va[2], vb[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = 8 * p + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    va[p] = (uint32_t)((lane >> 3) * g.lda * 2 + c * 16);
    vb[p] = (uint32_t)((lane >> 3) * g.ldb * 2 + c * 16);
  }
  // issue cursor: tile of the next DMA and its k-tile
  int iss_i = 0, iss_k = 0;
  const char *ia = nullptr, *ib = nullptr;
  int64_t ia_n = 0, ib_n = 0;
  auto iss_tile = [&](int i) {
    int tm, tn;
    grouped_tile(pos + i * G, tiles_m, tiles_n, 4, tm, tn);
    ia = (const char*)g.A + (int64_t)tm * X5_BM * g.lda * 2;
    ib = (const char*)g.B + (int64_t)tn * X5_BN * g.ldb * 2;
    ia_n = ((int64_t)g.M - tm * X5_BM) * g.lda * 2;
    ib_n = ((int64_t)g.N - tn * X5_BN) * g.ldb * 2;
  };
  if (my > 0) iss_tile(0);
  // one descriptor per operand and k-tile (rows past M / N read as zeros: the VGPR offset is
  // range-checked).  dma_begin(q) forms them for k-tile q (a k-tile past the stream gets an empty
  // descriptor: its 16 instructions still issue, so every vmcnt count stays static, and only write
  // zeros into a stage nobody reads any more); dma_one(k) issues instruction k (0-7 A, 8-15 B),
  // its row offset added at the instruction to an opaque copy of the lane part (no 16 hoisted sums).
  __amdgpu_buffer_rsrc_t d_ra, d_rb;
  char* d_st = smem;
  auto dma_begin = [&](int q) {
#if defined(__HIP_DEVICE_COMPILE__)
    const bool real = q < S;
    d_st = smem + (q & 1) * X5_STAGE;
    auto clampn = [](int64_t b) { return (int)(b < 0 ? 0 : (b > 0x7fffffff ? 0x7fffffff : b)); };
    const char* pa = real ? ia + iss_k * X5_ROWB : (const char*)g.A;
    const char* pb = real ? ib + iss_k * X5_ROWB : (const char*)g.B;
    d_ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(pa), (short)0, real ? clampn(ia_n - iss_k * X5_ROWB) : 0,
                                             0x00020000);
    d_rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(pb), (short)0, real ? clampn(ib_n - iss_k * X5_ROWB) : 0,
                                             0x00020000);
    if (real && ++iss_k == U) {
      iss_k = 0;
      if (++iss_i < my) iss_tile(iss_i);
    }
#endif
  };
  auto dma_one = [&](int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int op = k >> 3, i = k & 7;
    const int row0 = 64 * w + 8 * i;
    uint32_t vo = op ? vb[i & 1] : va[i & 1];
    asm volatile("" : "+v"(vo));
    vo += (uint32_t)(row0 * (op ? g.ldb : g.lda) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(op ? d_rb : d_ra, (lds_void*)(d_st + op * X5_OPB + row0 * X5_ROWB), 16,
                                             vo, 0, 0, 0);
#endif
  };
  auto dma_next = [&](int q) {  // a whole k-tile at once (prologue)
    dma_begin(q);
#pragma unroll
    for (int k = 0; k < 16; ++k) dma_one(k);
  };

  // ---- fragment reads: 32x32x16 operand of rows r0 .. r0+31 at k16 step s: lane reads row
  // r0 + l32, chunk 2s + h (slot ^ ((l32 >> 1) & 7)); fragment i = +i * 4096 (32 rows) immediate
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const lds_void*)smem;
  const int fsw = (l32 >> 1) & 7;
  // per-lane part of step s's address (A image, stage 0); B and stage 1 differ by wave-uniform
  // amounts added per step (4 VGPRs instead of 16)
  uint32_t la[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    la[s] = lds0 + wm * 128 * X5_ROWB + (uint32_t)(l32 * X5_ROWB + (((2 * s + h) ^ fsw) * 16));
  const uint32_t bdelta = (uint32_t)(X5_OPB + (wn - wm) * 128 * X5_ROWB);
  // (the base goes through an empty asm so the sums are formed at each use, not hoisted out of
  // the loop into 16 live registers)
  auto ra = [&](int st, int s) {
    uint32_t v = la[s];
    asm volatile("" : "+v"(v));
    return v + (uint32_t)(st * X5_STAGE);
  };
  auto rb = [&](int st, int s) {
    uint32_t v = la[s];
    asm volatile("" : "+v"(v));
    return v + (uint32_t)(st * X5_STAGE) + bdelta;
  };
#define X5_RD(dst, a, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(a), "i"(off))
  // read k of a step's batch, in the order the next step's MFMAs (i-major) first need them:
  // B0 A0 B1 B2 B3 A1 A2 A3 (so counted lgkmcnt waits let a step start on the early fragments)
  auto rd = [&](bf16x8 (&Fa)[4], bf16x8 (&Fb)[4], uint32_t a, uint32_t b, int k) {
    switch (k) {  // immediate offsets must be literals
      case 0: X5_RD(Fb[0], b, 0); break;
      case 1: X5_RD(Fa[0], a, 0); break;
      case 2: X5_RD(Fb[1], b, 4096); break;
      case 3: X5_RD(Fb[2], b, 8192); break;
      case 4: X5_RD(Fb[3], b, 12288); break;
      case 5: X5_RD(Fa[1], a, 4096); break;
      case 6: X5_RD(Fa[2], a, 8192); break;
      default: X5_RD(Fa[3], a, 12288); break;
    }
  };

  f32x16 acc[4][4];
  bf16x8 A0[4], B0[4], A1[4], B1[4];

  // ---- the packed previous tile and its stores: lane (l32, h) of store q = 2 (4 i + j) + p
  // writes C[c_m0 + 32 i + l32][c_n0 + 32 j + 16 p + 8 h .. + 8]: per-lane offset c_vb (rows past
  // M fall past the descriptor's record count: dropped; the check covers the VGPR offset only, so
  // each 32-row block i has its own), column part as the instruction's immediate.  Inline asm: nothing hoisted, every store issued.
  u32x4 cst[X5_NPK];  // stores X5_NIM .. 31
  // packed tile's per-lane byte offsets per 32-row block; before the first tile they point past the
  // records, so the first tile's (unconditional) store slots are dropped by the hardware
  uint32_t c_vb[4] = {0x7ffff000u, 0x7ffff000u, 0x7ffff000u, 0x7ffff000u};
  const int64_t cb = (int64_t)g.M * g.ldc * 2;  // < 0x7ffffff0 (host check)
  const uint32_t c_lo = (uint32_t)(uintptr_t)g.C, c_hi = (uint32_t)((uintptr_t)g.C >> 32);
  const i32x4_t crs = {(int)c_lo, (int)(c_hi & 0xffff), (int)cb, 0x00020000};
#define X5_STV(q, v)                                                                              \
  asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen offset:%3\n\ts_nop 1"                   \
               :                                                                                   \
               : "v"(v), "v"(c_vb[(q) >> 3]), "s"(crs), "i"((((q) >> 1) & 3) * 64 + ((q) & 1) * 32) \
               : "memory")
#define X5_ST(q) X5_STV(q, cst[(q) - X5_NIM])
  // (s_nop 1 ends the store: a dwordx4 store reads its data registers a cycle late, and hipcc,
  // which does not model the asm, may overwrite them with the very next VALU instruction)

  // 16 MFMAs of one k16 step on (Fa, Fb), the 8 reads of the next step interleaved (one per two
  // MFMAs); D' = B-fragment x A-fragment: lane holds column m = l32, rows n in its 16 registers
  // DM: one DMA instruction of the k-tile begun by dma_begin after every MFMA (the library's spread
  // schedule: the 16 instructions never queue ahead of a fragment read as one burst)
  auto step = [&](auto FIRSTc, auto RDc, auto DMc, const bf16x8 (&Fa)[4], const bf16x8 (&Fb)[4], bf16x8 (&Na)[4],
                  bf16x8 (&Nb)[4], uint32_t a, uint32_t b) {
    constexpr bool FIRST = decltype(FIRSTc)::value, RD = decltype(RDc)::value, DM = decltype(DMc)::value;
    // counted waits on the previous step's batch (issued one per two MFMAs of that step, in rd()'s
    // order): MFMAs 0-3 need reads 0-4, MFMA 4 read 5, MFMA 8 read 6, MFMA 12 read 7; this step's
    // own reads (after MFMAs 1, 3, 5, ...) are younger and in the count when RD
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j == 0) {
          if (i == 0) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
          else if (i == 1) { if constexpr (RD) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory"); else asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory"); }
          else if (i == 2) { if constexpr (RD) asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory"); else asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory"); }
          else { if constexpr (RD) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory"); else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
        }
        if constexpr (FIRST) mfma32_0(acc[i][j], Fb[j], Fa[i]);
        else mfma32(acc[i][j], Fb[j], Fa[i]);
        if constexpr (RD) if (j & 1) rd(Na, Nb, a, b, 2 * i + (j >> 1));
        if constexpr (DM) dma_one(4 * i + j);
      }
  };
  constexpr int kWaitLgkm0 = 0xC07F;

  // one k-tile q.  FIRST: the tile's first k-tile (its MFMAs start the accumulators with C = 0).
  // SB >= 0: the k-tile issues the previous tile's stores SB .. SB + 3 over steps 0..2 (static
  // indices: a peeled quad of k-tiles issues 16 .. 31, after which the packed tile is dead, so it
  // is never live across the k-loop).  Step 3's reads always go out (past the stream's end they
  // re-read a stage nobody uses): no branch around MFMA code.
  auto ktile = [&](auto FIRSTc, auto SBc, auto LASTc, int q) {
    constexpr int SB = decltype(SBc)::value;
    constexpr bool LAST = decltype(LASTc)::value;  // the tile's last k-tile: step 3 reads nothing
    const int st = q & 1;
    step(FIRSTc, bc<true>{}, bc<false>{}, A0, B0, A1, B1, ra(st, 1), rb(st, 1));
    if constexpr (SB >= 0) { X5_ST(SB); X5_ST(SB + 1); }
    step(bc<false>{}, bc<true>{}, bc<false>{}, A1, B1, A0, B0, ra(st, 2), rb(st, 2));
    if constexpr (SB >= 0) X5_ST(SB + 2);
    step(bc<false>{}, bc<true>{}, bc<false>{}, A0, B0, A1, B1, ra(st, 3), rb(st, 3));
    if constexpr (SB >= 0) X5_ST(SB + 3);
    // every wave's reads of this stage are done before the barrier that frees it for the DMA
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    // boundary: k-tile q + 1 landed (the only VMEM ops after its DMA: this k-tile's stores)
    if (q + 1 < S) {
      if constexpr (SB >= 0) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    dma_begin(q + 2);  // issued spread over step 3 (past the stream: an empty descriptor)
    const int st1 = (q + 1) & 1;
    step(bc<false>{}, bc<!LAST>{}, bc<true>{}, A1, B1, A0, B0, ra(st1, 0), rb(st1, 0));
  };
  // the next k-tile's step-0 fragments, read after an epilogue (not held through the packing)
  auto rd0 = [&](int q) {
#pragma unroll
    for (int k = 0; k < 8; ++k) rd(A0, B0, ra(q & 1, 0), rb(q & 1, 0), k);
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // bias as a rank-2 update inside the MFMAs: the tile's first 16 MFMAs multiply a fragment holding
  // (hi, lo) = (bf16(b), bf16(b - hi)) in k = 0, 1 of row n by a fragment of ones: D = hi + lo = b
  // to 2^-16 relative, added in f32 before any product (no epilogue VALU).  Each wave DMAs the
  // tile's 256-float bias row into its own 1-KiB LDS slot a tile ahead (one VMEM instruction, in
  // the in-order stream: landed by the second k-tile's boundary wait), and reads its lane's four
  // values from there (inline asm: no compiler-inserted vmcnt waits).
  const uint32_t bslot = lds0 + 2 * X5_STAGE + w * 1024;
  auto load_bias = [&](int ti) {
    if constexpr (HASB) {
#if defined(__HIP_DEVICE_COMPILE__)
      if (ti < my) {
        int tm, tn;
        grouped_tile(pos + ti * G, tiles_m, tiles_n, 4, tm, tn);
        const int left = (g.N - tn * X5_BN) * 4;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(g.bias + tn * X5_BN), (short)0, left, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(smem + 2 * X5_STAGE + w * 1024), 16,
                                                 (uint32_t)(lane * 16), 0, 0, 0);
      }
#endif
    }
  };
  auto bias_mfmas = [&]() {
    typedef __attribute__((ext_vector_type(4))) unsigned int w4_t;
    float b[4];
    const uint32_t ba = bslot + (uint32_t)((128 * wn + l32) * 4);
    asm volatile("ds_read_b32 %0, %1 offset:0" : "=v"(b[0]) : "v"(ba));
    asm volatile("ds_read_b32 %0, %1 offset:128" : "=v"(b[1]) : "v"(ba));
    asm volatile("ds_read_b32 %0, %1 offset:256" : "=v"(b[2]) : "v"(ba));
    asm volatile("ds_read_b32 %0, %1 offset:384" : "=v"(b[3]) : "v"(ba));
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t one2 = h == 0 ? 0x3F803F80u : 0u;  // bf16 (1, 1)
    const bf16x8 ones = __builtin_bit_cast(bf16x8, w4_t{one2, 0u, 0u, 0u});
    bf16x8 bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float hi = bf2f(f2bf(b[j]));
      const uint32_t wv = h == 0 ? pack2<BF16>(hi, b[j] - hi) : 0u;
      bfr[j] = __builtin_bit_cast(bf16x8, w4_t{wv, 0u, 0u, 0u});
    }
    // VALU-written MFMA operands: the wait states hipcc does not insert before an asm MFMA
    asm volatile("s_nop 1" ::"v"(bfr[0]), "v"(bfr[1]), "v"(bfr[2]), "v"(bfr[3]), "v"(ones));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) mfma32_0(acc[i][j], bfr[j], ones);
  };
  if (S > 0) {
    load_bias(0);  // before both DMAs: landed once k-tile 0 has
    dma_next(0);
    if (S > 1) {
      dma_next(1);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rd0(0);
  }

  // U >= 5 (host check): the first four k-tiles of every tile carry the previous tile's stores
  int q = 0;
  for (int ti = 0; ti < my; ++ti) {
    if (ti > 0) rd0(q);
    if constexpr (HASB) {
      bias_mfmas();
      load_bias(ti + 1);
      ktile(bc<false>{}, ic<16>{}, bc<false>{}, q++);
    } else {
      ktile(bc<true>{}, ic<16>{}, bc<false>{}, q++);
    }
    ktile(bc<false>{}, ic<20>{}, bc<false>{}, q++);
    ktile(bc<false>{}, ic<24>{}, bc<false>{}, q++);
    ktile(bc<false>{}, ic<28>{}, bc<false>{}, q++);
    for (int kt = 4; kt < U - 1; ++kt) ktile(bc<false>{}, ic<-1>{}, bc<false>{}, q++);
    ktile(bc<false>{}, ic<-1>{}, bc<true>{}, q++);  // U >= 5 (host check)
    // epilogue: pack this tile (accumulators + bias -> 16-bit, lane halves swapped so each store
    // covers 16 B); row blocks 0-1 go out at once, 2-3 under the next tile's first k-tiles
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMAs' results (16-pass XDL)
    int tm, tn;
    grouped_tile(pos + ti * G, tiles_m, tiles_n, 4, tm, tn);
    const int c_m0 = tm * X5_BM + 128 * wm;
    const int c_n0 = __builtin_amdgcn_readfirstlane(tn * X5_BN + 128 * wn);
    // N % 128 == 0 (host check): a wave's 128 columns are all in range or all out
    {  // 32-bit offsets (the host checks M * ldc * 2 < 2^31); a select, not a branch
      const bool in = c_n0 < g.N;
      const uint32_t o0 = (uint32_t)(((c_m0 + l32) * (int)g.ldc + c_n0 + 8 * h) * 2);
      const uint32_t blk = (uint32_t)(32 * (int)g.ldc * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) c_vb[i] = in ? o0 + i * blk : 0x7ffff000u;
    }
    auto pack_row = [&](auto Ic) {  // fragments (i, 0..3)
      constexpr int i = decltype(Ic)::value;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t pk[4][2];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = acc[i][j][4 * gq + e];
          }
          pk[gq][0] = pack2<CDT>(v[0], v[1]);
          pk[gq][1] = pack2<CDT>(v[2], v[3]);
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          // groups 2p (vdst) and 2p+1 (src): lanes 0-31 end with columns 16p + 0..7, lanes 32-63
          // with 16p + 8..15 (T21)
          auto r0 = __builtin_amdgcn_permlane32_swap(pk[2 * p][0], pk[2 * p + 1][0], false, false);
          auto r1 = __builtin_amdgcn_permlane32_swap(pk[2 * p][1], pk[2 * p + 1][1], false, false);
          const u32x4 v = u32x4{r0[0], r1[0], r0[1], r1[1]};
          if constexpr (i < X5_NIM / 8) {
            X5_STV(2 * (4 * i + j) + p, v);  // row blocks 0, 1: straight out (L2 absorbs half a tile)
          } else {
            cst[2 * (4 * i + j) + p - X5_NIM] = v;
          }
        }
        // one fragment at a time: the accumulator reads of the next one are not hoisted (their
        // temporaries would need the registers the packed tile occupies)
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    pack_row(ic<0>{});
    pack_row(ic<1>{});
    pack_row(ic<2>{});
    pack_row(ic<3>{});
  }
  // the last tile's stores (for a block with no tile: dropped, the offsets are past the records)
#pragma unroll
  for (int k = X5_NIM; k < X5_NST; ++k) X5_ST(k);
  // every LDS-DMA (the empty ones past the stream included) lands before the block's LDS is freed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef X5_ST
#undef X5_RD
}

}  // namespace

// C[M][N] = A[M][K] B[N][K]^T (+ bias[N]) on the persistent 256x256 kernel.  bf16 operands (16-byte
// aligned rows), K % 64 == 0, K >= 320, N % 128 == 0, ldc % 8 == 0, 16-bit C (c_dt bf16 / fp16) below 2 GiB.
RK_API int rk_xgemm5(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int c_dt,
                     const float* bias, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (K < 5 * X5_BK || K % X5_BK || N % 128 || ldc % 8 || c_dt == F32 || ((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) % 16 ||
      (lda * 2) % 16 || (ldb * 2) % 16)
    return (int)hipErrorInvalidValue;
  if ((int64_t)256 * lda * 2 >= (1ll << 31) || (int64_t)256 * ldb * 2 >= (1ll << 31) ||
      ((int64_t)M + 256) * ldc * 2 >= 0x7ffff000ll)
    return (int)hipErrorInvalidValue;
  static int ncu = 0;
  if (ncu <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const int tiles = ((M + X5_BM - 1) / X5_BM) * ((N + X5_BN - 1) / X5_BN);
  X5Args g{(const uint16_t*)a, (const uint16_t*)b, c, bias, lda, ldb, ldc, M, N, K, c_dt};
  const int grid = std::min(tiles, ncu);
  if (c_dt == F16) {
    if (bias) xgemm5_kernel<F16, true><<<grid, X5_NT, 0, s>>>(g);
    else xgemm5_kernel<F16, false><<<grid, X5_NT, 0, s>>>(g);
  } else {
    if (bias) xgemm5_kernel<BF16, true><<<grid, X5_NT, 0, s>>>(g);
    else xgemm5_kernel<BF16, false><<<grid, X5_NT, 0, s>>>(g);
  }
  return (int)hipGetLastError();
}
