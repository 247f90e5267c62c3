// Persistent MFMA GEMM with the output tile drained under the next tile's main loop
// (forward layout: A [M][K], B [N][K], both K-contiguous; C = A B^T [+ bias], 16-bit C).
//
// Why this kernel: the one-wave-per-SIMD 256x256 tile (xgemm4.hip) runs its K = 768 main loop at
// ~20 us per tile but then spends ~8 us storing the tile, with every CU storing at once (32 MiB in
// one burst, HBM-write bound), plus a 2 us pipeline fill per tile and wave quantisation
// (profiles/r5_x4_trace.md).  Here (measurements: profiles/r6_vit_gemm_inmodel.md):
//
// * persistent: one block per CU (two for 128 x 128 tiles) walks its tiles pos, pos + G, ...
//   (XCD-aware remap + grouped order); the LDS-DMA unit stream runs ACROSS tiles, so the next
//   tile's first units are already landing while the current one finishes (no per-tile prologue);
// * a "unit" is a 64-deep k-slice of both operand panels, staged by LDS-DMA in WHOLE CACHE LINES:
//   each 1-KiB piece is 8 rows x 128 B (the round-6 start used 16 rows x 64 B, half lines: the
//   ablations put 27% of the loop on those loads, and 128-B pieces took it back); 16-byte chunk c
//   of image row r sits at c ^ swz8(r) (swizzle applied to the source address, the LDS image is
//   lane-linear), so every ds_read_b128 fragment read is conflict-free;
// * an NS-unit LDS ring (3 where it fits in 160 KiB with the bias rows, else 2) with counted
//   vmcnt waits and ONE barrier per unit; a unit's DMA is issued after that barrier into the stage
//   it freed, spread over the step's MFMAs;
// * MFMA shape MF: 32x32x16 (four k16 steps per unit) or 16x16x32 (two k32 steps: same FLOP per
//   cycle, the chip holds a higher clock on it); WM x WN waves of FM x FN 32 x 32 blocks each
//   (accumulators in AGPRs), fragment reads front-loaded into the other register set with
//   lgkmcnt waits counted per MFMA (X5Sched);
// * epilogue = pack only (accumulators -> 16-bit; permlane32 / permlane16 swaps so every store is
//   16 B per lane, T21).  The first half of the wave's rows is stored at once; the second half stays
//   packed and is stored over the next tile's first units, as inline-asm buffer stores
//   (out-of-range lanes point past the descriptor's record count, so every store instruction issues
//   and the vmcnt counts stay static; 160-wide tiles also mask 32-column blocks past N);
// * bias as a rank-2 update INSIDE the MFMAs: the tile's first MFMAs multiply a fragment holding
//   (hi, lo) = (bf16(b), bf16(b - hi)) at k = 0, 1 by a fragment of ones (b to 2^-16 relative, in
//   f32 before any product; no epilogue work and no per-column loads there);
// * tile shape per problem (host): 256 x 256, 128 x 256, 256 x 128, 128 x 128 or 256 x 160 (ViT's
//   N = 768 in five column tiles: 495 tiles on 256 CUs instead of 297), by CU rounds, or a
//   two-launch row split (full rounds of 256 x 256 tiles, the remaining rows on a smaller tile).
//
// Per unit q (stage q % NS):
//   steps 0 .. NSTEP-2 : MFMAs on one fragment set || the next step's reads into the other set ||
//                        the remaining DMA groups of unit q + 1 (32x32x16 only)
//   boundary           : lgkmcnt(0) (this stage fully read); vmcnt = unit q + 1 landed; ONE barrier
//   last step          : MFMAs || reads of unit q + 1's first step || DMA group 0 of unit q + NS into
//                        this unit's stage || the previous tile's pending stores
// vmcnt counts rely on vector-memory ops completing in issue order (DMA loads and stores alike).
#include "mgemm_core.h"

#include <type_traits>

using namespace rk;

namespace {

constexpr int X5_BK = 64;     // a "unit": 64-deep k-slice, four k16 steps
constexpr int X5_ROWB = X5_BK * 2;  // 128-byte image rows: every DMA piece reads whole cache lines
#ifndef X5_DS
#define X5_DS 2  // steps carrying a unit's DMA: the previous unit's last step + this many - 1 of its own
#endif
// 16-byte chunk c of image row r sits at slot c ^ swz8(r): a ds_read_b128 lane group (16 rows
// distinct mod 16, one chunk) then covers all 16 slots of the 256-byte bank row (conflict-free)
__device__ __forceinline__ int swz8(int r) { return (r >> 1) & 7; }

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
__device__ __forceinline__ void mfma32(f32x4& c, const bf16x8& a, const bf16x8& b) {  // 16x16x32
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma32_0(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}
// f(ic<0>{}), f(ic<1>{}), ... f(ic<N-1>{}): compile-time indices for unrolled bodies
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
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

// Compile-time schedule of one k16 step of an FM x FN wave tile (Q = FM FN MFMAs, i-major; R =
// FM + FN fragment reads for the next step, in the order B0 A0 B1 .. B(FN-1) A1 .. A(FM-1)).
template <int FM, int FN>
struct X5Sched {
  static constexpr int Q = FM * FN, R = FM + FN;
  // read index of the fragment an MFMA needs
  static constexpr int rb(int j) { return j == 0 ? 0 : j + 1; }
  static constexpr int ra(int i) { return i == 0 ? 1 : FN + i; }
  // the MFMA after which read k goes out: front-loaded, one read per MFMA (the reads land in the
  // other fragment set, free since the previous step; the batch is complete long before the unit's
  // lgkmcnt(0) + barrier, so the MFMA pipe does not drain there)
  static constexpr int after(int k) { return k; }
  // which read (or -1) goes out right after MFMA m
  static constexpr int read_after(int m) {
    for (int k = 0; k < R; ++k)
      if (after(k) == m) return k;
    return -1;
  }
  // reads of the previous batch MFMA m and all before it need
  static constexpr int need(int m) {
    int n = 0;
    for (int x = 0; x <= m; ++x) {
      const int i = x / FN, j = x % FN;
      const int v = ra(i) > rb(j) ? ra(i) : rb(j);
      n = v > n ? v : n;
    }
    return n;
  }
  // lgkmcnt before MFMA m (-1: no wait needed there): the previous batch's reads younger than
  // need(m) may be outstanding, plus this step's own reads issued before m (when it reads)
  static constexpr int wait_before(int m, bool rd) {
    if (m > 0 && need(m) == need(m - 1)) return -1;
    int fresh = 0;
    if (rd)
      for (int k = 0; k < R; ++k)
        if (after(k) < m) ++fresh;
    const int w = (R - 1 - need(m)) + fresh;
    return w > 15 ? 15 : w;  // lgkmcnt is 4 bits: waiting for more than needed stays correct
  }
};

struct X5Args {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const float* bias;
  int64_t lda, ldb, ldc;
  int M, N, K, c_dt;
};

// 128x128 tiles (68 KiB of LDS) run two blocks per CU: one block's DMA issue and fill/drain
// overlap the other's MFMAs
template <int FM, int FN, int WM, int WN>
constexpr int x5_blocks_per_cu() { return FM * FN * WM * WN <= 16 ? 2 : 1; }

// MF: the MFMA shape, 32 (v_mfma_f32_32x32x16_bf16, four k16 steps per unit) or 16
// (v_mfma_f32_16x16x32_bf16, two k32 steps per unit; the same FLOP per cycle, and the chip holds a
// higher clock on it).  FM x FN count 32 x 32 blocks either way (a 32-block = 2 x 2 16-blocks).
template <int CDT, bool HASB, int FM, int FN, int WM, int WN, int MF = 32>
__global__ void __launch_bounds__(64 * WM * WN, (x5_blocks_per_cu<FM, FN, WM, WN>())) xgemm5_kernel(X5Args g) {
  static_assert(MF == 32 || MF == 16, "MFMA shape");
  constexpr int SUB = MF == 16 ? 2 : 1;        // MFMA blocks per 32-row (column) block
  constexpr int AM = FM * SUB, AN = FN * SUB;  // MFMA blocks per wave
  constexpr int NSTEP = MF == 16 ? 2 : 4;      // MFMA k-steps per 64-deep unit
  constexpr int NCV = MF == 16 ? 2 * FM : FM;  // per-lane store row offsets
  using accT = std::conditional_t<MF == 16, f32x4, f32x16>;
  constexpr int NW = WM * WN;                               // waves: WM x WN, each FM x FN fragments
  constexpr int BM = 32 * FM * WM, BN = 32 * FN * WN;      // block tile
  constexpr int OPA = BM * X5_ROWB, OPB = BN * X5_ROWB;  // operand images per stage
  constexpr int STAGE = OPA + OPB;
  constexpr int FR = MF * X5_ROWB;                        // one MF-row fragment block of an image
  constexpr int NIA = BM / (8 * NW), NIB = BN / (8 * NW);  // DMA pieces (8 rows x 128 B) per wave per operand
  static_assert(NIA * 8 * NW == BM && NIB * 8 * NW == BN, "a unit's images split evenly over the waves");
  constexpr int NDMA = NIA + NIB;
  constexpr int DS = MF == 16 ? 1 : X5_DS;  // (two steps per unit: all of it after the barrier)
  static_assert(DS >= 1 && DS <= NSTEP - 1, "a unit's DMA must leave a step to land in");
  constexpr int NST = 2 * FM * FN;                    // 16-byte stores per wave per tile
  constexpr int NIM = NST / 2;                        // issued at the epilogue (rows i < FM / 2)
  constexpr int NPK = NST - NIM;                      // kept packed, issued in the next tile's first NSU units
  constexpr int NSU = NPK % 4 == 0 ? 4 : 5;           // (U >= NSU + 1: host check)
  constexpr int SPK = NPK / NSU;                      // per unit of those
  static_assert(SPK * NSU == NPK, "stores split over four or five units");
  using SC = X5Sched<AM, AN>;
  // NS-stage ring + one 1-KiB bias row per wave (one __shared__ object: see the guide's trap 4(a))
  // LDS ring of NS units: 3 where they fit beside the bias rows (a third unit in flight hides the
  // HBM latency of operands that are not cache-resident, e.g. ViT's fc2 input), else 2
  constexpr int NS = (x5_blocks_per_cu<FM, FN, WM, WN>() == 1 && 3 * STAGE + NW * 1024 <= 163840) ? 3 : 2;
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE + NW * 1024];
  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const int total = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int pos = xcd_remap(blockIdx.x, G);
  const int my = pos < total ? (total - pos + G - 1) / G : 0;
  const int U = g.K / X5_BK;
  const int S = my * U;  // units in this block's stream
  const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WN, wn = w % WN;

  // ---- DMA: lane l of a 1-KiB piece (8 rows x 128 B) lands at image row l/8, slot l%8, i.e. holds
  // source chunk (l%8) ^ swz8(row).  Pieces start at 8-row boundaries: swz8 of the row depends on the
  // lane and on the piece's parity (row0 % 16 = 0 or 8; every wave's first piece is at a multiple
  // of 16 rows): two per-lane offsets per operand
  const int drow = lane >> 3;
  const uint32_t c0 = (uint32_t)(((lane & 7) ^ swz8(drow)) * 16), c8 = (uint32_t)(((lane & 7) ^ swz8(drow + 8)) * 16);
  const uint32_t va0 = (uint32_t)(drow * g.lda * 2) + c0, va8 = (uint32_t)(drow * g.lda * 2) + c8;
  const uint32_t vb0 = (uint32_t)(drow * g.ldb * 2) + c0, vb8 = (uint32_t)(drow * g.ldb * 2) + c8;
  // issue cursor: tile of the next DMA and its unit
  int iss_i = 0, iss_k = 0;
  const char *ia = nullptr, *ib = nullptr;
  int ia_n = 0, ib_n = 0;  // bytes from the tile's first row to the operand's end (clamped to 2^31 - 1)
  auto iss_tile = [&](int i) {
    int tm, tn;
    grouped_tile(pos + i * G, tiles_m, tiles_n, 4, tm, tn);
    ia = (const char*)g.A + (int64_t)tm * BM * g.lda * 2;
    ib = (const char*)g.B + (int64_t)tn * BN * g.ldb * 2;
    const int64_t an = ((int64_t)g.M - tm * BM) * g.lda * 2, bn = ((int64_t)g.N - tn * BN) * g.ldb * 2;
    ia_n = (int)(an > 0x7fffffff ? 0x7fffffff : an);
    ib_n = (int)(bn > 0x7fffffff ? 0x7fffffff : bn);
  };
  if (my > 0) iss_tile(0);
  // one descriptor per operand and unit (rows past M / N read as zeros: the VGPR offset is
  // range-checked).  dma_begin(q) forms them for unit q (a unit past the stream gets an empty
  // descriptor: its instructions still issue, so every vmcnt count stays static, and only write
  // zeros into a stage nobody reads any more); dma_one(k) issues piece k (A first, then B), its
  // row offset added at the instruction to an opaque copy of the lane part (no hoisted sums).
  // (the descriptors are formed at each instruction from plain scalars: rsrc-typed variables
  // carried across the tile-advance branch became a per-thread alloca that hipcc moved into LDS)
  const char *d_pa = (const char*)g.A, *d_pb = (const char*)g.B;
  int d_na = 0, d_nb = 0;
  char* d_st = smem;
  auto dma_begin = [&](int q) {
#if defined(__HIP_DEVICE_COMPILE__)
    const bool real = q < S;
    d_st = smem + (q % NS) * STAGE;
    const int koff = iss_k * X5_ROWB;
    const char* pa = real ? ia + koff : (const char*)g.A;
    const char* pb = real ? ib + koff : (const char*)g.B;
    const int na = real ? max(ia_n - koff, 0) : 0, nb = real ? max(ib_n - koff, 0) : 0;
    d_pa = pa;
    d_pb = pb;
    d_na = na;
    d_nb = nb;
    if (real && ++iss_k == U) {
      iss_k = 0;
      if (++iss_i < my) iss_tile(iss_i);
    }
#endif
  };
  auto dma_one = [&](int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    const bool opb = k >= NIA;
    const int i = opb ? k - NIA : k;
    const int row0 = (opb ? 8 * NIB : 8 * NIA) * w + 8 * i;  // wave w stages 1/NW of each image
    // (branches on the compile-time operand, not a ?: of captured lvalues: a select of two
    // variables' addresses keeps them in memory, and hipcc moved that memory into LDS)
    uint32_t vo;
    const char* pp;
    int nn;
    int64_t ld;
    // parity of the piece's first 8-row group (wave-uniform; compile-time for even NIA / NIB)
    const bool par = (((opb ? NIB : NIA) * w + i) & 1) != 0;
    if (opb) {
      vo = par ? vb8 : vb0;
      pp = d_pb;
      nn = d_nb;
      ld = g.ldb;
    } else {
      vo = par ? va8 : va0;
      pp = d_pa;
      nn = d_na;
      ld = g.lda;
    }
    asm volatile("" : "+v"(vo));
    vo += (uint32_t)(row0 * ld * 2);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(pp), (short)0, nn, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(d_st + (opb ? OPA : 0) + row0 * X5_ROWB),
                                             16, vo, 0, 0, 0);
#endif
  };
  // DMA group gi of a unit (DS groups): pieces [gi NDMA / DS, (gi + 1) NDMA / DS)
  auto dma_group = [&](auto Gc) {
    constexpr int gi = decltype(Gc)::value;
#pragma unroll
    for (int k = gi * NDMA / DS; k < (gi + 1) * NDMA / DS; ++k) dma_one(k);
  };

  // ---- fragment reads: 32x32x16 operand of rows r0 .. r0+31 at k16 step s (0..3) of a unit: lane
  // reads row r0 + l32, chunk 2s + h at slot chunk ^ swz8(row); fragment i = +i * FR (32 rows: the
  // swizzle of row r0 + l32 is that of l32)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const lds_void*)smem;
  // (16x16x32: lane reads row r0 + lane % 16, chunk 4 s + lane / 16 — a lane group's 16 rows are
  // still distinct mod 16: conflict-free under the same swizzle)
  const int frow = MF == 16 ? (lane & 15) : l32;
  const int fsw = swz8(frow);
  // per-lane part of step s's address (A image, stage 0); B and the other stage differ by
  // wave-uniform amounts added per step
  uint32_t la[NSTEP];
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int ch = MF == 16 ? 4 * s + (lane >> 4) : 2 * s + h;
    la[s] = lds0 + wm * 32 * FM * X5_ROWB + (uint32_t)(frow * X5_ROWB + ((ch ^ fsw) * 16));
  }
  const uint32_t bdelta = (uint32_t)(OPA + (wn * 32 * FN - wm * 32 * FM) * X5_ROWB);
  // (the base goes through an empty asm so the sums are formed at each use, not hoisted out of
  // the loop into live registers)
  auto ra = [&](int st, int s) {
    uint32_t v = la[s];
    asm volatile("" : "+v"(v));
    return v + (uint32_t)(st * STAGE);
  };
  auto rb = [&](int st, int s) {
    uint32_t v = la[s];
    asm volatile("" : "+v"(v));
    return v + (uint32_t)(st * STAGE) + bdelta;
  };
#define X5_RD(dst, a, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(a), "i"(off))
  // read k of a step's batch: B0 A0 B1 .. B(FN-1) A1 .. A(FM-1) (X5Sched)
  auto rd = [&](bf16x8 (&Fa)[AM], bf16x8 (&Fb)[AN], uint32_t a, uint32_t b, auto Kc) {
    constexpr int k = decltype(Kc)::value;
    if constexpr (k == 0) X5_RD(Fb[0], b, 0);
    else if constexpr (k == 1) X5_RD(Fa[0], a, 0);
    else if constexpr (k <= AN) X5_RD(Fb[k - 1], b, (k - 1) * FR);
    else X5_RD(Fa[k - AN], a, (k - AN) * FR);
  };

  accT acc[AM][AN];
  bf16x8 A0[AM], B0[AN], A1[AM], B1[AN];

  // ---- the packed previous tile and its stores: lane (l32, h) of store q = 2 (FN i + j) + p
  // writes C[c_m0 + 32 i + l32][c_n0 + 32 j + 16 p + 8 h .. + 8]: per-lane offset c_vb[i] (rows past
  // M fall past the descriptor's record count: dropped; the check covers the VGPR offset only, so
  // each 32-row block has its own), column part as the instruction's immediate.
  u32x4 cst[NPK];  // stores NIM .. NST - 1
  // before the first tile the offsets point past the records, so the first tile's (unconditional)
  // store slots are dropped by the hardware
  // (16x16 blocks: store q = 2 (FN i + j) + i2 writes rows 32 i + 16 i2 + lane % 16; lane group
  // g = lane / 16 holds columns 32 j + 16 (g & 1) + 8 (g >> 1) .. + 8 after the permlane16 swap)
  uint32_t c_vb[NCV];
#pragma unroll
  for (int i = 0; i < NCV; ++i) c_vb[i] = 0x7ffff000u;
  const int64_t cb = (int64_t)g.M * g.ldc * 2;  // < 2^31 (host check)
  const uint32_t c_lo = (uint32_t)(uintptr_t)g.C, c_hi = (uint32_t)((uintptr_t)g.C >> 32);
  const i32x4_t crs = {(int)c_lo, (int)(c_hi & 0xffff), (int)cb, 0x00020000};
  // (s_nop 1 ends each store: a dwordx4 store reads its data registers a cycle late, and hipcc,
  // which does not model the asm, may overwrite them with the very next VALU instruction)
  // (tiles narrower than a multiple of 128 columns, e.g. 160, can end past N: a 32-column block
  // whose first column is at or past N gets the dropped offset; c_nl = N - the wave's first column)
  int c_nl = 0;
  auto st_off = [&](int q) -> uint32_t {
    const uint32_t o = MF == 16 ? c_vb[(q / (2 * FN)) * 2 + (q & 1)] : c_vb[q / (2 * FN)];
    if constexpr (BN % 128 == 0) return o;
    else return 32 * ((q >> 1) % FN) < c_nl ? o : 0x7ffff000u;
  };
#define X5_STV(q, v)                                                                              \
  asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen offset:%3\n\ts_nop 1"                   \
               :                                                                                   \
               : "v"(v), "v"(st_off(q)), "s"(crs), "i"((((q) >> 1) % FN) * 64 + (MF == 16 ? 0 : ((q) & 1) * 32)) \
               : "memory")
#define X5_ST(q) X5_STV(q, cst[(q) - NIM])

  // Q MFMAs of one k16 step on (Fa, Fb) with the counted waits on the previous batch, the reads of
  // the next step (RD) and DMA group DG (-1: none) interleaved
  auto step = [&](auto FIRSTc, auto RDc, auto DGc, const bf16x8 (&Fa)[AM], const bf16x8 (&Fb)[AN],
                  bf16x8 (&Na)[AM], bf16x8 (&Nb)[AN], uint32_t a, uint32_t b) {
    constexpr bool FIRST = decltype(FIRSTc)::value, RD = decltype(RDc)::value;
    constexpr int DG = decltype(DGc)::value;
    auto one = [&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      constexpr int i = m / AN, j = m % AN;
      constexpr int wt = SC::wait_before(m, RD);
      if constexpr (wt >= 0) wait_lgkm<wt>();
      if constexpr (FIRST) mfma32_0(acc[i][j], Fb[j], Fa[i]);
      else mfma32(acc[i][j], Fb[j], Fa[i]);
      if constexpr (RD && SC::read_after(m) >= 0) rd(Na, Nb, a, b, ic<SC::read_after(m)>{});
      if constexpr (DG >= 0) {  // the group's pieces d with d * Q / NG == m
        constexpr int k0 = DG * NDMA / DS, NG = (DG + 1) * NDMA / DS - k0;
#pragma unroll
        for (int d = 0; d < NG; ++d)
          if (d * SC::Q / NG == m) dma_one(k0 + d);
      }
    };
    sfor<SC::Q>(one);
  };
  constexpr int kWaitLgkm0 = 0xC07F;

  // one unit q (four k16 steps).  FIRST: the tile's first unit (its MFMAs start the accumulators with
  // C = 0).  SB >= 0: the unit issues the previous tile's stores SB .. SB + SPK - 1 (static indices: a
  // peeled quad of units issues them all, after which the packed tile is dead, so it is never live
  // across the k-loop).  LAST: the tile's last unit, whose step 3 reads nothing.
  //   steps 0-2: MFMAs || reads of the next step (this stage) || DMA groups 1 .. DS-1 of unit q + 1
  //   lgkmcnt(0) (this stage fully read) + vmcnt(0) (unit q + 1 landed: nothing younger is a DMA)
  //   + ONE barrier
  //   step 3   : MFMAs || reads of step 0 of unit q + 1 || DMA group 0 of unit q + NS into this
  //              unit's stage (freed by the barrier) || the previous tile's stores
  auto unit = [&](auto FIRSTc, auto SBc, auto LASTc, int q) {
    constexpr int SB = decltype(SBc)::value;
    constexpr bool LAST = decltype(LASTc)::value;
    const int st = q % NS;
    if constexpr (NSTEP == 4) {
      step(FIRSTc, bc<true>{}, ic<(DS > 1 ? 1 : -1)>{}, A0, B0, A1, B1, ra(st, 1), rb(st, 1));
      step(bc<false>{}, bc<true>{}, ic<(DS > 2 ? 2 : -1)>{}, A1, B1, A0, B0, ra(st, 2), rb(st, 2));
      step(bc<false>{}, bc<true>{}, ic<-1>{}, A0, B0, A1, B1, ra(st, 3), rb(st, 3));
    } else {
      step(FIRSTc, bc<true>{}, ic<-1>{}, A0, B0, A1, B1, ra(st, 1), rb(st, 1));
    }
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    // unit q + 1 landed: the only DMA younger than it is unit q + 2's (NS = 3)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NS - 2) * NDMA) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    dma_begin(q + NS);  // past the stream: an empty descriptor
    if constexpr (SB >= 0) {
#pragma unroll
      for (int k = 0; k < SPK; ++k) X5_ST(SB + k);
    }
    const int st1 = (q + 1) % NS;
    step(bc<false>{}, bc<!LAST>{}, ic<0>{}, A1, B1, A0, B0, ra(st1, 0), rb(st1, 0));
  };
  // the next k-tile's step-0 fragments, read after an epilogue (not held through the packing)
  auto rd0 = [&](int q) {
    const uint32_t a = ra(q % NS, 0), b = rb(q % NS, 0);
    sfor<SC::R>([&](auto Kc) { rd(A0, B0, a, b, Kc); });
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // bias: each wave DMAs the tile's bias row (up to 256 floats) into its own 1-KiB LDS slot a tile
  // ahead (one VMEM instruction in the in-order stream: landed by the second k-tile's boundary
  // wait) and reads its lane's FN values from there (inline asm: no compiler-inserted vmcnt waits)
  const uint32_t bslot = lds0 + NS * STAGE + w * 1024;
  auto load_bias = [&](int ti) {
    if constexpr (HASB) {
#if defined(__HIP_DEVICE_COMPILE__)
      if (ti < my) {
        int tm, tn;
        grouped_tile(pos + ti * G, tiles_m, tiles_n, 4, tm, tn);
        const int left = (g.N - tn * BN) * 4;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(g.bias + tn * BN), (short)0, left, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(smem + NS * STAGE + w * 1024), 16,
                                                 (uint32_t)(lane * 16), 0, 0, 0);
      }
#endif
    }
  };
  auto bias_mfmas = [&]() {
    typedef __attribute__((ext_vector_type(4))) unsigned int w4_t;
    float b[AN];  // column wn 32 FN + MF j + lane % MF of the tile
    const uint32_t ba = bslot + (uint32_t)((wn * 32 * FN + (lane & (MF - 1))) * 4);
    static_assert(AN >= 2 && AN <= 10, "bias reads");
#define X5_BR(j) \
  if constexpr ((j) < AN) asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(b[(j) % AN]) : "v"(ba), "i"((j) * MF * 4))
    X5_BR(0); X5_BR(1); X5_BR(2); X5_BR(3); X5_BR(4); X5_BR(5); X5_BR(6); X5_BR(7); X5_BR(8); X5_BR(9);
#undef X5_BR
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    // the lanes holding k = 0 .. 7 of the operands: lanes 0-31 (32x32x16), 0-15 (16x16x32)
    const bool k0 = MF == 16 ? lane < 16 : h == 0;
    const uint32_t one2 = k0 ? 0x3F803F80u : 0u;  // bf16 (1, 1)
    const bf16x8 ones = __builtin_bit_cast(bf16x8, w4_t{one2, 0u, 0u, 0u});
    bf16x8 bfr[AN];
#pragma unroll
    for (int j = 0; j < AN; ++j) {
      const float hi = bf2f(f2bf(b[j]));
      const uint32_t wv = k0 ? pack2<BF16>(hi, b[j] - hi) : 0u;
      bfr[j] = __builtin_bit_cast(bf16x8, w4_t{wv, 0u, 0u, 0u});
    }
    // VALU-written MFMA operands: the wait states hipcc does not insert before an asm MFMA
    asm volatile("s_nop 1" ::"v"(bfr[0]), "v"(bfr[AN - 1]), "v"(ones));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
      for (int j = 0; j < AN; ++j) mfma32_0(acc[i][j], bfr[j], ones);
  };

  if (S > 0) {
    load_bias(0);  // before the DMAs: landed once unit 0 has
    for (int u = 0; u < NS - 1; ++u) {
      dma_begin(u);
#pragma unroll
      for (int k = 0; k < NDMA; ++k) dma_one(k);
    }
    dma_begin(NS - 1);  // its group 0 now (steady state: issued in unit 0's predecessor's last step)
    dma_group(ic<0>{});
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NS - 2) * NDMA + NDMA / DS) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rd0(0);
  }

  // U >= NSU + 1 (host check): the first NSU units of every tile carry the previous tile's stores
  int q = 0;
  for (int ti = 0; ti < my; ++ti) {
    if (ti > 0) rd0(q);
    if constexpr (HASB) {
      bias_mfmas();
      load_bias(ti + 1);
      unit(bc<false>{}, ic<NIM>{}, bc<false>{}, q++);
    } else {
      unit(bc<true>{}, ic<NIM>{}, bc<false>{}, q++);
    }
    unit(bc<false>{}, ic<NIM + SPK>{}, bc<false>{}, q++);
    unit(bc<false>{}, ic<NIM + 2 * SPK>{}, bc<false>{}, q++);
    unit(bc<false>{}, ic<NIM + 3 * SPK>{}, bc<false>{}, q++);
    if constexpr (NSU == 5) unit(bc<false>{}, ic<NIM + 4 * SPK>{}, bc<false>{}, q++);
    for (int kt = NSU; kt < U - 1; ++kt) unit(bc<false>{}, ic<-1>{}, bc<false>{}, q++);
    unit(bc<false>{}, ic<-1>{}, bc<true>{}, q++);
    // epilogue: pack this tile (accumulators -> 16-bit, lane halves swapped so each store covers
    // 16 B); the first half of the rows goes out at once, the rest under the next tile's quad
    // the last MFMAs' results (16-pass XDL) before any accumulator read.  The sched_barrier keeps
    // hipcc from hoisting an accumulator read above the nops (or above the last MFMAs, which it
    // does not know write late: fragment (0, 0), done 7 MFMAs early, was read too soon otherwise)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    int tm, tn;
    grouped_tile(pos + ti * G, tiles_m, tiles_n, 4, tm, tn);
    const int c_m0 = tm * BM + 32 * FM * wm;
    const int c_n0 = __builtin_amdgcn_readfirstlane(tn * BN + 32 * FN * wn);
    {  // 32-bit offsets (the host checks (M + BM) * ldc * 2 < 2^31); a select, not a branch
      const bool in = c_n0 < g.N;
      if constexpr (MF == 16) {
        const int gq = lane >> 4;
        const uint32_t o0 =
            (uint32_t)(((c_m0 + (lane & 15)) * (int)g.ldc + c_n0 + 16 * (gq & 1) + 8 * (gq >> 1)) * 2);
        const uint32_t blk = (uint32_t)(16 * (int)g.ldc * 2);
#pragma unroll
        for (int i = 0; i < NCV; ++i) c_vb[i] = in ? o0 + i * blk : 0x7ffff000u;
      } else {
        const uint32_t o0 = (uint32_t)(((c_m0 + l32) * (int)g.ldc + c_n0 + 8 * h) * 2);
        const uint32_t blk = (uint32_t)(32 * (int)g.ldc * 2);
#pragma unroll
        for (int i = 0; i < FM; ++i) c_vb[i] = in ? o0 + i * blk : 0x7ffff000u;
      }
      c_nl = g.N - c_n0;
    }
    // store q = 2 (FN i + j) + p of the 16-byte vector v: straight out (first half of the rows,
    // L2 absorbs it) or kept packed for the next tile's first units
    auto put = [&](auto Qc, const u32x4& v) {
      constexpr int qq = decltype(Qc)::value;
      if constexpr (qq < NIM) X5_STV(qq, v);
      else cst[qq - NIM] = v;
    };
    auto pack_row = [&](auto Ic) {  // 32-row block i, fragments (i, 0 .. FN-1)
      constexpr int i = decltype(Ic)::value;
      sfor<FN>([&](auto Jc) {
        constexpr int j = decltype(Jc)::value;
        if constexpr (MF == 32) {
          uint32_t pk[4][2];
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            pk[gq][0] = pack2<CDT>(acc[i][j][4 * gq], acc[i][j][4 * gq + 1]);
            pk[gq][1] = pack2<CDT>(acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]);
          }
          sfor<2>([&](auto Pc) {
            constexpr int p = decltype(Pc)::value;
            // groups 2p (vdst) and 2p+1 (src): lanes 0-31 end with columns 16p + 0..7, lanes 32-63
            // with 16p + 8..15 (T21)
            auto r0 = __builtin_amdgcn_permlane32_swap(pk[2 * p][0], pk[2 * p + 1][0], false, false);
            auto r1 = __builtin_amdgcn_permlane32_swap(pk[2 * p][1], pk[2 * p + 1][1], false, false);
            put(ic<2 * (FN * i + j) + p>{}, u32x4{r0[0], r1[0], r0[1], r1[1]});
          });
        } else {
          sfor<2>([&](auto I2c) {
            constexpr int i2 = decltype(I2c)::value;
            // 16-blocks X = (2i + i2, 2j) and Y = (.., 2j + 1): lane group g holds columns 4g .. 4g+3
            // of each; the permlane16 swap (odd groups' vdst <-> even groups' src) leaves X's 0..7
            // in group 0, Y's 0..7 in group 1, X's 8..15 in group 2, Y's 8..15 in group 3
            const accT& X = acc[2 * i + i2][2 * j];
            const accT& Y = acc[2 * i + i2][2 * j + 1];
            auto r0 = __builtin_amdgcn_permlane16_swap(pack2<CDT>(X[0], X[1]), pack2<CDT>(Y[0], Y[1]), false, false);
            auto r1 = __builtin_amdgcn_permlane16_swap(pack2<CDT>(X[2], X[3]), pack2<CDT>(Y[2], Y[3]), false, false);
            put(ic<2 * (FN * i + j) + i2>{}, u32x4{r0[0], r1[0], r0[1], r1[1]});
          });
        }
        // one fragment at a time: the accumulator reads of the next one are not hoisted (their
        // temporaries would need the registers the packed tile occupies)
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    sfor<FM>(pack_row);
  }
  // the last tile's stores (for a block with no tile: dropped, the offsets are past the records)
#pragma unroll
  for (int k = NIM; k < NST; ++k) X5_ST(k);
  // every LDS-DMA (the empty ones past the stream included) lands before the block's LDS is freed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef X5_ST
#undef X5_STV
#undef X5_RD
}

template <int CDT, bool HASB>
int x5_launch(int shape, int grid, const X5Args& g, hipStream_t s) {
  switch (shape) {
    case 1: xgemm5_kernel<CDT, HASB, 4, 4, 2, 2><<<grid, 256, 0, s>>>(g); break;
    case 2: xgemm5_kernel<CDT, HASB, 2, 4, 2, 2><<<grid, 256, 0, s>>>(g); break;
    case 3: xgemm5_kernel<CDT, HASB, 4, 2, 2, 2><<<grid, 256, 0, s>>>(g); break;
    case 4: xgemm5_kernel<CDT, HASB, 4, 2, 2, 4><<<grid, 512, 0, s>>>(g); break;
    case 5: xgemm5_kernel<CDT, HASB, 2, 2, 2, 4><<<grid, 512, 0, s>>>(g); break;
    case 6: xgemm5_kernel<CDT, HASB, 2, 2, 4, 2><<<grid, 512, 0, s>>>(g); break;
    case 7: xgemm5_kernel<CDT, HASB, 2, 2, 2, 2><<<grid, 256, 0, s>>>(g); break;
    case 8: xgemm5_kernel<CDT, HASB, 2, 5, 4, 1><<<grid, 256, 0, s>>>(g); break;
    case 9: xgemm5_kernel<CDT, HASB, 4, 4, 2, 2, 16><<<grid, 256, 0, s>>>(g); break;
    case 10: xgemm5_kernel<CDT, HASB, 2, 5, 4, 1, 16><<<grid, 256, 0, s>>>(g); break;
    case 11: xgemm5_kernel<CDT, HASB, 2, 4, 2, 2, 16><<<grid, 256, 0, s>>>(g); break;
    case 12: xgemm5_kernel<CDT, HASB, 4, 2, 2, 2, 16><<<grid, 256, 0, s>>>(g); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// tile shapes: 1 / 2 / 3 = 256x256 / 128x256 / 256x128 on 4 waves (one per SIMD), 4 / 5 / 6 the same
// tiles on 8 waves (two per SIMD), 7 = 128x128 on 4 waves, 8 = 256x160 on 4 waves (4 x 1, 64 x 160 per
// wave: N = 768 in 5 column tiles, 495 tiles on 256 CUs = two nearly full rounds)
int g_x5_shape = 0;   // diagnostics: force a tile shape (0 automatic)
int g_x5_split = 0;   // diagnostics: force the row split with this tail shape (0 automatic)
// automatic choice: family f's shapes {256x256, 128x256, 256x128, 256x160}
constexpr int kX5Fam[3][4] = {{1, 2, 3, 8}, {4, 5, 6, 8}, {9, 11, 12, 10}};
int g_x5_family = 2;

void x5_dims(int shape, int& bm, int& bn) {
  bm = (shape == 2 || shape == 5 || shape == 7 || shape == 11) ? 128 : 256;
  bn = (shape == 8 || shape == 10) ? 160 : (shape == 3 || shape == 6 || shape == 7 || shape == 12) ? 128 : 256;
}

}  // namespace

// Diagnostics: force the tile shape of later rk_xgemm5 calls (0 = automatic; 1..7, see g_x5_shape);
// 16 + f: the automatic choice uses family f (0: 4-wave 32x32x16 tiles, 1: 8-wave, 2: 4-wave
// 16x16x32); 32 + t: force the row split with tail shape t (32: automatic).
RK_API int rk_xgemm5_set_shape(int s) {
  if (s >= 32) g_x5_split = s - 32;
  else if (s >= 16) g_x5_family = (s - 16) % 3;
  else g_x5_shape = s;
  return 0;
}

// C[M][N] = A[M][K] B[N][K]^T (+ bias[N]) on the persistent kernel.  bf16 operands (16-byte aligned
// rows), K % 64 == 0, K >= 320, N % 128 == 0, ldc % 8 == 0, 16-bit C (c_dt bf16 / fp16), (M + 256)
// ldc * 2 < 2^31.  Tile shape: 256 x 256 unless a 128-deep one leaves fewer CU rounds (per the
// round time of its half-size tiles).
RK_API int rk_xgemm5(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int c_dt,
                     const float* bias, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (K < 320 || K % 64 || N % 128 || ldc % 8 || c_dt == F32 || ((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) % 16 ||
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
  // CU rounds x tile area, smaller tiles priced higher per element (their per-wave tiles read more
  // per MFMA): the single-launch cost of a shape over `rows` rows
  auto price = [](int bm, int bn) {
    return bm * bn == 65536 ? 1.0 : bm * bn == 40960 ? 1.08 : bm * bn == 32768 ? 1.15 : 1.4;
  };
  auto cost = [&](int shape, int rows) {
    int bm, bn;
    x5_dims(shape, bm, bn);
    const int t = ((rows + bm - 1) / bm) * ((N + bn - 1) / bn), slots = shape == 7 ? 2 * ncu : ncu;
    return ((t + slots - 1) / slots) * (double)bm * bn / 65536.0 * price(bm, bn) * (shape == 7 ? 2.0 : 1.0);
  };
  // Plan: one launch, or (when the 256x256 tiles leave the last CU round part-empty, e.g. ViT's
  // N = 768 products: 297 tiles on 256 CUs) the rows of the full rounds on 256x256 tiles and the
  // remaining rows on a smaller tile as a second launch.
  int s1 = (g_x5_shape == 8 || g_x5_shape == 10) && K < 384 ? 1 : g_x5_shape, s2 = 0, rows1 = M;
  if (s1 == 0) {
    const int* fam = kX5Fam[g_x5_family];
    s1 = fam[0];
    double best = cost(s1, M);
    for (int t = 1; t <= 2; ++t)
      if (cost(fam[t], M) < best - 1e-9) { best = cost(fam[t], M); s1 = fam[t]; }
    if (K >= 384 && cost(fam[3], M) < best - 1e-9) { best = cost(fam[3], M); s1 = fam[3]; }  // 256x160: U >= 6
    const int tn = (N + 255) / 256, full = ((M + 255) / 256) * tn;
    int r = full / ncu, r1 = (r * ncu / tn) * 256;
    if (g_x5_split > 0 && r1 <= 0) r1 = (M / 2) / 256 * 256;  // diagnostics on small problems
    if (r1 > 0 && r1 < M) {
      const int cand[4] = {fam[1], fam[2], 7, 0};
      for (int ci = 0; cand[ci]; ++ci) {
        const int t = g_x5_split > 0 ? g_x5_split : cand[ci];
        const double c = (double)(((r1 / 256) * tn + ncu - 1) / ncu) + cost(t, M - r1) + 0.2;  // a launch's fill + drain
        if (g_x5_split > 0 || c < best - 1e-9) { best = c; s1 = fam[0]; s2 = t; rows1 = r1; }
        if (g_x5_split > 0) break;
      }
    }
  }
  auto launch = [&](int shape, int r0, int rows) {
    int bm, bn;
    x5_dims(shape, bm, bn);
    const int grid = std::min(((rows + bm - 1) / bm) * ((N + bn - 1) / bn), shape == 7 ? 2 * ncu : ncu);
    X5Args g{(const uint16_t*)a + (int64_t)r0 * lda, (const uint16_t*)b, (char*)c + (int64_t)r0 * ldc * 2, bias,
             lda, ldb, ldc, rows, N, K, c_dt};
    if (c_dt == F16) return bias ? x5_launch<F16, true>(shape, grid, g, s) : x5_launch<F16, false>(shape, grid, g, s);
    return bias ? x5_launch<BF16, true>(shape, grid, g, s) : x5_launch<BF16, false>(shape, grid, g, s);
  };
  int rc = launch(s1, 0, rows1);
  if (rc == 0 && s2 > 0) rc = launch(s2, rows1, M - rows1);
  return rc;
}
