// Macro-tile bf16 MFMA GEMM (the round-4 main loop for the transformer projections and the
// weight gradients; same contract and epilogues as mgemm.hip's rk_mgemm, see its header).
//
//   C[M,N] (op)= epi( sum_k A(m,k) * B(n,k) ),  A/B each "row" (K contiguous) or "kmaj" (K-major)
//
// Main loop, designed around what the ISA of the earlier 128x128 / ping-pong loops showed
// (profiles/r2_mgemm_pingpong.md: ~12 VALU per LDS-DMA for 64-bit addresses, zero-page selects and
// clamps, and a barrier every 16 MFMAs):
// * BIG per-wave tiles: 4 waves x (128 x 128) (one wave per SIMD, 256 f32 accumulators each, held
//   in the accumulator registers) or 8 waves x (128 x 64) on a 256 x 256 block tile; 192 x 256 and
//   256 x 128 block tiles for the wave quantisation of N = 768 products (config table below).
// * LDS-DMA by BUFFER loads (buffer_load_dwordx4 ... lds): the per-lane source offsets are computed
//   once; per k-unit only the SGPR descriptor base moves (zero VALU per DMA), and the descriptor's
//   record count bounds every read, so rows past M / N and k rows past K read as zeros in hardware
//   (no clamps, no zero page).
// * k-units of 32 in a 4-slot ring: units u+1..u+3 in flight while u is consumed (~3 units of
//   MFMA time to cover L2 / MALL latency), ONE barrier per unit, counted vmcnt (never 0 inside the
//   loop), raw s_barrier (a __syncthreads() would drain the DMAs: cdna guide §5).
// * Fragments of unit u+1 are read into a second named register set while unit u's MFMAs run
//   (loop unrolled by two: no register copies), so the matrix core never waits on ds_read.
// * Swizzles (bank-conflict-free ds_read_b128 / ds_read_b64_tr_b16) and the fused epilogue are
//   mgemm_core.h's, shared with mgemm.hip and conv.hip.
#pragma once
#include "mgemm_core.h"

using namespace rk;

namespace {

// The buffer-resource type exists only in the device pass: code naming it is kept out of the host
// pass (there it silently suppressed the host launch stubs of the kernels that use it).

// LDS-DMA of one operand's 32-deep k-unit: R rows x 32 k (row image, 64-B rows) or 32 k-rows x R
// (kmaj image); lane-linear LDS image, swizzle on the per-lane SOURCE offset (guide rule 21).
template <int R, bool KMAJ, int NW>
struct BStager {
  static constexpr int BK = 32;
  static constexpr int NI = R * BK / (512 * NW);  // 1-KiB wave instructions per unit
  static_assert(NI >= 1 && R * BK % (512 * NW) == 0, "tile too small for the wave count");
  uint32_t off[NI];
  __device__ __forceinline__ void init(int64_t ld, int r0, int wid, int lane) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (wid * NI + i) * 64 + lane;  // 16-byte chunk of the lane-linear image
      if constexpr (!KMAJ) {
        const int r = q >> 2, c = q & 3;
        off[i] = (uint32_t)(((int64_t)(r0 + r) * ld + (c ^ rswz<32>(r)) * 8) * 2);
      } else {
        constexpr int CPR = R / 8;
        const int k = q / CPR, c = q % CPR;
        off[i] = (uint32_t)(((int64_t)k * ld + r0 + (c ^ kswz<R>(k)) * 8) * 2);
      }
    }
  }
  // base: wave-uniform address of this unit's (row 0 | k-row 0); bytes: the extent readable from it
  __device__ __forceinline__ void issue(const char* base, int64_t bytes, char* lds, int wid) const {
#if defined(__HIP_DEVICE_COMPILE__)
    const int n = (int)(bytes < 0 ? 0 : (bytes > 0x7fffffff ? 0x7fffffff : bytes));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, n, 0x00020000);
#pragma unroll
    for (int i = 0; i < NI; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + (wid * NI + i) * 1024), 16, off[i], 0, 0, 0);
#endif
  }
};

// MFMA with its accumulator pinned to the accumulator registers ("a"): with one wave per SIMD a
// wave's 128-256 accumulators live there, the 256 arch VGPRs hold operands and addresses.  (The
// builtin lets the backend pick: it keeps accumulators in arch VGPRs and spills.)  The accumulate
// chain on one register block needs no wait states; independent blocks none either.
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;

template <bool H>
__device__ __forceinline__ void mfma_agpr(f32x4& c, const bf16x8& a, const bf16x8& b) {
  if constexpr (H) asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// the same on arch-VGPR accumulators (builtin; the backend schedules and pads it); operands are
// carried as bf16x8 bit patterns either way
template <bool H>
__device__ __forceinline__ f32x4 mfma_v(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (H)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// s_waitcnt vmcnt(n), n in [0, 63] at run time (larger n clamps to 63: waiting for more is safe)
__device__ __forceinline__ void wait_vm_any(int n) {
  n = n < 0 ? 0 : (n > 63 ? 63 : n);
  if (n < 16) { wait_vm(n > 12 ? 12 : n); return; }
#define XG_W(k) if (n >= k) { asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); return; }
  XG_W(56) XG_W(48) XG_W(40) XG_W(32) XG_W(24) XG_W(16)
#undef XG_W
}

#if defined(__HIP_DEVICE_COMPILE__)
typedef unsigned int u32v4 __attribute__((vector_size(16)));
typedef unsigned int u32v2 __attribute__((vector_size(8)));
__device__ __forceinline__ void st128(__amdgpu_buffer_rsrc_t rs, uint32_t off, const float (&v)[4]) {
  u32v4 d = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(d, rs, off, 0, 0);
}
__device__ __forceinline__ void st64(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t a, uint32_t b) {
  u32v2 d = {a, b};
  __builtin_amdgcn_raw_buffer_store_b64(d, rs, off, 0, 0);
}
#endif

// One work item of a persistent block: an output tile of one K split, walked in 32-deep units.
struct XItem {
  int r0, c0, tn, split, kb, ke, nt;
};

// Persistent form of xgemm_kernel (one block per CU, each walking output tiles pos, pos + G, ...
// with pos XCD-aware, so an XCD's 32 CUs work on neighbouring tiles at every step): the k-units of
// ALL its tiles are ONE stream through the 4-slot ring, so the next tile's first units are in
// flight while the current tile's last ones are consumed -- no pipeline fill per tile.  Per-lane
// DMA offsets are tile-relative (the tile origin moves only the SGPR descriptor base).  The
// epilogue stores by buffer stores whose record bound drops out-of-range lanes in hardware: every
// wave issues a known number of stores, so the first boundary after an epilogue waits with an
// exact count instead of draining the ring.
template <int BM, int BN, int WM, int WN, bool AK, bool BKM, bool ROWS, bool H>
__global__ void __launch_bounds__(64 * WM * WN, 1) xgemm_pkernel(MArgs g, int64_t a_bytes, int64_t b_bytes) {
  constexpr int BK = 32, NS = 4, NW = WM * WN;
  constexpr bool AGPR_ACC = WM * WN == 4;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  using SA = BStager<BM, AK, NW>;
  using SB = BStager<BN, BKM, NW>;
  constexpr int NL = SA::NI + SB::NI;
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  const int dbg = g.dbg;  // diagnostics bits, read once (rk_xgemm_set_dbg)
  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int total = ntiles * g.splitk;
  const int G = gridDim.x;
  const int pos = xcd_remap(blockIdx.x, G);
  const int my = pos < total ? (total - pos + G - 1) / G : 0;

  auto place = [&](int i) {
    XItem it;
    const int lin = pos + i * G;
    it.split = lin / ntiles;
    const int tile = lin - it.split * ntiles;
    const int tm = tile / tiles_n;
    it.tn = tile - tm * tiles_n;
    it.r0 = tm * BM;
    it.c0 = it.tn * BN;
    it.kb = it.split * g.k_per_split;
    it.ke = min(g.K, it.kb + g.k_per_split);
    it.nt = (it.ke - it.kb + BK - 1) / BK;
    return it;
  };
  int S = 0;  // units in this block's stream
  for (int i = 0; i < my; ++i) S += place(i).nt;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  static_assert(FM % WN == 0, "row-sum fragments split evenly over the N-waves");
  constexpr int FR = FM / WN;
  f32x4 racc[FR];
#pragma unroll
  for (int i = 0; i < FR; ++i) racc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = __builtin_bit_cast(__bf16, (uint16_t)(H ? 0x3c00 : 0x3f80));

  SA sa;
  SB sb;
  sa.init(g.lda, 0, wid, lane);  // tile-relative offsets
  sb.init(g.ldb, 0, wid, lane);

  // issue cursor: item / unit of the next DMA
  XItem iss = place(0);
  int iss_i = 0, iss_kt = 0;
  auto issue_next = [&](int u) {
    char* buf = smem + (u & (NS - 1)) * STAGE;
    const int k0 = iss.kb + iss_kt * BK;
    const int64_t ao = AK ? ((int64_t)k0 * g.lda + iss.r0) * 2 : ((int64_t)iss.r0 * g.lda + k0) * 2;
    const int64_t bo = BKM ? ((int64_t)k0 * g.ldb + iss.c0) * 2 : ((int64_t)iss.c0 * g.ldb + k0) * 2;
    const int64_t a_end = AK ? (int64_t)iss.ke * g.lda * 2 : a_bytes;
    const int64_t b_end = BKM ? (int64_t)iss.ke * g.ldb * 2 : b_bytes;
    if (!(dbg & 1)) {
      sa.issue((const char*)g.a + ao, a_end - ao, buf, wid);
      sb.issue((const char*)g.b + bo, b_end - bo, buf + A_BYTES, wid);
    }
    if (++iss_kt == iss.nt) {
      iss_kt = 0;
      if (++iss_i < my) iss = place(iss_i);
    }
  };

  FragReader<BM, BK, AK, FM> ra;
  FragReader<BN, BK, BKM, FN> rb;
  ra.init(wm * TM, lane);
  rb.init(wn * TN, lane);
  bf16x8 A0[FM], B0[FN], A1[FM], B1[FN];
  auto read = [&](bf16x8 (&A)[FM], bf16x8 (&B)[FN], int u) {
    if (dbg & 4) return;
    const char* As = smem + (u & (NS - 1)) * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int j = 0; j < FN; ++j) B[j] = rb.get(Bs, j, 0);
#pragma unroll
    for (int i = 0; i < FM; ++i) A[i] = ra.get(As, i, 0);
  };
  XItem cur = place(0);  // compute cursor (the item being consumed)
  auto mma = [&](const bf16x8 (&A)[FM], const bf16x8 (&B)[FN]) {
    if (dbg & 8) return;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (AGPR_ACC) mfma_agpr<H>(acc[i][j], B[j], A[i]);
        else acc[i][j] = mfma_v<H>(B[j], A[i], acc[i][j]);
      }
    if constexpr (ROWS) {
      if (cur.tn == 0) {
#pragma unroll
        for (int w = 0; w < WN; ++w)
          if (wn == w) {
#pragma unroll
            for (int r = 0; r < FR; ++r) racc[r] = mfma_v<H>(ones, A[w * FR + r], racc[r]);
          }
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // C descriptor (records = the bytes of C / of one slab plane): out-of-range lanes get an offset
  // past the bound and their store is dropped.  Epilogues: + bias, C += (accumulate), f32 / bf16 /
  // fp16 out, or f32 split-K slabs (the activation epilogues stay on rk_mgemm: their per-element
  // code, unrolled over every fragment, no longer fits the pragma-unroll budget and the
  // accumulators would fall to scratch)
  const bool slab_out = g.splitk > 1;
  const int csz = (g.c_dt == F32 || slab_out) ? 4 : 2;
  const int64_t c_rec = slab_out ? (int64_t)g.M * g.N * 4 : ((int64_t)(g.M - 1) * g.ldc + g.N) * csz;
  const int c_n = (int)(c_rec > 0x7fffffff ? 0x7fffffff : c_rec);
  const int64_t ldc = slab_out ? g.N : g.ldc;
  const bool wide = g.c_dt == F32 || slab_out;
  const int n_st = FM * FN;  // stores every wave issues per epilogue
  auto epilogue = [&]() {
    if constexpr (AGPR_ACC) {
      asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 7" ::: "memory");
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[i][j]));
    }
    if constexpr (ROWS) {
      if (cur.tn == 0 && lane < 16) {
#pragma unroll
        for (int r = 0; r < FR; ++r) {
          const int m = cur.r0 + wm * TM + (wn * FR + r) * 16 + lane;
          if (m < g.M) atomicAdd(g.rowsum + m, racc[r][0]);
          racc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
#if defined(__HIP_DEVICE_COMPILE__)
    const int mbase = cur.r0 + wm * TM, nbase = cur.c0 + wn * TN;
    char* cbase = slab_out ? (char*)(g.slab + (int64_t)cur.split * g.M * g.N) : (char*)g.c;
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(cbase, (short)0, c_n, 0x00020000);
    const bool addb = !slab_out && g.bias != nullptr;
    const bool accum = !slab_out && g.accumulate;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nbase + j * 16 + 4 * (lane >> 4);
      const bool nok = n < g.N;  // N % 4 == 0: a lane's 4 columns are all in or all out
      float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
      if (addb && nok) bias = *(const float4*)(g.bias + n);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = mbase + i * 16 + (lane & 15);
        const bool ok = nok && m < g.M;
        const int64_t e = (int64_t)m * ldc + n;
        const uint32_t off = ok ? (uint32_t)(e * csz) : 0x80000000u;
        float v[4] = {acc[i][j][0] + bias.x, acc[i][j][1] + bias.y, acc[i][j][2] + bias.z, acc[i][j][3] + bias.w};
        if (wide) {
          if (accum && ok) {
            const float4 o = *(const float4*)((const float*)g.c + e);
            v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
          }
          st128(crs, off, v);
        } else {
          if (accum && ok) {
            const uint2 o = *(const uint2*)((const uint16_t*)g.c + e);
            v[0] += lo16(o.x, g.c_dt); v[1] += hi16(o.x, g.c_dt); v[2] += lo16(o.y, g.c_dt); v[3] += hi16(o.y, g.c_dt);
          }
          st64(crs, off, pack16(v[0], v[1], g.c_dt), pack16(v[2], v[3], g.c_dt));
        }
      }
    }
#endif
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  auto sync = [&]() {
    if (dbg & 2) return;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  int pend = 0;  // stores of an epilogue since the last boundary (counted by vmcnt)
  auto boundary = [&](int u) {
    const int cnt = (min(S - 1, u + 3) - (u + 1)) * NL + pend;
    if (cnt == 2 * NL) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NL) : "memory");  // steady state
    else wait_vm_any(cnt);
    sync();
    if (u + 4 < S) issue_next(u + 4);
    pend = 0;
  };
  // unit u: make u+1 visible (u+2, u+3 may stay in flight, plus the last epilogue's stores), refill
  // u's slot with u+4, read u+1's fragments into (NA, NB) under u's MFMAs on (CA, CB)
#define XP_UNIT(u, CA, CB, NA, NB) \
  do {                             \
    boundary(u);                   \
    read(NA, NB, (u) + 1);         \
    mma(CA, CB);                   \
  } while (0)
  // a tile's last unit: MFMAs, the epilogue (both operand sets dead: its temporaries fit beside the
  // accumulators), then the next tile's first fragments into (A0, B0)
#define XP_LAST(u, CA, CB)                       \
  do {                                           \
    const bool more = (u) + 1 < S;               \
    if (more) boundary(u);                       \
    mma(CA, CB);                                 \
    epilogue();                                  \
    asm volatile("" ::: "memory");               \
    __builtin_amdgcn_sched_barrier(0);           \
    pend = n_st;                                 \
    if (more) read(A0, B0, (u) + 1);             \
  } while (0)

  if (S > 0) {
#pragma unroll
    for (int u = 0; u < NS - 1; ++u)
      if (u < S) issue_next(u);
    wait_vm(min(S - 1, NS - 2) * NL);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (NS - 1 < S) issue_next(NS - 1);
    read(A0, B0, 0);
    int u = 0;
    for (int i = 0; i < my; ++i) {
      cur = place(i);
      int kt = 0;
      for (; kt + 2 < cur.nt; kt += 2, u += 2) {  // every unit of the pair has a successor in the tile
        XP_UNIT(u, A0, B0, A1, B1);
        XP_UNIT(u + 1, A1, B1, A0, B0);
      }
      if (kt + 1 < cur.nt) {
        XP_UNIT(u, A0, B0, A1, B1);
        XP_LAST(u + 1, A1, B1);
        u += 2;
      } else {
        XP_LAST(u, A0, B0);
        u += 1;
      }
    }
  }
#undef XP_LAST
#undef XP_UNIT
  // every store of this block retired before the block ends (and the LDS ring is idle)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// launch one layout's kernel (persistent: at most one block per CU, each walking items pos,
// pos + grid, ...); the row-sum variant when a wgrad also forms the bias gradient
template <int BM, int BN, int WM, int WN, bool AK, bool BKM, bool H>
int launch_l(const MArgs& g, int64_t a_bytes, int64_t b_bytes, int num_cus, hipStream_t s) {
  const int items = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN) * g.splitk;
  const dim3 grid(std::min(items, num_cus)), block(64 * WM * WN);
  if (AK && BKM && g.rowsum)
    xgemm_pkernel<BM, BN, WM, WN, AK, BKM, AK && BKM, H><<<grid, block, 0, s>>>(g, a_bytes, b_bytes);
  else
    xgemm_pkernel<BM, BN, WM, WN, AK, BKM, false, H><<<grid, block, 0, s>>>(g, a_bytes, b_bytes);
  return (int)hipGetLastError();
}

// block tile of each config (the host entry checks shapes against it)
constexpr int kXBM[] = {256, 256};
constexpr int kXBN[] = {256, 128};

template <bool AK, bool BKM>
int launch_layout(const void* gp, int cfg, int h, int64_t a_bytes, int64_t b_bytes, int num_cus, hipStream_t s) {
  const MArgs& g = *(const MArgs*)gp;
  switch (cfg * 2 + (h ? 1 : 0)) {
    case 0: return launch_l<256, 256, 2, 4, AK, BKM, false>(g, a_bytes, b_bytes, num_cus, s);
    case 1: return launch_l<256, 256, 2, 4, AK, BKM, true>(g, a_bytes, b_bytes, num_cus, s);
    case 2: return launch_l<256, 128, 4, 2, AK, BKM, false>(g, a_bytes, b_bytes, num_cus, s);
    case 3: return launch_l<256, 128, 4, 2, AK, BKM, true>(g, a_bytes, b_bytes, num_cus, s);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// One translation unit per operand layout instantiates the launchers (parallel compilation):
//   layout 0: A row, B row (forward)  1: A row, B kmaj (dgrad)  2: A kmaj, B kmaj (wgrad)
// Configs: 0 = 256 x 256 block, 8 waves (2 x 4), 128 x 64 per wave; 1 = 256 x 128 block, 8 waves
// (4 x 2), 64 x 64 per wave.  h: fp16 operands.
#define RKX_DECLARE(L) extern "C" int rkx_launch_l##L(const void* g, int cfg, int h, int64_t a_bytes, int64_t b_bytes, \
                                                     int num_cus, hipStream_t s)
RKX_DECLARE(0);
RKX_DECLARE(1);
RKX_DECLARE(2);
