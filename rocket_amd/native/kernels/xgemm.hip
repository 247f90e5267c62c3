// Macro-tile bf16 MFMA GEMM (the round-4 main loop for the transformer projections and the
// weight gradients; same contract and epilogues as mgemm.hip's rk_mgemm, see its header).
//
//   C[M,N] (op)= epi( sum_k A(m,k) * B(n,k) ),  A/B each "row" (K contiguous) or "kmaj" (K-major)
//
// Main loop, designed around what the ISA of the earlier 128x128 / ping-pong loops showed
// (profiles/r2_mgemm_pingpong.md: ~12 VALU per LDS-DMA for 64-bit addresses, zero-page selects and
// clamps, and a barrier every 16 MFMAs):
// * BIG per-wave tiles, accumulators in the register file's accumulator half: 4 waves x (128 x 128)
//   (one wave per SIMD, 256 f32 accumulators each) or 8 waves x (128 x 64) on a 256 x 256 block
//   tile, or 4 waves x (160 x 128) on a 320 x 256 tile (M = 25216 tokens = 79 row tiles: 237 / 711
//   / 948 tiles for N = 768 / 2304 / 3072, i.e. 93 % of the last wave of 256 CUs is busy, against
//   58 % for 297 tiles of 256 x 256 at N = 768).
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

template <int BM, int BN, int WM, int WN, bool AK, bool BKM, bool ROWS>
__global__ void __launch_bounds__(64 * WM * WN, 1) xgemm_kernel(MArgs g, int64_t a_bytes, int64_t b_bytes) {
  constexpr int BK = 32, NS = 4, NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  using SA = BStager<BM, AK, NW>;
  using SB = BStager<BN, BKM, NW>;
  constexpr int NL = SA::NI + SB::NI;  // DMA wave instructions per unit
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / ntiles;
  const int tile = lin % ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int kb = split * g.k_per_split;
  const int ke = min(g.K, kb + g.k_per_split);
  const int nt = (ke - kb + BK - 1) / BK;  // a partial last unit (both operands kmaj) reads zeros past K

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // bias-gradient row sums (wgrad, ROWS): tile column 0 only; wave wn sums A fragments
  // [wn*FR, (wn+1)*FR) against a ones fragment
  const bool want_rows = ROWS && tn == 0;
  static_assert(FM % WN == 0, "row-sum fragments split evenly over the N-waves");
  constexpr int FR = FM / WN;
  f32x4 racc[FR];
#pragma unroll
  for (int i = 0; i < FR; ++i) racc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  SA sa;
  SB sb;
  sa.init(g.lda, row0, wid, lane);
  sb.init(g.ldb, col0, wid, lane);
  // operand bases at k = kb and the byte step of one unit; every descriptor is built from
  // wave-uniform values (SGPRs), its record count = the bytes left from its base
  const int64_t a_k0 = AK ? (int64_t)kb * g.lda * 2 : (int64_t)kb * 2;
  const int64_t b_k0 = BKM ? (int64_t)kb * g.ldb * 2 : (int64_t)kb * 2;
  const int64_t a_step = AK ? (int64_t)BK * g.lda * 2 : BK * 2;
  const int64_t b_step = BKM ? (int64_t)BK * g.ldb * 2 : BK * 2;
  // the K extent of this split as a record bound: a kmaj operand's rows past ke read as zeros
  const int64_t a_end = AK ? (int64_t)ke * g.lda * 2 : a_bytes;
  const int64_t b_end = BKM ? (int64_t)ke * g.ldb * 2 : b_bytes;
  auto issue = [&](int t) {
    char* buf = smem + (t & (NS - 1)) * STAGE;
    const int64_t ao = a_k0 + t * a_step, bo = b_k0 + t * b_step;
    sa.issue((const char*)g.a + ao, a_end - ao, buf, wid);
    sb.issue((const char*)g.b + bo, b_end - bo, buf + A_BYTES, wid);
  };
  FragReader<BM, BK, AK, FM> ra;
  FragReader<BN, BK, BKM, FN> rb;
  ra.init(wm * TM, lane);
  rb.init(wn * TN, lane);

  bf16x8 A0[FM], B0[FN], A1[FM], B1[FN];
  auto read = [&](bf16x8 (&A)[FM], bf16x8 (&B)[FN], int t) {
    const char* As = smem + (t & (NS - 1)) * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int j = 0; j < FN; ++j) B[j] = rb.get(Bs, j, 0);
#pragma unroll
    for (int i = 0; i < FM; ++i) A[i] = ra.get(As, i, 0);
  };
  auto mma = [&](const bf16x8 (&A)[FM], const bf16x8 (&B)[FN]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[j], A[i], acc[i][j], 0, 0, 0);
    if constexpr (ROWS) {
      if (want_rows) {  // one wave-uniform branch per N-wave, static fragment indices inside
#pragma unroll
        for (int w = 0; w < WN; ++w)
          if (wn == w) {
#pragma unroll
            for (int r = 0; r < FR; ++r)
              racc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, A[w * FR + r], racc[r], 0, 0, 0);
          }
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // top of unit t: unit t+1 landed in every wave (units up to t+3 may stay in flight), every wave
  // retired its reads of unit t (lgkmcnt(0)): unit t's slot takes unit t+4.  `steady`: t+4 < nt,
  // so the wait count is the compile-time 2*NL and the refill is unconditional (no branch trees
  // inside the main loop: they split its scheduling regions)
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  auto boundary_steady = [&](int t) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NL) : "memory");
    sync();
    issue(t + 4);
  };
  auto boundary = [&](int t) {
    wait_vm((min(nt - 1, t + 3) - (t + 1)) * NL);
    sync();
    if (t + 4 < nt) issue(t + 4);
  };

  // prologue: units 0..3 in flight, unit 0 landed and read
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nt) issue(t);
  wait_vm(min(nt - 1, NS - 2) * NL);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (NS - 1 < nt) issue(NS - 1);
  read(A0, B0, 0);

  // A macro, not a lambda over array references: each set stays a distinct named register block
#define XG_STEADY(t, CA, CB, NA, NB) \
  do {                               \
    boundary_steady(t);              \
    read(NA, NB, (t) + 1);           \
    mma(CA, CB);                     \
  } while (0)
#define XG_UNIT(t, CA, CB, NA, NB)     \
  do {                                 \
    if ((t) + 1 < nt) {                \
      boundary(t);                     \
      read(NA, NB, (t) + 1);           \
    }                                  \
    mma(CA, CB);                       \
  } while (0)

  int t = 0;
  for (; t + 5 < nt; t += 2) {  // main loop: both units of the pair refill the ring
    XG_STEADY(t, A0, B0, A1, B1);
    XG_STEADY(t + 1, A1, B1, A0, B0);
  }
  for (; t < nt; t += 2) {  // the last <= 5 units: the ring drains
    XG_UNIT(t, A0, B0, A1, B1);
    if (t + 1 < nt) XG_UNIT(t + 1, A1, B1, A0, B0);
  }
#undef XG_UNIT
#undef XG_STEADY

  if (want_rows && lane < 16) {
#pragma unroll
    for (int r = 0; r < FR; ++r) {
      const int m = row0 + wm * TM + (wn * FR + r) * 16 + lane;
      if (m < g.M) atomicAdd(g.rowsum + m, racc[r][0]);
    }
  }
  const uint2 nos[FM][FN] = {};
  store_tile<FM, FN, false>(g, acc, nos, row0 + wm * TM, col0 + wn * TN, lane, split);
}

template <int BM, int BN, int WM, int WN>
int launch_x(const MArgs& g, int a_kmaj, int b_kmaj, int64_t a_bytes, int64_t b_bytes, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  const dim3 grid(tiles * g.splitk), block(64 * WM * WN);
  if (!a_kmaj && !b_kmaj) xgemm_kernel<BM, BN, WM, WN, false, false, false><<<grid, block, 0, s>>>(g, a_bytes, b_bytes);
  else if (!a_kmaj && b_kmaj) xgemm_kernel<BM, BN, WM, WN, false, true, false><<<grid, block, 0, s>>>(g, a_bytes, b_bytes);
  else if (a_kmaj && b_kmaj && g.rowsum)
    xgemm_kernel<BM, BN, WM, WN, true, true, true><<<grid, block, 0, s>>>(g, a_bytes, b_bytes);
  else if (a_kmaj && b_kmaj) xgemm_kernel<BM, BN, WM, WN, true, true, false><<<grid, block, 0, s>>>(g, a_bytes, b_bytes);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

}  // namespace

// Configs (block tile, waves, per-wave tile; 1 block per CU, 4-slot ring of 32-deep k-units):
//   0: 256 x 256, 4 waves (2 x 2), 128 x 128 per wave   (128 KiB LDS)
//   1: 256 x 256, 8 waves (2 x 4), 128 x 64 per wave    (128 KiB)
//   2: 320 x 256, 4 waves (2 x 2), 160 x 128 per wave   (144 KiB; row-layout A only)
//   3: 256 x 128, 4 waves (2 x 2), 128 x 64 per wave    (96 KiB)
// Requirements (hipErrorInvalidValue otherwise; the caller falls back to rk_mgemm): K % 32 == 0
// unless both operands are kmaj; N % 8; a kmaj operand's extent % 8; 16-byte aligned operands and
// leading dimensions; every per-lane source offset < 2^31 bytes.
RK_API int rk_xgemm(const void* a, int64_t lda, int a_kmaj, const void* b, int64_t ldb, int b_kmaj, void* c, int c_dt,
                    int64_t ldc, void* c_pre, const float* bias, const void* aux, int epi, int accumulate,
                    float* rowsum, int M, int N, int K, int splitk, int cfg, float* slab, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (cfg < 0 || cfg > 3 || (cfg == 2 && a_kmaj)) return (int)hipErrorInvalidValue;
  if (K <= 0 || ((!a_kmaj || !b_kmaj) && K % 32) || N % 8 || (a_kmaj && M % 8) || ldc % 4)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)a | (uintptr_t)b) % 16 || (lda * 2) % 16 || (ldb * 2) % 16) return (int)hipErrorInvalidValue;
  if ((epi == kMulGeluGrad || epi == kMulReluGrad) && aux == nullptr) return (int)hipErrorInvalidValue;
  const int BM = cfg == 2 ? 320 : 256, BN = cfg == 3 ? 128 : 256;
  // operand extents in bytes (row: rows x ld; kmaj: K rows x ld) and the largest per-lane offset
  const int64_t a_bytes = a_kmaj ? (int64_t)K * lda * 2 : (int64_t)M * lda * 2;
  const int64_t b_bytes = b_kmaj ? (int64_t)K * ldb * 2 : (int64_t)N * ldb * 2;
  const int64_t a_off_max = a_kmaj ? (int64_t)32 * lda * 2 + (M + BM) * 2 : (int64_t)(M + BM) * lda * 2;
  const int64_t b_off_max = b_kmaj ? (int64_t)32 * ldb * 2 + (N + BN) * 2 : (int64_t)(N + BN) * ldb * 2;
  if (a_off_max >= (1ll << 31) || b_off_max >= (1ll << 31)) return (int)hipErrorInvalidValue;
  MArgs g;
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c; g.c_pre = c_pre; g.bias = bias;
  g.aux = (const uint16_t*)aux; g.rowsum = rowsum; g.slab = slab;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.c_dt = c_dt; g.epi = epi; g.accumulate = accumulate;
  g.lds_epi = 0;
  if (splitk < 1) splitk = 1;
  const int kq = 32;  // split boundaries on whole units
  const int kps = ((K + kq - 1) / kq + splitk - 1) / splitk * kq;
  splitk = (K + kps - 1) / kps;
  if (splitk > 1 && (slab == nullptr || epi != kNone || c_pre)) return (int)hipErrorInvalidValue;
  g.splitk = splitk;
  g.k_per_split = kps;
  int rc;
  switch (cfg) {
    case 0: rc = launch_x<256, 256, 2, 2>(g, a_kmaj, b_kmaj, a_bytes, b_bytes, s); break;
    case 1: rc = launch_x<256, 256, 2, 4>(g, a_kmaj, b_kmaj, a_bytes, b_bytes, s); break;
    case 2: rc = launch_x<320, 256, 2, 2>(g, a_kmaj, b_kmaj, a_bytes, b_bytes, s); break;
    default: rc = launch_x<256, 128, 2, 2>(g, a_kmaj, b_kmaj, a_bytes, b_bytes, s); break;
  }
  if (rc || splitk == 1) return rc;
  launch_mgemm_reduce(slab, splitk, M, N, bias, c, c_dt, ldc, accumulate, s);
  return (int)hipGetLastError();
}
