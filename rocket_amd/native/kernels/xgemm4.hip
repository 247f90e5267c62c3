// One-wave-per-SIMD macro-tile GEMM (forward layout: A row, B row; C = A B^T [+ bias]):
//
//   256 x 256 block tile, 4 waves (2 x 2), 128 x 128 per wave = 8 x 8 MFMA 16x16x32 fragments whose
//   256 f32 accumulators live in the accumulator registers (inline-asm MFMAs with "+a" operands:
//   the builtin keeps them in arch VGPRs, which a 128 x 128 wave tile overflows).
//
// Why one wave per SIMD: a wave's LDS traffic per MFMA falls with its tile's perimeter/area, and
// 128 x 128 per wave halves it against the 8-wave 128 x 64 layout (xgemm_impl.h); nothing else
// shares the SIMD, so the schedule below must hide every latency itself:
//
//   k-tiles of 64 in a 2-stage LDS ring (2 x 64 KiB, LDS-DMA by buffer loads: zero VALU, hardware
//   OOB zeros); per k-tile t, two k-halves:
//     sub 0: fragment reads of half 1 of tile t  ||  64 MFMAs on half 0 (registers R0)
//     mid  : lgkmcnt(0) + vmcnt(0) (tile t+1 landed; issued one k-tile ago) + ONE barrier,
//            then the DMA of tile t+2 into tile t's stage (every wave has finished reading it)
//     sub 1: fragment reads of half 0 of tile t+1  ||  64 MFMAs on half 1 (registers R1)
//   so the DMA has a whole k-tile (128 MFMAs per wave, ~2k cycles) to land, fragment reads always
//   run under the other register set's MFMAs, and there is one barrier per 128 MFMAs.
//
// LDS images: [256 rows][64 k] bf16, 128-byte rows, the 16-byte k-chunk c of row r stored at
// chunk c ^ ((r >> 1) & 7): every ds_read_b128 lane group covers the 16 bank slots exactly once
// (tools/lds_banks.py); the DMA writes lane-linear 1-KiB pieces (8 rows) with the swizzle applied
// to each lane's SOURCE offset.
#include "mgemm_core.h"

using namespace rk;

namespace {

constexpr int X4_BM = 256, X4_BN = 256, X4_BK = 64, X4_NT = 256;
constexpr int X4_ROWB = X4_BK * 2;                 // 128-byte image rows
constexpr int X4_OPB = X4_BM * X4_ROWB;            // 32 KiB per operand per stage
constexpr int X4_STAGE = 2 * X4_OPB;               // A + B
constexpr int X4_NI = X4_OPB / (1024 * 4);         // 8 DMA instructions per operand per wave

__device__ __forceinline__ void mfma_a(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

#if defined(__HIP_DEVICE_COMPILE__)
// 8 rows x 128 B per instruction; wave w stages rows 64w .. 64w+63 of the operand's 256
__device__ __forceinline__ void x4_dma(const char* base, int64_t bytes, int64_t ld2, char* lds, int w,
                                       const uint32_t (&voff)[2]) {
  const int n = (int)(bytes < 0 ? 0 : (bytes > 0x7fffffff ? 0x7fffffff : bytes));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, n, 0x00020000);
#pragma unroll
  for (int i = 0; i < X4_NI; ++i) {
    // the row offset goes into the VGPR offset: only (voffset + inst offset) is range-checked
    // against the record count, so rows past M / N read as zeros only if it is there
    const int row0 = 64 * w + 8 * i;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + row0 * X4_ROWB), 16,
                                             voff[i & 1] + (uint32_t)(row0 * ld2), 0, 0, 0);
  }
}
#endif

__global__ void __launch_bounds__(X4_NT, 1) xgemm4_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                          const uint16_t* __restrict__ B, int64_t ldb, void* C,
                                                          int64_t ldc, int c_dt, const float* __restrict__ bias,
                                                          int M, int N, int K, int dbg) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * X4_STAGE];
  const int tiles_n = (N + X4_BN - 1) / X4_BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = (tile / tiles_n) * X4_BM, c0 = (tile % tiles_n) * X4_BN;
  const int lane = threadIdx.x & 63, lo = lane & 15, hi = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int T = K / X4_BK;

  // DMA source offsets: lane l of a 1-KiB piece lands at image row l/8, chunk l%8 = c ^ f(row);
  // f depends on row bits 1..3, bit 3 being the piece's parity -> two patterns
  uint32_t va[2], vb[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = 8 * p + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    va[p] = (uint32_t)((lane >> 3) * lda * 2 + c * 16);
    vb[p] = (uint32_t)((lane >> 3) * ldb * 2 + c * 16);
  }
  const char* abase = (const char*)A + (int64_t)r0 * lda * 2;
  const char* bbase = (const char*)B + (int64_t)c0 * ldb * 2;
  const int64_t abytes = ((int64_t)M - r0) * lda * 2, bbytes = ((int64_t)N - c0) * ldb * 2;
  auto dma = [&](int t) {
#if defined(__HIP_DEVICE_COMPILE__)
    char* st = smem + (t & 1) * X4_STAGE;
    x4_dma(abase + t * X4_ROWB, abytes - t * X4_ROWB, lda * 2, st, w, va);
    x4_dma(bbase + t * X4_ROWB, bbytes - t * X4_ROWB, ldb * 2, st + X4_OPB, w, vb);
#endif
  };

  // Fragment reads (inline asm, issued in a fixed interleave with the MFMAs; the compiler does
  // not track them, so every consumer is preceded by an explicit lgkmcnt(0) below).  A fragment i
  // of half s: image row 128 wm + 16 i + lo (chunk (4 s + hi) ^ f(row), f = (lo >> 1) & 7); the
  // fragment index only moves the row by 16 -> an immediate offset of i * 2048 bytes.
  const int fa = (lo >> 1) & 7;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const lds_void*)smem;
  const uint32_t arow = lds0 + (uint32_t)((128 * wm + lo) * X4_ROWB);
  const uint32_t brow = lds0 + (uint32_t)(X4_OPB + (128 * wn + lo) * X4_ROWB);
  auto addr = [&](uint32_t row, int t, int s) {
    return row + (uint32_t)((t & 1) * X4_STAGE) + (uint32_t)((((4 * s + hi) ^ fa)) * 16);
  };
#define X4_RD(dst, a, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(a), "i"(off))
  // the 16 reads of one register set (8 A, 8 B fragments)
#define X4_READ_ALL(RA, RB, aa, ab)                                                                     \
  do {                                                                                                 \
    X4_RD(RA[0], aa, 0); X4_RD(RA[1], aa, 2048); X4_RD(RA[2], aa, 4096); X4_RD(RA[3], aa, 6144);       \
    X4_RD(RA[4], aa, 8192); X4_RD(RA[5], aa, 10240); X4_RD(RA[6], aa, 12288); X4_RD(RA[7], aa, 14336); \
    X4_RD(RB[0], ab, 0); X4_RD(RB[1], ab, 2048); X4_RD(RB[2], ab, 4096); X4_RD(RB[3], ab, 6144);       \
    X4_RD(RB[4], ab, 8192); X4_RD(RB[5], ab, 10240); X4_RD(RB[6], ab, 12288); X4_RD(RB[7], ab, 14336); \
  } while (0)

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // 64 MFMAs on (Ra, Rb); when `rd`, the next register set's 16 reads go one per 4 MFMAs
  // (row i of the MFMA grid issues reads 2i, 2i+1: A fragment i and B fragment i)
  auto mma = [&](const bf16x8 (&Ra)[8], const bf16x8 (&Rb)[8], bool rd, bf16x8 (&Na)[8], bf16x8 (&Nb)[8],
                 uint32_t aa, uint32_t ab) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (rd) {
        switch (i) {  // immediate offsets must be literals
          case 0: X4_RD(Na[0], aa, 0); X4_RD(Nb[0], ab, 0); break;
          case 1: X4_RD(Na[1], aa, 2048); X4_RD(Nb[1], ab, 2048); break;
          case 2: X4_RD(Na[2], aa, 4096); X4_RD(Nb[2], ab, 4096); break;
          case 3: X4_RD(Na[3], aa, 6144); X4_RD(Nb[3], ab, 6144); break;
          case 4: X4_RD(Na[4], aa, 8192); X4_RD(Nb[4], ab, 8192); break;
          case 5: X4_RD(Na[5], aa, 10240); X4_RD(Nb[5], ab, 10240); break;
          case 6: X4_RD(Na[6], aa, 12288); X4_RD(Nb[6], ab, 12288); break;
          default: X4_RD(Na[7], aa, 14336); X4_RD(Nb[7], ab, 14336); break;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma_a(acc[i][j], Rb[j], Ra[i]);  // D[n][m]: 4 consecutive n per lane
    }
  };

  // simm16 of s_waitcnt: vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8]
  constexpr int kWaitLgkm0 = 0xC07F, kWaitAll0 = 0x0070;
  bf16x8 A0[8], B0[8], A1[8], B1[8];
  if (T > 0) {
    dma(0);
    if (T > 1) dma(1);
    if (T > 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0's 16 DMAs, tile 1's in flight
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    X4_READ_ALL(A0, B0, addr(arow, 0, 0), addr(brow, 0, 0));
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
  }
  for (int t = 0; t < T; ++t) {
    // sub 0: MFMAs on half 0 of tile t, reads of half 1 of tile t
    __builtin_amdgcn_s_setprio(1);
    mma(A0, B0, true, A1, B1, addr(arow, t, 1), addr(brow, t, 1));
    __builtin_amdgcn_s_setprio(0);
    // mid: half 1 in registers, every read of tile t's stage done, tile t+1 landed; one barrier
    if (t + 1 < T) __builtin_amdgcn_s_waitcnt(kWaitAll0);
    else __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(dbg & 2)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < T && !(dbg & 1)) dma(t + 2);  // into tile t's stage
    // sub 1: MFMAs on half 1, reads of half 0 of tile t+1
    __builtin_amdgcn_s_setprio(1);
    mma(A1, B1, t + 1 < T, A0, B0, addr(arow, t + 1, 0), addr(brow, t + 1, 0));
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
#undef X4_READ_ALL
#undef X4_RD

  // epilogue: lane holds D[n = 16 j + 4 hi + r][m = 16 i + lo]
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 7" ::: "memory");
  const int mb = r0 + 128 * wm, nb = c0 + 128 * wn;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = nb + 16 * j + 4 * hi;
    const bool nok = n < N;  // N % 4 == 0
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bias && nok) bv = *(const float4*)(bias + n);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mb + 16 * i + lo;
      if (!nok || m >= M) continue;
      const float v0 = acc[i][j][0] + bv.x, v1 = acc[i][j][1] + bv.y, v2 = acc[i][j][2] + bv.z,
                  v3 = acc[i][j][3] + bv.w;
      if (c_dt == F32) *(float4*)((float*)C + (int64_t)m * ldc + n) = make_float4(v0, v1, v2, v3);
      else *(uint2*)((uint16_t*)C + (int64_t)m * ldc + n) = make_uint2(pack16(v0, v1, c_dt), pack16(v2, v3, c_dt));
    }
  }
}

}  // namespace

// C[M][N] = A[M][K] B[N][K]^T (+ bias[N]); bf16 operands (rows 16-byte aligned), K % 64 == 0,
// N % 4 == 0; C f32 / bf16 / fp16 (c_dt).
int g_x4_dbg = 0;
RK_API int rk_xgemm4_set_dbg(int bits) {  // diagnostics: bit 0 no in-loop DMA, bit 1 no barrier
  g_x4_dbg = bits;
  return 0;
}
RK_API int rk_xgemm4(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int c_dt,
                     const float* bias, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % X4_BK || N % 4 || ((uintptr_t)a | (uintptr_t)b) % 16 || (lda * 2) % 16 || (ldb * 2) % 16)
    return (int)hipErrorInvalidValue;
  // per-lane + per-instruction DMA offsets stay below 2^31 (256 rows of the operand)
  if ((int64_t)256 * lda * 2 >= (1ll << 31) || (int64_t)256 * ldb * 2 >= (1ll << 31)) return (int)hipErrorInvalidValue;
  const int tiles = ((M + X4_BM - 1) / X4_BM) * ((N + X4_BN - 1) / X4_BN);
  xgemm4_kernel<<<tiles, X4_NT, 0, s>>>((const uint16_t*)a, lda, (const uint16_t*)b, ldb, c, ldc, c_dt, bias, M, N, K,
                                        g_x4_dbg);
  return (int)hipGetLastError();
}
