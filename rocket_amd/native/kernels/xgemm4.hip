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
// the same with C = 0: starts an accumulation (no zeroing of the accumulator registers needed)
__device__ __forceinline__ void mfma_a0(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
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
// one of the X4_NI instructions of x4_dma (the spread schedule issues them between MFMAs)
__device__ __forceinline__ void x4_dma1(const char* base, int64_t bytes, int64_t ld2, char* lds, int w,
                                        const uint32_t (&voff)[2], int i) {
  const int n = (int)(bytes < 0 ? 0 : (bytes > 0x7fffffff ? 0x7fffffff : bytes));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, n, 0x00020000);
  const int row0 = 64 * w + 8 * i;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + row0 * X4_ROWB), 16, voff[i & 1] + (uint32_t)(row0 * ld2),
                                           0, 0, 0);
}
#endif

// Fused epilogues of the LDS-staged store path (16-bit C, N % 8 == 0).  The staged tile holds
// t = round16(acc + bias), exactly what an unfused GEMM would have written, so the fused forms keep
// the unfused numerics:
//   X4_GELU      c_pre = t (the pre-activation, for the backward), C = round16(gelu(t))
//   X4_MULGELU   C = round16(t * gelu'(aux)) (aux = the GELU's input z: the input gradient of a GELU
//                that fed this layer), and colsum[n] += sum over the tile's rows of the f32 product
//                (the bias gradient of the layer that produced z), one f32 atomic per column per wave
enum X4EpiKind : int { X4_NONE = 0, X4_GELU = 1, X4_MULGELU = 2 };
struct X4Epi {
  void* c_pre;
  const uint16_t* aux;
  float* colsum;
  int kind;
};

template <bool SPREAD>
__global__ void __launch_bounds__(X4_NT, 1) xgemm4_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                          const uint16_t* __restrict__ B, int64_t ldb, void* C,
                                                          int64_t ldc, int c_dt, const float* __restrict__ bias,
                                                          int M, int N, int K, int dbg, uint64_t* trace, X4Epi ep) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * X4_STAGE];
  // diagnostics (rk_xgemm4_set_trace): thread 0 stamps s_memrealtime (100 MHz) at block start,
  // prologue done, main loop done, epilogue done, plus the tile id: trace[block][0..4]
  uint64_t* const tr = trace ? trace + (int64_t)blockIdx.x * 8 : nullptr;
  if (tr && threadIdx.x == 0) tr[0] = __builtin_amdgcn_s_memrealtime();
  const int tiles_n = (N + X4_BN - 1) / X4_BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  if (dbg & 8) { tm = tile / tiles_n; tn = tile % tiles_n; }  // row-major walk (diagnostics)
  else grouped_tile(tile, (M + X4_BM - 1) / X4_BM, tiles_n, 4, tm, tn);
  const int r0 = tm * X4_BM, c0 = tn * X4_BN;
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
  if (tr && threadIdx.x == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
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
    if constexpr (!SPREAD) {
      if (t + 2 < T && !(dbg & 1)) dma(t + 2);  // into tile t's stage
      // sub 1: MFMAs on half 1, reads of half 0 of tile t+1
      __builtin_amdgcn_s_setprio(1);
      mma(A1, B1, t + 1 < T, A0, B0, addr(arow, t + 1, 0), addr(brow, t + 1, 0));
      __builtin_amdgcn_s_setprio(0);
    } else {
      // spread schedule (the library's): tile t+2's 16 DMA instructions go out one per 4 MFMAs of
      // sub 1 instead of as one burst at the barrier, so they never queue ahead of a fragment read
      const bool dm = t + 2 < T && !(dbg & 1);
      const bool rd = t + 1 < T;
      const uint32_t aa = addr(arow, t + 1, 0), ab = addr(brow, t + 1, 0);
#if defined(__HIP_DEVICE_COMPILE__)
      char* st = smem + (t & 1) * X4_STAGE;
      const char* ga = abase + (t + 2) * X4_ROWB;
      const char* gb = bbase + (t + 2) * X4_ROWB;
      const int64_t na = abytes - (t + 2) * X4_ROWB, nb = bbytes - (t + 2) * X4_ROWB;
#endif
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (rd) {
          switch (i) {
            case 0: X4_RD(A0[0], aa, 0); X4_RD(B0[0], ab, 0); break;
            case 1: X4_RD(A0[1], aa, 2048); X4_RD(B0[1], ab, 2048); break;
            case 2: X4_RD(A0[2], aa, 4096); X4_RD(B0[2], ab, 4096); break;
            case 3: X4_RD(A0[3], aa, 6144); X4_RD(B0[3], ab, 6144); break;
            case 4: X4_RD(A0[4], aa, 8192); X4_RD(B0[4], ab, 8192); break;
            case 5: X4_RD(A0[5], aa, 10240); X4_RD(B0[5], ab, 10240); break;
            case 6: X4_RD(A0[6], aa, 12288); X4_RD(B0[6], ab, 12288); break;
            default: X4_RD(A0[7], aa, 14336); X4_RD(B0[7], ab, 14336); break;
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          mfma_a(acc[i][j], B1[j], A1[i]);
#if defined(__HIP_DEVICE_COMPILE__)
          if (dm && (j & 3) == 3) {  // 2 per row i: A instructions in rows 0-3, B in rows 4-7
            const int q = 2 * i + (j >> 2);
            if (q < X4_NI) x4_dma1(ga, na, lda * 2, st, w, va, q);
            else x4_dma1(gb, nb, ldb * 2, st + X4_OPB, w, vb, q - X4_NI);
          }
#endif
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
#undef X4_READ_ALL
#undef X4_RD

  // epilogue: lane holds D[n = 16 j + 4 hi + r][m = 16 i + lo]
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 7" ::: "memory");
  if (tr && threadIdx.x == 0) tr[2] = __builtin_amdgcn_s_memrealtime();
  const int mb = r0 + 128 * wm, nb = c0 + 128 * wn;
  if (SPREAD && c_dt != F32 && (N & 7) == 0 && (ldc & 7) == 0) {
    // 16-bit C through LDS: each wave packs its 128 x 128 tile into its own 32 KiB of the (now idle)
    // staging ring as 256-B rows, then stores whole rows 16 B per lane (4 rows = 8 full 128-B lines
    // per instruction).  Writing the fragments straight out (8 B per lane, 32-B pieces of 16 rows per
    // instruction) measured 15-16 us per 256 x 256 tile — as long as a K = 768 main loop.
    // Row m_l's 16-B chunk c sits at slot c ^ (m_l & 15): the 16 rows a ds_write_b64 covers land in
    // 16 different slots.
    __builtin_amdgcn_s_barrier();  // every wave is done reading the last k-tile's stage
    asm volatile("" ::: "memory");
    char* const wb = smem + w * 32768;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = nb + 16 * j + 4 * hi;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bias && n < N) bv = *(const float4*)(bias + n);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int ml = 16 * i + lo;
        const int slot = (2 * j + (hi >> 1)) ^ lo;
        *(uint2*)(wb + ml * 256 + slot * 16 + (hi & 1) * 8) =
            make_uint2(pack16(acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, c_dt),
                       pack16(acc[i][j][2] + bv.z, acc[i][j][3] + bv.w, c_dt));
      }
    }
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // own rows only: no barrier needed
    asm volatile("" ::: "memory");
    const int rl = lane >> 4, cc = lane & 15;
    const int n = nb + 8 * cc;
    if (ep.kind == X4_NONE) {
#pragma unroll 8
      for (int q = 0; q < 32; ++q) {
        const int ml = 4 * q + rl;
        const uint4 v = *(const uint4*)(wb + ml * 256 + ((cc ^ (ml & 15)) * 16));
        const int m = mb + ml;
        if (m < M && n < N) *(uint4*)((uint16_t*)C + (int64_t)m * ldc + n) = v;
      }
    } else if (ep.kind == X4_GELU) {
#pragma unroll 4
      for (int q = 0; q < 32; ++q) {
        const int ml = 4 * q + rl;
        const uint4 v = *(const uint4*)(wb + ml * 256 + ((cc ^ (ml & 15)) * 16));
        const int m = mb + ml;
        if (m < M && n < N) {
          const int64_t off = (int64_t)m * ldc + n;
          if (ep.c_pre) *(uint4*)((uint16_t*)ep.c_pre + off) = v;
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = pack16(gelu_f(lo16(w[e], c_dt)), gelu_f(hi16(w[e], c_dt)), c_dt);
          *(uint4*)((uint16_t*)C + off) = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
    } else {  // X4_MULGELU
      float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int q = 0; q < 32; ++q) {
        const int ml = 4 * q + rl;
        const int m = mb + ml;
        const bool ok = m < M && n < N;
        const int64_t off = (int64_t)(ok ? m : 0) * ldc + (ok ? n : 0);
        const uint4 z = *(const uint4*)(ep.aux + off);  // (any in-range row when !ok: never used)
        const uint4 v = *(const uint4*)(wb + ml * 256 + ((cc ^ (ml & 15)) * 16));
        const uint32_t w[4] = {v.x, v.y, v.z, v.w}, zw[4] = {z.x, z.y, z.z, z.w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d0 = lo16(w[e], c_dt) * gelu_grad(lo16(zw[e], c_dt));
          const float d1 = hi16(w[e], c_dt) * gelu_grad(hi16(zw[e], c_dt));
          cs[2 * e] += ok ? d0 : 0.f;
          cs[2 * e + 1] += ok ? d1 : 0.f;
          o[e] = pack16(d0, d1, c_dt);
        }
        if (ok) *(uint4*)((uint16_t*)C + off) = make_uint4(o[0], o[1], o[2], o[3]);
      }
      if (ep.colsum) {  // the 4 lanes of a column group (rl = 0..3): one atomic per column per wave
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          cs[e] += __shfl_xor(cs[e], 16, 64);
          cs[e] += __shfl_xor(cs[e], 32, 64);
        }
        if (rl == 0 && n < N) {
#pragma unroll
          for (int e = 0; e < 8; ++e) atomicAdd(ep.colsum + n + e, cs[e]);
        }
      }
    }
  } else {
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
  if (tr && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr[3] = __builtin_amdgcn_s_memrealtime();
    tr[4] = (uint64_t)tile;
  }
}

// Variant R: the same 4-wave 256x256 tile on 32-deep k-units in a 4-slot LDS ring (4 x 32 KiB):
// per unit u (64 MFMAs per wave): wait for unit u+1 (units u+2, u+3 stay in flight: vmcnt(16)),
// ONE barrier, DMA of unit u+4 into unit u's slot, then the MFMAs on u's registers interleaved
// with the fragment reads of u+1.  Three units (~3k MFMA cycles, 96 KiB in flight) hide each DMA
// instead of one 64-deep tile (~2k, 64 KiB), at one barrier per 64 MFMAs.  Image rows are 64 B, chunk c of row r at
// c ^ rswz<32>(r) (mgemm_core.h; conflict-free ds_read_b128).
constexpr int XR_BK = 32, XR_ROWB = 64, XR_OPB = 256 * XR_ROWB, XR_SLOT = 2 * XR_OPB, XR_NS = 4;

#if defined(__HIP_DEVICE_COMPILE__)
// 16 rows x 64 B per 1-KiB instruction; wave w stages rows 64w .. 64w+63 (4 instructions)
__device__ __forceinline__ void xr_dma(const char* base, int64_t bytes, int64_t ld2, char* lds, int w, uint32_t voff) {
  const int n = (int)(bytes < 0 ? 0 : (bytes > 0x7fffffff ? 0x7fffffff : bytes));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, n, 0x00020000);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row0 = 64 * w + 16 * i;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + row0 * XR_ROWB), 16, voff + (uint32_t)(row0 * ld2),
                                             0, 0, 0);
  }
}
#endif

__global__ void __launch_bounds__(X4_NT, 1) xgemm4r_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                           const uint16_t* __restrict__ B, int64_t ldb, void* C,
                                                           int64_t ldc, int c_dt, const float* __restrict__ bias,
                                                           int M, int N, int K, int dbg) {
  __shared__ __attribute__((aligned(1024))) char smem[XR_NS * XR_SLOT];
  const int tiles_n = (N + X4_BN - 1) / X4_BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  if (dbg & 8) { tm = tile / tiles_n; tn = tile % tiles_n; }  // row-major walk (diagnostics)
  else grouped_tile(tile, (M + X4_BM - 1) / X4_BM, tiles_n, 4, tm, tn);
  const int r0 = tm * X4_BM, c0 = tn * X4_BN;
  const int lane = threadIdx.x & 63, lo = lane & 15, hi = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int U = K / XR_BK;

  // DMA lane pattern: image row (lane >> 2) of the 16-row piece, chunk (lane & 3) holds source
  // chunk (lane & 3) ^ rswz<32>(row); rswz reads row bits 2..3 = lane bits 4..5: one pattern
  const int prow = lane >> 2;
  const uint32_t va = (uint32_t)(prow * lda * 2 + (((lane & 3) ^ rswz<32>(prow)) * 16));
  const uint32_t vb = (uint32_t)(prow * ldb * 2 + (((lane & 3) ^ rswz<32>(prow)) * 16));
  const char* abase = (const char*)A + (int64_t)r0 * lda * 2;
  const char* bbase = (const char*)B + (int64_t)c0 * ldb * 2;
  const int64_t abytes = ((int64_t)M - r0) * lda * 2, bbytes = ((int64_t)N - c0) * ldb * 2;
  auto dma = [&](int u) {
#if defined(__HIP_DEVICE_COMPILE__)
    char* st = smem + (u & (XR_NS - 1)) * XR_SLOT;
    xr_dma(abase + u * XR_ROWB, abytes - u * XR_ROWB, lda * 2, st, w, va);
    xr_dma(bbase + u * XR_ROWB, bbytes - u * XR_ROWB, ldb * 2, st + XR_OPB, w, vb);
#endif
  };
  // fragment i: image row 128 wm + 16 i + lo (rows 16 apart: immediate offsets of i * 1024)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const lds_void*)smem;
  const uint32_t ch = (uint32_t)((hi ^ rswz<32>(lo)) * 16);
  const uint32_t arow = lds0 + (uint32_t)((128 * wm + lo) * XR_ROWB) + ch;
  const uint32_t brow = lds0 + (uint32_t)(XR_OPB + (128 * wn + lo) * XR_ROWB) + ch;
#define XR_RD(dst, a, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(a), "i"(off))
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto rd_pair = [&](bf16x8 (&Na)[8], bf16x8 (&Nb)[8], uint32_t aa, uint32_t ab, int i) {
    switch (i) {
      case 0: XR_RD(Na[0], aa, 0); XR_RD(Nb[0], ab, 0); break;
      case 1: XR_RD(Na[1], aa, 1024); XR_RD(Nb[1], ab, 1024); break;
      case 2: XR_RD(Na[2], aa, 2048); XR_RD(Nb[2], ab, 2048); break;
      case 3: XR_RD(Na[3], aa, 3072); XR_RD(Nb[3], ab, 3072); break;
      case 4: XR_RD(Na[4], aa, 4096); XR_RD(Nb[4], ab, 4096); break;
      case 5: XR_RD(Na[5], aa, 5120); XR_RD(Nb[5], ab, 5120); break;
      case 6: XR_RD(Na[6], aa, 6144); XR_RD(Nb[6], ab, 6144); break;
      default: XR_RD(Na[7], aa, 7168); XR_RD(Nb[7], ab, 7168); break;
    }
  };
  auto mma = [&](const bf16x8 (&Ra)[8], const bf16x8 (&Rb)[8], bool rd, bf16x8 (&Na)[8], bf16x8 (&Nb)[8],
                 uint32_t aa, uint32_t ab) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (rd) rd_pair(Na, Nb, aa, ab, i);
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma_a(acc[i][j], Rb[j], Ra[i]);
    }
  };
  auto slot = [&](int u) { return (uint32_t)((u & (XR_NS - 1)) * XR_SLOT); };
  constexpr int kWaitLgkm0 = 0xC07F;
  bf16x8 A0[8], B0[8], A1[8], B1[8];
  if (U > 0) {
#pragma unroll
    for (int u = 0; u < XR_NS; ++u)
      if (u < U) dma(u);
    // unit 0 landed (units 1..3 may be in flight: 8 instructions each)
    if (U >= 4) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (U == 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (U == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) rd_pair(A0, B0, arow + slot(0), brow + slot(0), i);
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
  }
  // one unit: [wait unit u+1 (u+2, u+3 in flight) + barrier] -> DMA u+4 into u's slot (u's
  // fragments are already in registers: every wave finished reading the slot before this
  // barrier) -> MFMAs(u) || reads(u+1).  DMA(u+4) is waited for at the top of unit u+3.
#define XR_UNIT(u, CA, CB, NA, NB)                                                          \
  do {                                                                                      \
    const int u_ = (u);                                                                     \
    if (u_ + 3 < U) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");                       \
    else if (u_ + 2 < U) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                  \
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                   \
    if (!(dbg & 2)) __builtin_amdgcn_s_barrier();                                           \
    asm volatile("" ::: "memory");                                                          \
    if (u_ + 4 < U && !(dbg & 1)) dma(u_ + 4);                                              \
    __builtin_amdgcn_s_setprio(1);                                                          \
    mma(CA, CB, u_ + 1 < U, NA, NB, arow + slot(u_ + 1), brow + slot(u_ + 1));              \
    __builtin_amdgcn_s_setprio(0);                                                          \
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);                                                 \
  } while (0)
  int u = 0;
  for (; u + 1 < U; u += 2) {
    XR_UNIT(u, A0, B0, A1, B1);
    XR_UNIT(u + 1, A1, B1, A0, B0);
  }
  if (u < U) XR_UNIT(u, A0, B0, A1, B1);
#undef XR_UNIT
#undef XR_RD

  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 7" ::: "memory");
  const int mb = r0 + 128 * wm, nb = c0 + 128 * wn;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = nb + 16 * j + 4 * hi;
    const bool nok = n < N;
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

// Variant P: variant R made persistent (grid = one block per CU; block b walks tiles pos, pos + G,
// ... in the grouped order) with ONE unit stream across its tiles: the DMAs of the next tile's
// first units are in flight while the current tile's last units and its epilogue run, so there is
// no pipeline fill or drain per tile (ViT's K = 768 products are only 24 units deep).  The
// epilogue's stores join the vmcnt queue; the first wait after it allows for them.
__global__ void __launch_bounds__(X4_NT, 1) xgemm4p_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                           const uint16_t* __restrict__ B, int64_t ldb, void* C,
                                                           int64_t ldc, int c_dt, const float* __restrict__ bias,
                                                           int M, int N, int K, int dbg) {
  __shared__ __attribute__((aligned(1024))) char smem[XR_NS * XR_SLOT];
  const int tiles_m = (M + X4_BM - 1) / X4_BM, tiles_n = (N + X4_BN - 1) / X4_BN;
  const int total = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int pos = xcd_remap(blockIdx.x, G);
  const int my = pos < total ? (total - pos + G - 1) / G : 0;
  const int U = K / XR_BK;
  const int S = my * U;  // units in this block's stream
  const int lane = threadIdx.x & 63, lo = lane & 15, hi = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;

  const int prow = lane >> 2;
  const uint32_t va = (uint32_t)(prow * lda * 2 + (((lane & 3) ^ rswz<32>(prow)) * 16));
  const uint32_t vb = (uint32_t)(prow * ldb * 2 + (((lane & 3) ^ rswz<32>(prow)) * 16));
  // issue cursor (tile of the next DMA, its unit) and compute cursor (tile being multiplied)
  int iss_i = 0, iss_u = 0;
  const char *ia = nullptr, *ib = nullptr;
  int64_t ia_n = 0, ib_n = 0;
  auto iss_tile = [&](int i) {
    int tm, tn;
    grouped_tile(pos + i * G, tiles_m, tiles_n, 4, tm, tn);
    ia = (const char*)A + (int64_t)tm * X4_BM * lda * 2;
    ib = (const char*)B + (int64_t)tn * X4_BN * ldb * 2;
    ia_n = ((int64_t)M - tm * X4_BM) * lda * 2;
    ib_n = ((int64_t)N - tn * X4_BN) * ldb * 2;
  };
  if (my > 0) iss_tile(0);
  auto dma_next = [&](int q) {  // global unit q of the stream
#if defined(__HIP_DEVICE_COMPILE__)
    char* st = smem + (q & (XR_NS - 1)) * XR_SLOT;
    if (!(dbg & 1)) {
      xr_dma(ia + iss_u * XR_ROWB, ia_n - iss_u * XR_ROWB, lda * 2, st, w, va);
      xr_dma(ib + iss_u * XR_ROWB, ib_n - iss_u * XR_ROWB, ldb * 2, st + XR_OPB, w, vb);
    }
#endif
    if (++iss_u == U) {
      iss_u = 0;
      if (++iss_i < my) iss_tile(iss_i);
    }
  };
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const lds_void*)smem;
  const uint32_t ch = (uint32_t)((hi ^ rswz<32>(lo)) * 16);
  const uint32_t arow = lds0 + (uint32_t)((128 * wm + lo) * XR_ROWB) + ch;
  const uint32_t brow = lds0 + (uint32_t)(XR_OPB + (128 * wn + lo) * XR_ROWB) + ch;
#define XP_RD(dst, a, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(a), "i"(off))
  // accumulators: defined by the first unit of every tile (MFMAs with C = 0), so the epilogue
  // never writes them (a zeroing assignment inside the persistent loop made the allocator move them
  // out of the accumulator registers: hundreds of spills)
  f32x4 acc[8][8];
  auto rd_pair = [&](bf16x8 (&Na)[8], bf16x8 (&Nb)[8], uint32_t aa, uint32_t ab, int i) {
    switch (i) {
      case 0: XP_RD(Na[0], aa, 0); XP_RD(Nb[0], ab, 0); break;
      case 1: XP_RD(Na[1], aa, 1024); XP_RD(Nb[1], ab, 1024); break;
      case 2: XP_RD(Na[2], aa, 2048); XP_RD(Nb[2], ab, 2048); break;
      case 3: XP_RD(Na[3], aa, 3072); XP_RD(Nb[3], ab, 3072); break;
      case 4: XP_RD(Na[4], aa, 4096); XP_RD(Nb[4], ab, 4096); break;
      case 5: XP_RD(Na[5], aa, 5120); XP_RD(Nb[5], ab, 5120); break;
      case 6: XP_RD(Na[6], aa, 6144); XP_RD(Nb[6], ab, 6144); break;
      default: XP_RD(Na[7], aa, 7168); XP_RD(Nb[7], ab, 7168); break;
    }
  };
  // the next unit's 16 fragment reads go out first (asm: the compiler adds no waits; they land
  // under the 64 MFMAs), then the MFMAs, starting a tile's accumulation with C = 0 in its first unit
  auto mma = [&](const bf16x8 (&Ra)[8], const bf16x8 (&Rb)[8], bool rd, bf16x8 (&Na)[8], bf16x8 (&Nb)[8],
                 uint32_t aa, uint32_t ab, bool first) {
    if (rd) {
#pragma unroll
      for (int i = 0; i < 8; ++i) rd_pair(Na, Nb, aa, ab, i);
    }
    if (first) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) mfma_a0(acc[i][j], Rb[j], Ra[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) mfma_a(acc[i][j], Rb[j], Ra[i]);
    }
  };
  auto slot = [&](int q) { return (uint32_t)((q & (XR_NS - 1)) * XR_SLOT); };
  constexpr int kWaitLgkm0 = 0xC07F;
  int cur_i = 0;
  auto epilogue = [&]() {
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 7" ::: "memory");
    int tm, tn;
    grouped_tile(pos + cur_i * G, tiles_m, tiles_n, 4, tm, tn);
    const int mb = tm * X4_BM + 128 * wm, nb = tn * X4_BN + 128 * wn;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = nb + 16 * j + 4 * hi;
      const bool nok = n < N;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bias && nok) bv = *(const float4*)(bias + n);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = mb + 16 * i + lo;
        const float v0 = acc[i][j][0] + bv.x, v1 = acc[i][j][1] + bv.y, v2 = acc[i][j][2] + bv.z,
                    v3 = acc[i][j][3] + bv.w;
        if (!nok || m >= M) continue;
        *(uint2*)((uint16_t*)C + (int64_t)m * ldc + n) = make_uint2(pack16(v0, v1, c_dt), pack16(v2, v3, c_dt));
      }
      // one column of fragments at a time: the accumulator reads of the next column are not
      // hoisted (the next tile's first fragments are live in arch VGPRs meanwhile)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  bf16x8 A0[8], B0[8], A1[8], B1[8];
  if (S > 0) {
#pragma unroll
    for (int q = 0; q < XR_NS; ++q)
      if (q < S) dma_next(q);
    if (S >= 4) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (S == 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (S == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) rd_pair(A0, B0, arow + slot(0), brow + slot(0), i);
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
  }
  // after an epilogue its (many) stores sit behind the DMAs in the vmcnt queue: the first wait
  // then saturates at 63 (it may also wait for a few of the oldest stores)
  bool after_epi = false;
#define XP_UNIT(q, u, CA, CB, NA, NB, EPI)                                                 \
  do {                                                                                     \
    const int q_ = (q);                                                                    \
    if (after_epi) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");                       \
    if (q_ + 3 < S) { if (!after_epi) asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); } \
    else if (q_ + 2 < S) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                 \
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                  \
    after_epi = false;                                                                     \
    if (!(dbg & 2)) __builtin_amdgcn_s_barrier();                                          \
    asm volatile("" ::: "memory");                                                         \
    if (q_ + 4 < S) dma_next(q_ + 4);                                                      \
    __builtin_amdgcn_s_setprio(1);                                                         \
    mma(CA, CB, q_ + 1 < S, NA, NB, arow + slot(q_ + 1), brow + slot(q_ + 1), (u) == 0);   \
    __builtin_amdgcn_s_setprio(0);                                                         \
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);                                                \
    if (EPI && (u) == U - 1) {                                                             \
      epilogue();                                                                          \
      ++cur_i;                                                                             \
      after_epi = true;                                                                    \
    }                                                                                      \
  } while (0)
  // U is even for every supported K (K % 64 == 0): units pair up inside a tile
  for (int q = 0; q < S; q += 2) {
    const int u = q % U;
    XP_UNIT(q, u, A0, B0, A1, B1, false);  // u is even: never a tile's last unit
    XP_UNIT(q + 1, u + 1, A1, B1, A0, B0, true);
  }
#undef XP_UNIT
#undef XP_RD
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

// C[M][N] = A[M][K] B[N][K]^T (+ bias[N]); bf16 operands (rows 16-byte aligned), K % 64 == 0,
// N % 4 == 0; C f32 / bf16 / fp16 (c_dt).
int g_x4_dbg = 0;
uint64_t* g_x4_trace = nullptr;
RK_API int rk_xgemm4_set_trace(void* tr) {  // diagnostics: per-block phase stamps [blocks][8] (or null)
  g_x4_trace = (uint64_t*)tr;
  return 0;
}
RK_API int rk_xgemm4_set_dbg(int bits) {  // diagnostics: bit 0 no in-loop DMA, bit 1 no barrier, bit 5 spread DMA
  g_x4_dbg = bits;
  return 0;
}
static int xgemm4_launch(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int c_dt,
                         const float* bias, int M, int N, int K, X4Epi ep, hipStream_t s);

RK_API int rk_xgemm4(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int c_dt,
                     const float* bias, int M, int N, int K, hipStream_t s) {
  return xgemm4_launch(a, lda, b, ldb, c, ldc, c_dt, bias, M, N, K, X4Epi{nullptr, nullptr, nullptr, X4_NONE}, s);
}

// C[M][N] = epi(A[M][K] B[N][K]^T + bias) on the spread-DMA 256x256 kernel with the LDS-staged epilogue
// (16-bit C, N % 8 == 0, ldc % 8 == 0): epi 0 none, 1 GELU (c_pre = pre-activation, may be null),
// 2 multiply by gelu'(aux) (+ colsum[n] += column sums of the f32 product, colsum may be null).
RK_API int rk_xgemm4_epi(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int c_dt,
                         const float* bias, void* c_pre, const void* aux, float* colsum, int epi, int M, int N, int K,
                         hipStream_t s) {
  if (c_dt == F32 || N % 8 || ldc % 8 || epi < 0 || epi > 2 || (epi == X4_MULGELU && !aux)) return (int)hipErrorInvalidValue;
  const int saved = g_x4_dbg;
  g_x4_dbg = 32;  // the spread schedule (the fused epilogues live in its LDS-staged store path)
  const int rc = xgemm4_launch(a, lda, b, ldb, c, ldc, c_dt, bias, M, N, K,
                               X4Epi{c_pre, (const uint16_t*)aux, colsum, epi}, s);
  g_x4_dbg = saved;
  return rc;
}

static int xgemm4_launch(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int c_dt,
                         const float* bias, int M, int N, int K, X4Epi ep, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % X4_BK || N % 4 || ((uintptr_t)a | (uintptr_t)b) % 16 || (lda * 2) % 16 || (ldb * 2) % 16)
    return (int)hipErrorInvalidValue;
  // per-lane + per-instruction DMA offsets stay below 2^31 (256 rows of the operand)
  if ((int64_t)256 * lda * 2 >= (1ll << 31) || (int64_t)256 * ldb * 2 >= (1ll << 31)) return (int)hipErrorInvalidValue;
  const int tiles = ((M + X4_BM - 1) / X4_BM) * ((N + X4_BN - 1) / X4_BN);
  if (g_x4_dbg & 16) {  // variant P (persistent R): one block per CU
    static int ncu = 0;
    if (ncu <= 0) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    }
    xgemm4p_kernel<<<std::min(tiles, ncu), X4_NT, 0, s>>>((const uint16_t*)a, lda, (const uint16_t*)b, ldb, c, ldc,
                                                          c_dt, bias, M, N, K, g_x4_dbg);
    return (int)hipGetLastError();
  }
  if (g_x4_dbg & 4) {  // variant R (32-deep units, 4-slot ring); K % 32 suffices
    xgemm4r_kernel<<<tiles, X4_NT, 0, s>>>((const uint16_t*)a, lda, (const uint16_t*)b, ldb, c, ldc, c_dt, bias, M, N,
                                           K, g_x4_dbg);
    return (int)hipGetLastError();
  }
  if (g_x4_dbg & 32)
    xgemm4_kernel<true><<<tiles, X4_NT, 0, s>>>((const uint16_t*)a, lda, (const uint16_t*)b, ldb, c, ldc, c_dt, bias, M,
                                                N, K, g_x4_dbg, g_x4_trace, ep);
  else
    xgemm4_kernel<false><<<tiles, X4_NT, 0, s>>>((const uint16_t*)a, lda, (const uint16_t*)b, ldb, c, ldc, c_dt, bias, M,
                                                 N, K, g_x4_dbg, g_x4_trace, ep);
  return (int)hipGetLastError();
}

// 16-bit transpose dst[c][r] = src[r][c] (rows x cols, both dense): the transformer MLP's input-gradient
// GEMM reads fc2's weight as the forward layout's B operand (K contiguous) from this copy.  64 x 64
// tiles through LDS (row pitch 66 elements: the column reads hit 32 distinct banks), 16-byte global
// reads, 4-byte global writes of row-contiguous pairs.
namespace {
__global__ void __launch_bounds__(256) transpose16_kernel(const uint16_t* __restrict__ src, int rows, int cols,
                                                          uint16_t* __restrict__ dst) {
  __shared__ uint16_t t[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  // load: 64 rows x 8 chunks of 8 elements; thread -> (row tid / 8 + 32 k, chunk tid % 8)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int r = threadIdx.x / 8 + 32 * k, ch = threadIdx.x % 8;
    const int gr = r0 + r, gc = c0 + 8 * ch;
    uint16_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (gr < rows && gc + 8 <= cols) {
      const uint4 q = *(const uint4*)(src + (int64_t)gr * cols + gc);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = (uint16_t)(w[e] & 0xffff);
        v[2 * e + 1] = (uint16_t)(w[e] >> 16);
      }
    } else if (gr < rows) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (gc + e < cols) v[e] = src[(int64_t)gr * cols + gc + e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) t[r][8 * ch + e] = v[e];
  }
  __syncthreads();
  // store: dst row (c0 + c) holds src rows r0 .. r0+63 of column c; thread -> (c = tid / 4 .. , pair)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = threadIdx.x / 32 + 8 * k, rp = threadIdx.x % 32;  // rows 2 rp, 2 rp + 1
    const int gc = c0 + c, gr = r0 + 2 * rp;
    if (gc >= cols) continue;
    if (gr + 1 < rows) {
      *(uint32_t*)(dst + (int64_t)gc * rows + gr) = (uint32_t)t[2 * rp][c] | ((uint32_t)t[2 * rp + 1][c] << 16);
    } else if (gr < rows) {
      dst[(int64_t)gc * rows + gr] = t[2 * rp][c];
    }
  }
}
}  // namespace

RK_API int rk_transpose16(const void* src, int rows, int cols, void* dst, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return 0;
  if (((uintptr_t)src | (uintptr_t)dst) & 15 || cols % 8 || rows % 2) return (int)hipErrorInvalidValue;
  const dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  transpose16_kernel<<<grid, 256, 0, s>>>((const uint16_t*)src, rows, cols, (uint16_t*)dst);
  return (int)hipGetLastError();
}
