// Shared device pieces of the MFMA GEMM family (mgemm.hip: dense GEMMs; conv.hip: implicit-GEMM
// convolutions): LDS-DMA stagers with source-side swizzles, fragment readers (ds_read_b128 /
// ds_read_b64_tr_b16), counted vmcnt waits and the fused epilogue.  Layout and swizzle rules:
// header comment of mgemm.hip.  Everything is in an anonymous namespace (one copy per TU).
#pragma once
#include "rk_common.h"

#include <algorithm>

namespace {

using namespace rk;


typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

enum Epi : int { kNone = 0, kRelu = 1, kGelu = 2, kMulGeluGrad = 3, kMulReluGrad = 4 };

struct MArgs {
  const uint16_t* a;
  const uint16_t* b;
  void* c;
  void* c_pre;           // kGelu: pre-activation out (bf16/f32 like C), optional
  const float* bias;     // [N] or null
  const uint16_t* aux;   // kMulGeluGrad / kMulReluGrad: bf16 [M][ldc]
  float* rowsum;         // [M] f32 += row sums of A, or null
  float* slab;           // split-K partial tiles [splitk][M][N] f32 (reduced by mgemm_reduce), or null
  int64_t lda, ldb, ldc;
  int M, N, K;
  int c_dt;
  int epi;
  int accumulate;
  int splitk, k_per_split;
  int lds_epi;  // conv.hip: bf16 tile stored through LDS in row-contiguous 16-byte chunks
  int tgroup;   // grouped tile walk (rk_common.h grouped_tile): tile-rows per group, <= 1 row-major
  int dbg;      // xgemm.hip diagnostics (rk_xgemm_set_dbg): bit 0 no DMA, 1 no barrier, 2 no ds_read, 3 no MFMA
};

// kmaj image slot swizzle (see header)
// R >= 128 columns (>= 16 slots per k-row): slot ^= ((k & 3) | ((k >> 1) & 4)) << 1 (even, < 16);
// R = 64 (128-byte k-rows, two per bank row): slot ^= (k & 2) | ((k >> 1) & 4) (even, < 8) -- the
// 16 (row, chunk) pairs of a 32-lane transposed read then land on 16 distinct bank slots either way.
template <int R>
__device__ __forceinline__ int kswz(int k) {
  if constexpr (R >= 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
  else return (k & 2) | ((k >> 1) & 4);
}
// row image slot swizzle: BK = 64 (128-B rows, 8 slots) / BK = 32 (64-B rows, 4 slots)
template <int BK>
__device__ __forceinline__ int rswz(int r) {
  if constexpr (BK == 64) return (r >> 1) & 7;
  else return (0x78 >> (2 * ((r >> 2) & 3))) & 3;  // [0, 2, 3, 1][(r >> 2) & 3]
}

// LDS-DMA of one operand's k-tile: R rows x BK (row image) or BK rows x R (kmaj image);
// R*BK*2 bytes = NI wave instructions of 1 KiB per wave.  Every per-lane source offset is computed
// once: per k-tile only the wave-uniform base moves (SGPR base + VGPR offset addressing).
template <int R, int BK, bool KMAJ, int NW>
struct Stager {
  static constexpr int NI = R * BK / (512 * NW);
  static_assert(NI >= 1 && R * BK % (512 * NW) == 0, "tile too small for the wave count");
  uint32_t off[NI];  // byte offsets from the k-tile base
  __device__ __forceinline__ void init(int64_t ld, int r0, int rdim, int wid, int lane) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (wid * NI + i) * 64 + lane;  // 16-byte chunk index in the lane-linear image
      if constexpr (!KMAJ) {
        constexpr int CPR = BK / 8;
        const int r = q / CPR, c = q % CPR;
        const int chunk = c ^ rswz<BK>(r);
        const int gr = min(r0 + r, rdim - 1);  // rows past the edge: any valid row (never stored)
        off[i] = (uint32_t)(((int64_t)gr * ld + chunk * 8) * 2);
      } else {
        constexpr int CPR = R / 8;  // chunks per k-row
        const int k = q / CPR, c = q % CPR;
        const int chunk = c ^ kswz<R>(k);
        const int gc = min(r0 + chunk * 8, rdim - 8);
        off[i] = (uint32_t)(((int64_t)k * ld + gc) * 2);
      }
    }
  }
  // base: wave-uniform address of element (row 0, k0) [row] / (k0, col 0) [kmaj]
  __device__ __forceinline__ void issue(const char* base, char* lds, int wid) const {
#pragma unroll
    for (int i = 0; i < NI; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(base + off[i]), (lds_void*)(lds + (wid * NI + i) * 1024), 16, 0,
                                       0);
  }
  // the partial last k-tile (kvalid < BK valid k): chunks past K are DMA'd from a zero page, so
  // the MFMAs over the whole tile add exact zeros
  __device__ __forceinline__ void issue_tail(const char* base, char* lds, int wid, int lane, int kvalid,
                                             const char* zero) const {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (wid * NI + i) * 64 + lane;
      int kpos;
      if constexpr (!KMAJ) {
        constexpr int CPR = BK / 8;
        kpos = ((q % CPR) ^ rswz<BK>(q / CPR)) * 8;
      } else {
        kpos = q / (R / 8);
      }
      const char* src = kpos < kvalid ? base + off[i] : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (wid * NI + i) * 1024), 16, 0, 0);
    }
  }
};

__device__ __attribute__((aligned(16))) uint4 g_mgemm_zero[1];  // 16 zero bytes (static storage)

// Fragment reads (16 rows x 32 k, MFMA 16x16x32 operand map) of the NF fragments a wave owns,
// rows rbase + 16*f.  Per-lane offsets are precomputed; k-step and fragment terms are immediates.
//   row image: one ds_read_b128 per fragment; the slot swizzle depends only on (lane & 15), so
//              fragment f is at +f*16 rows; one offset per k-step (the XOR flips slot bit 2).
//   kmaj image: two ds_read_b64_tr_b16 (k rows 8g+q and 8g+4+q); kswz(k) reduces to a per-lane
//              constant S (k & 3 = q, bit 3 of k = g & 1), so only the chunk term depends on f.
template <int R, int BK, bool KMAJ, int NF>
struct FragReader {
  static constexpr int KK = BK / 32;
  uint32_t off[KMAJ ? NF : KK];
  __device__ __forceinline__ void init(int rbase, int lane) {
    if constexpr (!KMAJ) {
      const int row = rbase + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) off[kk] = row * (BK * 2) + (((kk * 4 + (lane >> 4)) ^ rswz<BK>(row)) << 4);
    } else {
      const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
      const int S = kswz<R>(8 * g + q);
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int chunk = (rbase >> 3) + 2 * f + (p >> 1);
        off[f] = (8 * g + q) * (2 * R) + ((chunk ^ S) << 4) + ((p & 1) << 3);
      }
    }
  }
  __device__ __forceinline__ bf16x8 get(const char* img, int f, int kk) const {
    if constexpr (!KMAJ) {
      return *(const bf16x8*)(img + off[kk] + f * 16 * (BK * 2));
    } else {
      const char* p0 = img + off[f] + kk * 32 * (2 * R);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 4 * (2 * R)));
      typedef __attribute__((ext_vector_type(8))) short s16x8;
      const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

// s_waitcnt vmcnt(n) for a run-time n (the field is an immediate)
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Epilogue of one wave's FM x FN fragments: lane holds C[m][n..n+3], m = mbase + 16 i + (lane & 15),
// n = nbase + 16 j + 4 (lane >> 4).  PRE: the side inputs (aux / old bf16 C) were loaded before the
// main loop into `side`; otherwise they are loaded here.
struct IdRow {  // GEMM row m is output row m
  __device__ __forceinline__ int64_t operator()(int m) const { return m; }
};

template <int FM, int FN, bool PRE, typename RowMap = IdRow>
__device__ __forceinline__ void store_tile(const MArgs& g, f32x4 (&acc)[FM][FN], const uint2 (&side)[FM][FN],
                                           int mbase, int nbase, int lane, int split, const RowMap& rowmap = RowMap()) {
  if (g.splitk > 1) {  // partial tile -> this split's slab (plain stores; mgemm_reduce combines)
    float* slab = g.slab + (int64_t)split * g.M * g.N;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nbase + j * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = mbase + i * 16 + (lane & 15);
        if (m < g.M) *(float4*)(slab + (int64_t)m * g.N + n) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }
  // all side inputs were loaded before the main loop (aux / old C); compute, then store
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = nbase + j * 16 + 4 * (lane >> 4);
    const bool nok = n < g.N;  // N % 4 == 0 (host-checked): a lane's 4 columns are all in or all out
    float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.bias && nok) bias = *(const float4*)(g.bias + n);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = mbase + i * 16 + (lane & 15);
      if (!nok || m >= g.M) continue;
      const int64_t off = rowmap(m) * g.ldc + n;
      float v[4] = {acc[i][j][0] + bias.x, acc[i][j][1] + bias.y, acc[i][j][2] + bias.z, acc[i][j][3] + bias.w};
      if (g.epi == kGelu || g.epi == kRelu) {
        if (g.c_pre) {
          if (g.c_dt != F32)
            *(uint2*)((uint16_t*)g.c_pre + off) = make_uint2(pack16(v[0], v[1], g.c_dt), pack16(v[2], v[3], g.c_dt));
          else
            *(float4*)((float*)g.c_pre + off) = make_float4(v[0], v[1], v[2], v[3]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = g.epi == kGelu ? gelu_f(v[e]) : fmaxf(v[e], 0.f);
      } else if (g.epi == kMulGeluGrad || g.epi == kMulReluGrad) {
        const uint2 z = PRE ? side[i][j] : *(const uint2*)(g.aux + off);
        const int adt = g.c_dt == F16 ? F16 : BF16;  // aux is 16-bit, same format as a 16-bit C
        const float zz[4] = {lo16(z.x, adt), hi16(z.x, adt), lo16(z.y, adt), hi16(z.y, adt)};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = g.epi == kMulGeluGrad ? v[e] * gelu_grad(zz[e]) : (zz[e] > 0.f ? v[e] : 0.f);
      }
      if (g.c_dt != F32) {
        uint16_t* c = (uint16_t*)g.c + off;
        if (g.accumulate) {
          const uint2 o = PRE ? side[i][j] : *(const uint2*)c;
          v[0] += lo16(o.x, g.c_dt);
          v[1] += hi16(o.x, g.c_dt);
          v[2] += lo16(o.y, g.c_dt);
          v[3] += hi16(o.y, g.c_dt);
        }
        *(uint2*)c = make_uint2(pack16(v[0], v[1], g.c_dt), pack16(v[2], v[3], g.c_dt));
      } else {
        float* c = (float*)g.c + off;
        if (g.accumulate) {
          const float4 o = *(const float4*)c;
          v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
        }
        *(float4*)c = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// C[m][n] (+)= sum_s slab[s][m][n] + bias[n]  (f32, bf16 or f16 C; N % 4 == 0).  G consecutive lanes share
// one output float4, lane g summing the slabs s = g, g + G, ... (four loads in flight), combined by
// xor-shuffles: small outputs with many splits (ResNet wgrads: 9k float4 x 32 splits) get G-fold more
// loads in flight instead of a long serial slab loop per thread.  Fixed order: deterministic.
// block `bid` of `nb` blocks (`nt` threads each) of the combine: mgemm_reduce's body, also run by
// extra blocks appended to a later launch (conv.hip: the tail-reduce job of a stride-1 dgrad)
template <int G>
__device__ __forceinline__ void reduce_slabs(const float* __restrict__ slab, int splitk, int M, int N,
                                             const float* __restrict__ bias, void* c, int c_dt, int64_t ldc,
                                             int accumulate, int bid, int nb, int nt) {
  const int64_t nq = (int64_t)M * N / 4;
  const int64_t plane = (int64_t)M * N;
  const int g = (int)(threadIdx.x % G);
  for (int64_t q = ((int64_t)bid * nt + threadIdx.x) / G; q < nq; q += (int64_t)nb * (nt / G)) {
    const int64_t e = q * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = g;
    for (; s + 3 * G < splitk; s += 4 * G) {  // four independent slab loads in flight per lane
      const float4 w0 = *(const float4*)(slab + s * plane + e);
      const float4 w1 = *(const float4*)(slab + (s + G) * plane + e);
      const float4 w2 = *(const float4*)(slab + (s + 2 * G) * plane + e);
      const float4 w3 = *(const float4*)(slab + (s + 3 * G) * plane + e);
      v.x += (w0.x + w1.x) + (w2.x + w3.x);
      v.y += (w0.y + w1.y) + (w2.y + w3.y);
      v.z += (w0.z + w1.z) + (w2.z + w3.z);
      v.w += (w0.w + w1.w) + (w2.w + w3.w);
    }
    for (; s < splitk; s += G) {
      const float4 w = *(const float4*)(slab + s * plane + e);
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
      v.x += __shfl_xor(v.x, o, 64);
      v.y += __shfl_xor(v.y, o, 64);
      v.z += __shfl_xor(v.z, o, 64);
      v.w += __shfl_xor(v.w, o, 64);
    }
    if (g != 0) continue;
    const int m = (int)(e / N), n = (int)(e % N);
    if (bias) {
      const float4 b = *(const float4*)(bias + n);
      v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    }
    const int64_t off = (int64_t)m * ldc + n;
    if (c_dt != F32) {
      uint16_t* o = (uint16_t*)c + off;
      if (accumulate) {
        const uint2 p = *(const uint2*)o;
        v.x += lo16(p.x, c_dt); v.y += hi16(p.x, c_dt);
        v.z += lo16(p.y, c_dt); v.w += hi16(p.y, c_dt);
      }
      *(uint2*)o = make_uint2(pack16(v.x, v.y, c_dt), pack16(v.z, v.w, c_dt));
    } else {
      float* o = (float*)c + off;
      if (accumulate) {
        const float4 p = *(const float4*)o;
        v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
      }
      *(float4*)o = v;
    }
  }
}

template <int G>
__global__ void __launch_bounds__(256) mgemm_reduce(const float* __restrict__ slab, int splitk, int M, int N,
                                                    const float* __restrict__ bias, void* c, int c_dt, int64_t ldc,
                                                    int accumulate) {
  reduce_slabs<G>(slab, splitk, M, N, bias, c, c_dt, ldc, accumulate, blockIdx.x, gridDim.x, 256);
}

// launch the split-K combine: 4 lanes per output float4 once there are >= 8 slabs
inline void launch_mgemm_reduce(const float* slab, int splitk, int M, int N, const float* bias, void* c, int c_dt,
                                int64_t ldc, int accumulate, hipStream_t s) {
  const int64_t nq = (int64_t)M * N / 4;
  if (splitk >= 8) {
    const int blocks = (int)std::min<int64_t>((nq * 4 + 255) / 256, 8192);
    mgemm_reduce<4><<<blocks, 256, 0, s>>>(slab, splitk, M, N, bias, c, c_dt, ldc, accumulate);
  } else {
    const int blocks = (int)std::min<int64_t>((nq + 255) / 256, 4096);
    mgemm_reduce<1><<<blocks, 256, 0, s>>>(slab, splitk, M, N, bias, c, c_dt, ldc, accumulate);
  }
}

}  // namespace
