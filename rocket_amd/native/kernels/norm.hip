// Normalisation kernels: BatchNorm over channels-last activations and LayerNorm over rows
// (the BatchNorm of ResNet-18/50 and the LayerNorm of ViT-B/16).
//
// BatchNorm (training), x viewed as [R = N*H*W][C] (channels-last, C contiguous):
//   bn_stats      grid (C/64, RB): a block reduces rows [rb*rpb, ...) x 64 channels; each thread
//                 owns 8 consecutive channels (one 16-byte load per row) and accumulates
//                 shifted sums (pivot = row 0, kills E[x^2]-E[x]^2 cancellation).  Per-block
//                 partials go to a workspace; the LAST block of each channel column (ticket)
//                 merges them, writes mean / invstd, the fused scale/shift (a = g*invstd,
//                 b = beta - mean*a) and updates the running statistics (unbiased var).
//   bn_apply      y = relu?(x*a + b + residual?), 8 channels per thread, coefficients in registers.
//   bn_bwd_reduce per channel sum(dy') and sum(dy'*xhat), dy' = dy*[y>0] when ReLU was fused;
//                 the last block writes dgamma/dbeta (accumulated into the grads) and the two
//                 per-channel coefficients of the input gradient.
//   bn_bwd_apply  dx = a*(dy' - k1 - xhat*k2) (folded to P*dy' + Q*x + S) and d(residual) = dy'.
// LayerNorm over the last dim (C <= 4096), one wave per row:
//   ln_fwd        two-pass mean/var in registers, y = xhat*g + b (bf16 or f32 out),
//                 saves mean/rstd.
//   ln_bwd        dx per row; dgamma/dbeta column partials per block, then a parallel column-sum
//                 launch accumulates them into the parameter gradients.
#include "rk_common.h"

using namespace rk;

namespace {

constexpr int BN_T = 256;        // threads per block
constexpr int BN_CT = 64;        // channels per block column
constexpr int BN_RG = BN_T / 8;  // row groups per block pass (each thread: 8 channels)
constexpr int BN_U = 4;          // rows in flight per thread per loop iteration (two-tensor passes)
constexpr int BN_US = 8;         // rows in flight per thread in the one-tensor statistics pass
constexpr int BN_GS = 16;        // row blocks per first-level finalize group
constexpr int BN_MAXRB = 2048;   // row blocks per column (upper bound)
constexpr int BN_CNT = 1 + BN_MAXRB / BN_GS;  // ticket counters per column: column + groups
constexpr int BN_ROWQ = BN_US * BN_RG;       // row-block granularity (multiple of both unrolls)
constexpr int BN_FU = 4;                     // partial-tile rows in flight per thread (finalize launches)

template <typename T> struct V8;
template <> struct V8<uint16_t> {
  static __device__ __forceinline__ void unpack(const uint4 u, float* v) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ uint4 pack(const float* v) {
    uint4 u;
    uint32_t* w = (uint32_t*)&u;
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f2bf(v[2 * k]) | ((uint32_t)f2bf(v[2 * k + 1]) << 16);
    return u;
  }
  // streaming forms (nontemporal: the elementwise BatchNorm passes touch each element once)
  static __device__ __forceinline__ void load_nt(const uint16_t* p, float* v) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 t = __builtin_nontemporal_load((const u32x4*)p);
    unpack(make_uint4(t.x, t.y, t.z, t.w), v);
  }
  static __device__ __forceinline__ void store_nt(uint16_t* p, const float* v) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const uint4 u = pack(v);
    __builtin_nontemporal_store(u32x4{u.x, u.y, u.z, u.w}, (u32x4*)p);
  }
  static __device__ __forceinline__ void load(const uint16_t* p, float* v) {
    const uint4 u = *(const uint4*)p;
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float* v) {
    uint4 u;
    uint32_t* w = (uint32_t*)&u;
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f2bf(v[2 * k]) | ((uint32_t)f2bf(v[2 * k + 1]) << 16);
    *(uint4*)p = u;
  }
};
template <> struct V8<f16_t> {
  static __device__ __forceinline__ void load(const f16_t* p, float* v) {
    const uint4 u = *(const uint4*)p;
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = h2f((uint16_t)(w[k] & 0xffffu));
      v[2 * k + 1] = h2f((uint16_t)(w[k] >> 16));
    }
  }
  static __device__ __forceinline__ void store(f16_t* p, const float* v) {
    uint4 u;
    uint32_t* w = (uint32_t*)&u;
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f2h(v[2 * k]) | ((uint32_t)f2h(v[2 * k + 1]) << 16);
    *(uint4*)p = u;
  }
};
template <> struct V8<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// elementwise-pass variant (bf16 -> bf16 only; ROCKET_BN_EW, A/B knob): bit 0 = nontemporal loads /
// stores, bit 1 = 8 rows in flight per thread instead of BN_U
template <typename T, int EV> struct BnEw {
  static constexpr bool NT = (EV & 1) && std::is_same<T, uint16_t>::value;
  static constexpr int U = (EV & 2) ? 8 : BN_U;
  static __device__ __forceinline__ void load(const T* p, float* v) {
    if constexpr (NT) V8<uint16_t>::load_nt((const uint16_t*)p, v);
    else V8<T>::load(p, v);
  }
  static __device__ __forceinline__ void store(T* p, const float* v) {
    if constexpr (NT) V8<uint16_t>::store_nt((uint16_t*)p, v);
    else V8<T>::store(p, v);
  }
};

// reduce per-thread [8] accumulators over the BN_RG row groups of the block into out[64]: the 8
// row groups of a wave (lanes sharing lane & 7) by xor-shuffles, then the BN_T / 64 wave rows
// through LDS, written as whole 32-byte channel runs (no bank conflicts; the round-2 version
// parked every thread's 8 values in a [BN_RG][65] image: 2-way conflicts on every store, 31 %
// SQ_LDS_BANK_CONFLICT on the BatchNorm reductions).  Fixed order: deterministic.
constexpr int BN_WV = BN_T / 64;  // waves per block
__device__ __forceinline__ void reduce_rowgroups(const float* v, float (*lds)[BN_CT], float* out) {
  float w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float t = v[k] + __shfl_xor(v[k], 8, 64);
    t += __shfl_xor(t, 16, 64);
    w[k] = t + __shfl_xor(t, 32, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < 8) {  // lane == channel group cg
    *(float4*)&lds[wv][lane * 8] = make_float4(w[0], w[1], w[2], w[3]);
    *(float4*)&lds[wv][lane * 8 + 4] = make_float4(w[4], w[5], w[6], w[7]);
  }
  __syncthreads();
  if (threadIdx.x < BN_CT) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < BN_WV; ++g) s += lds[g][threadIdx.x];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

// ---- two-level in-launch column reduction -------------------------------------------------
// A reduction launch has grid (C/64 column blocks, RB row blocks).  Each block stores its 64x2
// partial sums into part[b]; the last block (ticket) of every group of BN_GS row blocks sums that
// group into part2[g]; the last group of the column sums the RB/BN_GS group totals.  Both serial
// tails are short (<= 16 and <= 128 partials over 4 threads per channel), so the grid can be
// ~2048 blocks — enough bytes in flight to stream HBM — without a long single-block finalize.
// Hand-off without fences (cdna guide §6 G16 R1): partials are stored write-through (sc1, relaxed
// agent atomics), every storing wave drains vmcnt before the workgroup barrier, lane 0 takes the
// ticket, and the reducer reads EVERY partial with sc1 loads — no L2 write-back, no L1 invalidate.
// Fixed summation order: results are deterministic.  Counters self-reset (graph replays).
__device__ __forceinline__ void bn_sum_parts(const float* part, int C, int c0, int b0, int b1, float& t1,
                                             float& t2) {
  const int ch = threadIdx.x >> 2, sub = threadIdx.x & 3, cc = c0 + ch;
  float s1 = 0.f, s2 = 0.f;
  if (cc < C) {
#pragma unroll 8
    for (int b = b0 + sub; b < b1; b += 4) {
      const float* p = part + (int64_t)b * 2 * C;
      s1 += ld_sc1(p + cc);
      s2 += ld_sc1(p + C + cc);
    }
  }
  s1 += __shfl_xor(s1, 1, 64);
  s1 += __shfl_xor(s1, 2, 64);
  s2 += __shfl_xor(s2, 1, 64);
  s2 += __shfl_xor(s2, 2, 64);
  t1 = s1;
  t2 = s2;
}

// call from all threads after this block's sc1 stores; true in all threads of the block whose
// ticket completes `total`
__device__ __forceinline__ bool bn_ticket(unsigned* cnt, unsigned total, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores are done
  __syncthreads();
  if (threadIdx.x == 0)
    *flag = (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1);
  __syncthreads();
  return *flag != 0;
}

// s1/s2: this block's 64 channel sums (LDS).  Returns true in the one finalising block of the
// column; the column totals are then in (t1, t2) of the threads with (tid & 3) == 0, channel
// c0 + tid / 4.
__device__ __forceinline__ bool bn_column_reduce(const float* s1, const float* s2, float* part, int C, int c0,
                                                 unsigned* cnt, float& t1, float& t2, int* flag) {
  const int rb = gridDim.y, b = blockIdx.y, g = b / BN_GS, ng = (rb + BN_GS - 1) / BN_GS;
  float* part2 = part + (int64_t)rb * 2 * C;
  unsigned* col = cnt + blockIdx.x * BN_CNT;
  if (threadIdx.x < BN_CT && c0 + threadIdx.x < C) {
    st_sc1(part + (int64_t)b * 2 * C + c0 + threadIdx.x, s1[threadIdx.x]);
    st_sc1(part + (int64_t)b * 2 * C + C + c0 + threadIdx.x, s2[threadIdx.x]);
  }
  const int gb0 = g * BN_GS, gb1 = min(rb, gb0 + BN_GS);
  if (!bn_ticket(col + 1 + g, (unsigned)(gb1 - gb0), flag)) return false;
  if (threadIdx.x == 0) __hip_atomic_store(col + 1 + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bn_sum_parts(part, C, c0, gb0, gb1, t1, t2);
  if (ng == 1) return true;
  const int ch = threadIdx.x >> 2;
  if ((threadIdx.x & 3) == 0 && c0 + ch < C) {
    st_sc1(part2 + (int64_t)g * 2 * C + c0 + ch, t1);
    st_sc1(part2 + (int64_t)g * 2 * C + C + c0 + ch, t2);
  }
  if (!bn_ticket(col, (unsigned)ng, flag)) return false;
  if (threadIdx.x == 0) __hip_atomic_store(col, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bn_sum_parts(part2, C, c0, 0, ng, t1, t2);
  return true;
}

struct BnStatsArgs {
  const void* x;
  int64_t R;
  int C, rpb;
  float* part;         // [RB][2][C] + [RB/BN_GS][2][C]
  unsigned* counters;  // [C/64][BN_CNT]
  const float* gamma;
  const float* beta;
  float* mean;
  float* invstd;
  float* scale;  // a
  float* shift;  // b
  float* run_mean;
  float* run_var;
  int64_t* nbt;  // num_batches_tracked, may be null
  float momentum, eps;
};

// one tensor streamed: BN_US rows (16 B each) in flight per thread
template <typename T>
__global__ void __launch_bounds__(BN_T) bn_stats_kernel(BnStatsArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[BN_WV][BN_CT];
  __shared__ float s1[BN_CT], s2[BN_CT];
  __shared__ int flag;
  const T* x = (const T*)a.x;
  const int c0 = blockIdx.x * BN_CT;
  const int cg = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int c = c0 + cg * 8;
  const bool cok = c < a.C;  // C % 8 == 0 (host check)
  const int64_t r0 = (int64_t)blockIdx.y * a.rpb;
  const int64_t r1 = min(a.R, r0 + a.rpb);
  float piv[8], acc1[8], acc2[8];
  V8<T>::load(x + (cok ? c : 0), piv);  // pivot: row 0 (same for every block)
#pragma unroll
  for (int k = 0; k < 8; ++k) acc1[k] = acc2[k] = 0.f;
  for (int64_t r = r0 + rg; r < r1; r += BN_US * BN_RG) {
    float v[BN_US][8];
#pragma unroll
    for (int u = 0; u < BN_US; ++u) V8<T>::load(x + min(r + u * BN_RG, r1 - 1) * a.C + (cok ? c : 0), v[u]);
#pragma unroll
    for (int u = 0; u < BN_US; ++u) {
      const bool ok = r + u * BN_RG < r1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = ok ? v[u][k] - piv[k] : 0.f;
        acc1[k] += d;
        acc2[k] += d * d;
      }
    }
  }
  if (!cok) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc1[k] = acc2[k] = 0.f;
  }
  reduce_rowgroups(acc1, lds, s1);
  reduce_rowgroups(acc2, lds, s2);
  float t1, t2;
  if (!bn_column_reduce(s1, s2, a.part, a.C, c0, a.counters, t1, t2, &flag)) return;
  const int cc = c0 + (threadIdx.x >> 2);
  if ((threadIdx.x & 3) == 0 && cc < a.C) {
    const double n = (double)a.R;
    const float p0 = Ld<T>::get(x, cc);  // the pivot the partial sums were shifted by
    const float dm = (float)(t1 / n);
    const float mean = p0 + dm;
    float var = (float)(t2 / n) - dm * dm;
    var = fmaxf(var, 0.f);
    const float inv = rsqrtf(var + a.eps);
    a.mean[cc] = mean;
    a.invstd[cc] = inv;
    const float g = a.gamma ? a.gamma[cc] : 1.f;
    const float bb = a.beta ? a.beta[cc] : 0.f;
    a.scale[cc] = g * inv;
    a.shift[cc] = bb - mean * g * inv;
    if (a.run_mean) {
      const float unb = a.R > 1 ? var * (float)(n / (n - 1.0)) : var;
      a.run_mean[cc] = (1.f - a.momentum) * a.run_mean[cc] + a.momentum * mean;
      a.run_var[cc] = (1.f - a.momentum) * a.run_var[cc] + a.momentum * unb;
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.nbt) a.nbt[0] += 1;
}

// Statistics from per-row-slice partials written by the producing convolution's epilogue
// (conv.hip tile_bn_stats: sum and sum of squares per channel over slices of `tile_rows` rows).
// Each slice contributes shifted sums S1 = s - n p, S2 = q - 2 p s + n p^2 with the pivot p =
// slice 0's mean, so the column reduction and the finalisation are bn_stats' own (mean =
// p + S1/n, var = S2/n - (S1/n)^2).  "Rows" of this launch are the slices.
__global__ void __launch_bounds__(BN_T) bn_finalize_kernel(BnStatsArgs a, const float* __restrict__ tp, int ntiles,
                                                           int tile_rows) {
  __shared__ __attribute__((aligned(16))) float lds[BN_WV][BN_CT];
  __shared__ float s1[BN_CT], s2[BN_CT];
  __shared__ int flag;
  const int c0 = blockIdx.x * BN_CT;
  const int cg = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int c = c0 + cg * 8;
  const bool cok = c < a.C;
  const int cs = cok ? c : 0;
  const int64_t t0 = (int64_t)blockIdx.y * a.rpb;
  const int64_t t1e = min((int64_t)ntiles, t0 + a.rpb);
  const float n0 = (float)min((int64_t)tile_rows, a.R);
  float piv[8], acc1[8], acc2[8];
  V8<float>::load(tp + cs, piv);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    piv[k] /= n0;
    acc1[k] = acc2[k] = 0.f;
  }
  for (int64_t t = t0 + rg; t < t1e; t += BN_FU * BN_RG) {  // BN_FU tiles' loads in flight per thread
    float sm[BN_FU][8], sq[BN_FU][8];
#pragma unroll
    for (int u = 0; u < BN_FU; ++u) {
      const int64_t tu = min(t + u * BN_RG, t1e - 1);
      V8<float>::load(tp + tu * 2 * a.C + cs, sm[u]);
      V8<float>::load(tp + tu * 2 * a.C + a.C + cs, sq[u]);
    }
#pragma unroll
    for (int u = 0; u < BN_FU; ++u) {
      const int64_t tu = t + u * BN_RG;
      const float n = tu < t1e ? (float)min((int64_t)tile_rows, a.R - tu * tile_rows) : 0.f;
      const float on = tu < t1e ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc1[k] += on * sm[u][k] - n * piv[k];
        acc2[k] += on * (sq[u][k] - 2.f * piv[k] * sm[u][k]) + n * piv[k] * piv[k];
      }
    }
  }
  if (!cok) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc1[k] = acc2[k] = 0.f;
  }
  reduce_rowgroups(acc1, lds, s1);
  reduce_rowgroups(acc2, lds, s2);
  float t1, t2;
  if (!bn_column_reduce(s1, s2, a.part, a.C, c0, a.counters, t1, t2, &flag)) return;
  const int cc = c0 + (threadIdx.x >> 2);
  if ((threadIdx.x & 3) == 0 && cc < a.C) {
    const double n = (double)a.R;
    const float p0 = tp[cc] / (float)min((int64_t)tile_rows, a.R);
    const float dm = (float)(t1 / n);
    const float mean = p0 + dm;
    float var = (float)(t2 / n) - dm * dm;
    var = fmaxf(var, 0.f);
    const float inv = rsqrtf(var + a.eps);
    a.mean[cc] = mean;
    a.invstd[cc] = inv;
    const float g = a.gamma ? a.gamma[cc] : 1.f;
    const float bb = a.beta ? a.beta[cc] : 0.f;
    a.scale[cc] = g * inv;
    a.shift[cc] = bb - mean * g * inv;
    if (a.run_mean) {
      const float unb = a.R > 1 ? var * (float)(n / (n - 1.0)) : var;
      a.run_mean[cc] = (1.f - a.momentum) * a.run_mean[cc] + a.momentum * mean;
      a.run_var[cc] = (1.f - a.momentum) * a.run_var[cc] + a.momentum * unb;
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.nbt) a.nbt[0] += 1;
}

// Column sums of a [R][C] tensor accumulated into out[C] (+=): the bias gradient of a linear layer
// (sum of d(out) over the rows).  Same grid / two-level reduction as bn_stats, one tensor stream.
template <typename T>
__global__ void __launch_bounds__(BN_T) colsum_acc_kernel(const T* __restrict__ x, int64_t R, int C, int rpb,
                                                          float* part, unsigned* counters, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[BN_WV][BN_CT];
  __shared__ float s1[BN_CT], s2[BN_CT];
  __shared__ int flag;
  const int c0 = blockIdx.x * BN_CT;
  const int cg = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int c = c0 + cg * 8;
  const bool cok = c < C;
  const int64_t r0 = (int64_t)blockIdx.y * rpb;
  const int64_t r1 = min(R, r0 + rpb);
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  for (int64_t r = r0 + rg; r < r1; r += BN_US * BN_RG) {
    float v[BN_US][8];
#pragma unroll
    for (int u = 0; u < BN_US; ++u) V8<T>::load(x + min(r + u * BN_RG, r1 - 1) * C + (cok ? c : 0), v[u]);
#pragma unroll
    for (int u = 0; u < BN_US; ++u) {
      const bool ok = r + u * BN_RG < r1;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += ok ? v[u][k] : 0.f;
    }
  }
  if (!cok) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  }
  reduce_rowgroups(acc, lds, s1);
  if (threadIdx.x < BN_CT) s2[threadIdx.x] = 0.f;
  float t1, t2;
  if (!bn_column_reduce(s1, s2, part, C, c0, counters, t1, t2, &flag)) return;
  const int cc = c0 + (threadIdx.x >> 2);
  if ((threadIdx.x & 3) == 0 && cc < C) out[cc] += t1;
}

// dz = dh * gelu'(z) (bf16 [R][C]) AND out[c] += sum_r dz[r][c]: the transformer MLP's GELU
// backward fused with fc1's bias gradient, so the [tokens x hidden] gradient is read once instead of
// twice.  Grid and two-level reduction as colsum_acc_kernel.
template <typename T, int EV = 0>  // uint16_t: bf16, f16_t: fp16; EV: see BnEw (bf16 only)
__global__ void __launch_bounds__(BN_T) gelu_bwd_colsum_kernel(const T* __restrict__ dh,
                                                               const T* __restrict__ z, T* __restrict__ dz,
                                                               int64_t R, int C, int rpb, float* part,
                                                               unsigned* counters, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[BN_WV][BN_CT];
  __shared__ float s1[BN_CT], s2[BN_CT];
  __shared__ int flag;
  const int c0 = blockIdx.x * BN_CT;
  const int cg = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int c = c0 + cg * 8;
  const bool cok = c < C;
  const int64_t r0 = (int64_t)blockIdx.y * rpb;
  const int64_t r1 = min(R, r0 + rpb);
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  // the block's rows as one wave-uniform base + 32-bit per-lane offsets (rpb * C < 2^31, host
  // check): no 64-bit address arithmetic per row
  const int64_t base = r0 * C;
  const T* dhb = dh + base;
  const T* zb = z + base;
  T* dzb = dz + base;
  const int nr = (int)(r1 - r0);
  using EX = BnEw<T, EV>;
  constexpr int U = EX::U;
  for (int r = rg; r < nr; r += U * BN_RG) {
    float g[U][8], v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // byte offset: base (SGPR) + zero-extended 32-bit VGPR offset = the saddr load form
      const uint32_t off = ((uint32_t)min(r + u * BN_RG, nr - 1) * (uint32_t)C + (uint32_t)(cok ? c : 0)) * 2u;
      EX::load((const T*)((const char*)dhb + off), g[u]);
      EX::load((const T*)((const char*)zb + off), v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = r + u * BN_RG < nr && cok;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[u][k] = g[u][k] * gelu_grad(v[u][k]);
        acc[k] += ok ? v[u][k] : 0.f;
      }
      if (ok) EX::store((T*)((char*)dzb + ((uint32_t)(r + u * BN_RG) * (uint32_t)C + c) * 2u), v[u]);
    }
  }
  reduce_rowgroups(acc, lds, s1);
  if (threadIdx.x < BN_CT) s2[threadIdx.x] = 0.f;
  float t1, t2;
  if (!bn_column_reduce(s1, s2, part, C, c0, counters, t1, t2, &flag)) return;
  const int cc = c0 + (threadIdx.x >> 2);
  if ((threadIdx.x & 3) == 0 && cc < C) out[cc] += t1;
}

// Global average pool of a channels-last [N][HW][C] activation -> [N][C] (the ResNet head):
// a thread owns 8 channels of one sample and walks its HW rows with 4 loads in flight, fp32 sums.
template <typename T, typename TO>
__global__ void __launch_bounds__(256) gap_fwd_kernel(const T* __restrict__ x, TO* __restrict__ out, int N, int HW,
                                                      int C) {
  const int CV = C >> 3;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * CV) return;
  const int n = (int)(t / CV), cv = (int)(t - (int64_t)n * CV);
  const T* p = x + (int64_t)n * HW * C + cv * 8;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  int h = 0;
  for (; h + 3 < HW; h += 4) {
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) V8<T>::load(p + (int64_t)(h + u) * C, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[u][k];
  }
  for (; h < HW; ++h) {
    float v[8];
    V8<T>::load(p + (int64_t)h * C, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += v[k];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] *= inv;
  V8<TO>::store(out + (int64_t)n * C + cv * 8, acc);
}

// its backward: dx[n][hw][c] = dy[n][c] / HW (a thread writes 8 channels of one pixel)
template <typename TG, typename T>
__global__ void __launch_bounds__(256) gap_bwd_kernel(const TG* __restrict__ dy, T* __restrict__ dx, int N, int HW,
                                                      int C) {
  const int CV = C >> 3;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * HW * CV) return;
  const int64_t pix = t / CV;
  const int cv = (int)(t - pix * CV), n = (int)(pix / HW);
  float v[8];
  V8<TG>::load(dy + (int64_t)n * C + cv * 8, v);
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] *= inv;
  V8<T>::store(dx + pix * C + cv * 8, v);
}

// ViT patchify: x [B][C][H][W] (f32 or 16-bit) -> patches [B * gh * gw][C * k * k] in a 16-bit dtype,
// the im2col of a stride-k, kernel-k conv (a permutation: no duplication).  A thread moves 8
// consecutive kx of one (patch, c, ky) row: one 32-/16-byte read, one 16-byte write.  k % 8 == 0.
template <typename T, typename TO>
__global__ void __launch_bounds__(256) patchify_kernel(const T* __restrict__ x, TO* __restrict__ out, int B, int C,
                                                       int H, int W, int k) {
  const int gh = H / k, gw = W / k, kk = k * k, row_len = C * kk;
  const int64_t total = (int64_t)B * gh * gw * row_len / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int64_t e = t * 8;
  const int64_t row = e / row_len;
  const int col = (int)(e - row * row_len);
  const int c = col / kk, r = col - c * kk, ky = r / k, kx = r - ky * k;
  const int P = gh * gw;
  const int b = (int)(row / P), pp = (int)(row - (int64_t)b * P);
  const int py = pp / gw, px = pp - py * gw;
  float v[8];
  V8<T>::load(x + (((int64_t)b * C + c) * H + py * k + ky) * W + px * k + kx, v);
  V8<TO>::store(out + e, v);
}

// Elementwise passes: thread t owns channel vector cv = t % CV (CV = C/8 <= 256) for the whole
// launch, so its per-channel coefficients live in registers (loaded once), and walks rows
// r = r0 + t / CV, stepping by RPP = BN_T / CV rows; 4 rows per iteration with clamped
// (always valid) addresses keep 4 independent 16-byte loads in flight per tensor.
// y = relu?(x*a + b + res?).  With ReLU the launch also writes the 1-bit mask [y > 0]
// (mask[r][cv], bit k = channel 8cv + k): the backward reads 1 byte per 8 elements instead of y.
// RES: the residual input is a template flag, not a run-time test per element (a conditional load
// in the unrolled row loop makes hipcc wait for each load on its own: vmcnt(0) per element)
// Addresses: the block's rows start at a wave-uniform (SGPR) base; each lane adds a 32-bit byte
// offset (host check: rpb * C * 4 < 2^32), so every load / store is the saddr form with no 64-bit
// address arithmetic per row (64-bit per-row index math left these passes instruction-bound at
// ~3.6 TB/s, profiles/r3_pmc_resnet50.md).
template <typename T>
__device__ __forceinline__ T* at_b(T* base, uint32_t e) {
  return (T*)((char*)base + e * (uint32_t)sizeof(T));
}
template <typename T>
__device__ __forceinline__ const T* at_b(const T* base, uint32_t e) {
  return (const T*)((const char*)base + e * (uint32_t)sizeof(T));
}

template <typename T, typename TO, bool RES, bool RELU, int EV = 0>
__global__ void __launch_bounds__(BN_T) bn_apply_kernel(const T* __restrict__ x, const TO* __restrict__ res,
                                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                                        TO* __restrict__ y, uint8_t* __restrict__ mask, int64_t R,
                                                        int C, int rpb) {
  const int CV = C >> 3, RPP = BN_T / CV;
  if ((int)threadIdx.x >= RPP * CV) return;
  const int cv = threadIdx.x % CV, c = cv * 8;
  float A[8], B[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    A[k] = scale[c + k];
    B[k] = shift[c + k];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int nr = (int)(min(R, r0 + rpb) - r0);
  const T* xb = x + r0 * C;
  const TO* qb = RES ? res + r0 * C : res;
  TO* yb = y + r0 * C;
  uint8_t* mb = mask ? mask + r0 * (C >> 3) : mask;
  using EX = BnEw<T, EV>;
  using EO = BnEw<TO, EV>;
  constexpr int U = EX::U;
  for (int r = threadIdx.x / CV; r < nr; r += U * RPP) {
    float v[U][8], q[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t e = (uint32_t)min(r + u * RPP, nr - 1) * (uint32_t)C + (uint32_t)c;
      EX::load(at_b(xb, e), v[u]);
      if constexpr (RES) EO::load(at_b(qb, e), q[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      unsigned m = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float o = v[u][k] * A[k] + B[k];
        if constexpr (RES) o += q[u][k];
        if constexpr (RELU) {
          o = fmaxf(o, 0.f);
          m |= (o > 0.f ? 1u : 0u) << k;
        }
        v[u][k] = o;
      }
      const int ru = r + u * RPP;
      if (ru < nr) {
        EO::store(at_b(yb, (uint32_t)ru * (uint32_t)C + (uint32_t)c), v[u]);
        if (RELU && mb) mb[(uint32_t)ru * (uint32_t)CV + (uint32_t)cv] = (uint8_t)m;
      }
    }
  }
}

struct BnBwdArgs {
  const void* dy;
  const void* x;
  const uint8_t* mask;  // fused-ReLU mask [R][C/8] (bit k: channel 8cv + k), may be null
  int64_t R;
  int C, rpb;
  const float* mean;
  const float* invstd;
  float* part;
  unsigned* counters;
  float* dgamma;  // accumulated (+=), may be null
  float* dbeta;
  const float* scale;  // a = gamma * invstd
  float* coef;         // [3][C]: dx = P*dy' + Q*x + S
};

template <typename T, typename TO>
__global__ void __launch_bounds__(BN_T) bn_bwd_reduce_kernel(BnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[BN_WV][BN_CT];
  __shared__ float s1[BN_CT], s2[BN_CT];
  __shared__ int flag;
  const TO* dy = (const TO*)a.dy;
  const T* x = (const T*)a.x;
  const uint8_t* mk = a.mask;
  const int c0 = blockIdx.x * BN_CT;
  const int cg = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int c = c0 + cg * 8;
  const bool cok = c < a.C;
  const int cs = cok ? c : 0;
  const int CV = a.C >> 3, cv = cs >> 3;
  float mu[8], is[8], acc1[8], acc2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = a.mean[cs + k];
    is[k] = a.invstd[cs + k];
    acc1[k] = acc2[k] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.y * a.rpb;
  const int64_t r1 = min(a.R, r0 + a.rpb);
  for (int64_t r = r0 + rg; r < r1; r += BN_U * BN_RG) {
    float g[BN_U][8], xv[BN_U][8];
    unsigned mb[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const int64_t ru = min(r + u * BN_RG, r1 - 1);
      V8<TO>::load(dy + ru * a.C + cs, g[u]);
      V8<T>::load(x + ru * a.C + cs, xv[u]);
      mb[u] = mk ? mk[ru * CV + cv] : 0xFFu;
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const bool ok = r + u * BN_RG < r1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gg = (ok && ((mb[u] >> k) & 1u)) ? g[u][k] : 0.f;
        acc1[k] += gg;
        acc2[k] += gg * (xv[u][k] - mu[k]) * is[k];
      }
    }
  }
  if (!cok) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc1[k] = acc2[k] = 0.f;
  }
  reduce_rowgroups(acc1, lds, s1);
  reduce_rowgroups(acc2, lds, s2);
  float t1, t2;
  if (!bn_column_reduce(s1, s2, a.part, a.C, c0, a.counters, t1, t2, &flag)) return;
  const int cc = c0 + (threadIdx.x >> 2);
  if ((threadIdx.x & 3) == 0 && cc < a.C) {
    if (a.dbeta) a.dbeta[cc] += t1;
    if (a.dgamma) a.dgamma[cc] += t2;
    // dx = a*(dy' - k1 - xhat*k2), xhat = (x - mean)*invstd  ->  P*dy' + Q*x + S
    const float k1 = t1 / (float)a.R, k2 = t2 / (float)a.R;
    const float sa = a.scale[cc], is = a.invstd[cc], mu = a.mean[cc];
    a.coef[cc] = sa;
    a.coef[a.C + cc] = -sa * k2 * is;
    a.coef[2 * a.C + cc] = sa * (k2 * is * mu - k1);
  }
}

// bn_bwd_reduce's result from per-tile partials (sum dy', sum dy'*xhat) written by the stride-1
// conv dgrad that produced dy' (conv.hip store_tile_lds<BNB>): "rows" of this launch are the tiles.
__global__ void __launch_bounds__(BN_T) bn_bwd_finalize_kernel(BnBwdArgs a, const float* __restrict__ tp, int ntiles) {
  __shared__ __attribute__((aligned(16))) float lds[BN_WV][BN_CT];
  __shared__ float s1[BN_CT], s2[BN_CT];
  __shared__ int flag;
  const int c0 = blockIdx.x * BN_CT;
  const int cg = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int c = c0 + cg * 8;
  const bool cok = c < a.C;
  const int cs = cok ? c : 0;
  const int64_t t0 = (int64_t)blockIdx.y * a.rpb;
  const int64_t t1e = min((int64_t)ntiles, t0 + a.rpb);
  float acc1[8], acc2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc1[k] = acc2[k] = 0.f;
  for (int64_t t = t0 + rg; t < t1e; t += BN_FU * BN_RG) {  // BN_FU tiles' loads in flight per thread
    float sm[BN_FU][8], sq[BN_FU][8];
#pragma unroll
    for (int u = 0; u < BN_FU; ++u) {
      const int64_t tu = min(t + u * BN_RG, t1e - 1);
      V8<float>::load(tp + tu * 2 * a.C + cs, sm[u]);
      V8<float>::load(tp + tu * 2 * a.C + a.C + cs, sq[u]);
    }
#pragma unroll
    for (int u = 0; u < BN_FU; ++u) {
      const float on = t + u * BN_RG < t1e ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc1[k] += on * sm[u][k];
        acc2[k] += on * sq[u][k];
      }
    }
  }
  if (!cok) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc1[k] = acc2[k] = 0.f;
  }
  reduce_rowgroups(acc1, lds, s1);
  reduce_rowgroups(acc2, lds, s2);
  float t1, t2;
  if (!bn_column_reduce(s1, s2, a.part, a.C, c0, a.counters, t1, t2, &flag)) return;
  const int cc = c0 + (threadIdx.x >> 2);
  if ((threadIdx.x & 3) == 0 && cc < a.C) {
    if (a.dbeta) a.dbeta[cc] += t1;
    if (a.dgamma) a.dgamma[cc] += t2;
    const float k1 = t1 / (float)a.R, k2 = t2 / (float)a.R;
    const float sa = a.scale[cc], is = a.invstd[cc], mu = a.mean[cc];
    a.coef[cc] = sa;
    a.coef[a.C + cc] = -sa * k2 * is;
    a.coef[2 * a.C + cc] = sa * (k2 * is * mu - k1);
  }
}

// dx = P*dy' + Q*x + S (per-channel coefficients in registers); dres = dy'
template <typename T, typename TO, int EV = 0>
__global__ void __launch_bounds__(BN_T) bn_bwd_apply_kernel(const TO* __restrict__ dy, const T* __restrict__ x,
                                                            const uint8_t* __restrict__ mask,
                                                            const float* __restrict__ coef, T* __restrict__ dx,
                                                            TO* __restrict__ dres, int64_t R, int C, int rpb) {
  const int CV = C >> 3, RPP = BN_T / CV;
  if ((int)threadIdx.x >= RPP * CV) return;
  const int cv = threadIdx.x % CV, c = cv * 8;
  float P[8], Q[8], S[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    P[k] = coef[c + k];
    Q[k] = coef[C + c + k];
    S[k] = coef[2 * C + c + k];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int nr = (int)(min(R, r0 + rpb) - r0);
  const TO* gb = dy + r0 * C;
  const T* xb = x + r0 * C;
  T* dxb = dx + r0 * C;
  TO* drb = dres ? dres + r0 * C : dres;
  const uint8_t* mkb = mask ? mask + r0 * CV : mask;
  using EX = BnEw<T, EV>;
  using EO = BnEw<TO, EV>;
  constexpr int U = EX::U;
  for (int r = threadIdx.x / CV; r < nr; r += U * RPP) {
    float g[U][8], xv[U][8];
    unsigned mb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t ru = (uint32_t)min(r + u * RPP, nr - 1);
      const uint32_t e = ru * (uint32_t)C + (uint32_t)c;
      EO::load(at_b(gb, e), g[u]);
      EX::load(at_b(xb, e), xv[u]);
      mb[u] = mkb ? mkb[ru * (uint32_t)CV + (uint32_t)cv] : 0xFFu;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (mkb) {
#pragma unroll
        for (int k = 0; k < 8; ++k) g[u][k] = ((mb[u] >> k) & 1u) ? g[u][k] : 0.f;
      }
      const int ru = r + u * RPP;
      const bool ok = ru < nr;
      const uint32_t e = (uint32_t)ru * (uint32_t)C + (uint32_t)c;
      if (ok && drb) EO::store(at_b(drb, e), g[u]);
#pragma unroll
      for (int k = 0; k < 8; ++k) xv[u][k] = P[k] * g[u][k] + Q[k] * xv[u][k] + S[k];
      if (ok) EX::store(at_b(dxb, e), xv[u]);
    }
  }
}

// ------------------------------------------------------------------ LayerNorm
constexpr int LN_T = 256;
constexpr int LN_W = LN_T / 64;
constexpr int LN_MAXV = 16;  // up to 16 x 4 elements per lane -> C <= 4096

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float* v);
template <>
__device__ __forceinline__ void ld4<float>(const float* p, float* v) {
  const float4 a = *(const float4*)p;
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
template <>
__device__ __forceinline__ void ld4<uint16_t>(const uint16_t* p, float* v) {
  const uint2 u = *(const uint2*)p;
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
}
template <typename T>
__device__ __forceinline__ void st4(T* p, const float* v);
template <>
__device__ __forceinline__ void st4<float>(float* p, const float* v) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ __forceinline__ void st4<uint16_t>(uint16_t* p, const float* v) {
  uint2 u;
  u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *(uint2*)p = u;
}

template <>
__device__ __forceinline__ void ld4<f16_t>(const f16_t* p, float* v) {
  const uint2 u = *(const uint2*)p;
  v[0] = h2f((uint16_t)(u.x & 0xffffu)); v[1] = h2f((uint16_t)(u.x >> 16));
  v[2] = h2f((uint16_t)(u.y & 0xffffu)); v[3] = h2f((uint16_t)(u.y >> 16));
}
template <>
__device__ __forceinline__ void st4<f16_t>(f16_t* p, const float* v) {
  uint2 u;
  u.x = (uint32_t)f2h(v[0]) | ((uint32_t)f2h(v[1]) << 16);
  u.y = (uint32_t)f2h(v[2]) | ((uint32_t)f2h(v[3]) << 16);
  *(uint2*)p = u;
}

template <typename T, typename TO, int NV>
__global__ void __launch_bounds__(LN_T) ln_fwd_kernel(const T* __restrict__ x, const TO* __restrict__ res,
                                                      T* __restrict__ sum_out, const float* __restrict__ g,
                                                      const float* __restrict__ b, TO* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int64_t rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * LN_W + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * C;
  float v[NV][4], r[NV][4], ga[NV][4], be[NV][4];
  float s = 0.f;
  // every load of the row (x, the residual branch, gamma / beta) is issued before any use
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * 64 + lane) * 4;
    const int cc = c < C ? c : 0;
    ld4<T>(xr + cc, v[j]);
    if (res) ld4<TO>(res + row * C + cc, r[j]);
    if (g) ld4<float>(g + cc, ga[j]);
    if (b) ld4<float>(b + cc, be[j]);
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * 64 + lane) * 4;
    if (c < C) {
      if (res) {  // fused residual add: s = x + branch, written once for the next residual
#pragma unroll
        for (int k = 0; k < 4; ++k) v[j][k] += r[j][k];
        st4<T>(sum_out + row * C + c, v[j]);
      }
    } else {
      v[j][0] = v[j][1] = v[j][2] = v[j][3] = 0.f;
    }
    s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * 64 + lane) * 4;
    if (c < C) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = v[j][k] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * 64 + lane) * 4;
    if (c < C) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (v[j][k] - mean) * rstd * (g ? ga[j][k] : 1.f) + (b ? be[j][k] : 0.f);
      st4<TO>(y + row * C + c, o);
    }
  }
}

// a 4-element group kept as loaded (16-bit: 2 registers instead of 4) until its use
template <typename T> struct Raw4 {
  uint2 u;
  __device__ __forceinline__ void load(const T* p) { u = *(const uint2*)p; }
  __device__ __forceinline__ void get(float* v) const { ld4<T>((const T*)&u, v); }
};
template <> struct Raw4<float> {
  float4 u;
  __device__ __forceinline__ void load(const float* p) { u = *(const float4*)p; }
  __device__ __forceinline__ void get(float* v) const { v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w; }
};

// NP = 2: block partials of dgamma / dbeta; NP = 3: also the column sums of the added branch's
// gradient (dres) — the bias gradient of the linear layer that produced the branch (ViT proj /
// fc2), so that layer's backward needs no column-sum pass over its output gradient.
// Streaming design: the row reductions run on the DPP network (no LDS instructions), gamma is held
// in registers, loads stay packed until used and the next row's loads are in flight while a row is
// reduced and stored.
template <typename T, typename TO, int NV, int NP>
__global__ void __launch_bounds__(LN_T) ln_bwd_kernel(const TO* __restrict__ dy, const T* __restrict__ x,
                                                      const float* __restrict__ g, const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                      const T* __restrict__ dsum, TO* __restrict__ dres,
                                                      float* part, int64_t rows, int C, int rows_per_block,
                                                      int use_pf) {
  extern __shared__ float sm[];  // [LN_W][NP][C]
  // w (so each row index and row pointer) is wave-uniform: the row bases live in SGPRs and every
  // lane addresses all five tensors with the same small column offset
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float ag[NV][4], ab[NV][4], ar[NV][4], gm[NV][4];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * 64 + lane) * 4;
    if (g && c < C) ld4<float>(g + c, gm[j]);
    else gm[j][0] = gm[j][1] = gm[j][2] = gm[j][3] = 1.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) ag[j][k] = ab[j][k] = ar[j][k] = 0.f;
  }
  const int64_t rb = (int64_t)blockIdx.x * rows_per_block;
  const int64_t re = min(rows, rb + rows_per_block);
  // software prefetch: the next row's loads are in flight while this row is reduced and stored
  Raw4<T> xr[NV], sr[NV], xn[NV], sn[NV];
  Raw4<TO> dr[NV], dn[NV];
  auto fetch = [&](int64_t row, Raw4<T> (&xa)[NV], Raw4<TO> (&da)[NV], Raw4<T> (&sa)[NV]) {
    const T* xrow = x + row * C;
    const TO* dyrow = dy + row * C;
    const T* dsrow = dsum ? dsum + row * C : nullptr;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = (j * 64 + lane) * 4;
      const int cc = c < C ? c : 0;
      xa[j].load(xrow + cc);
      da[j].load(dyrow + cc);
      if (dsum) sa[j].load(dsrow + cc);
    }
  };
  // wide rows (C > 1024): no room for a second row's registers
  const bool PF = NV <= 4 && use_pf;
  if (PF && rb + w < re) fetch(rb + w, xr, dr, sr);
  for (int64_t row = rb + w; row < re; row += LN_W) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    if (!PF) fetch(row, xr, dr, sr);
    else if (row + LN_W < re) fetch(row + LN_W, xn, dn, sn);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = (j * 64 + lane) * 4;
      if (c < C) {
        float xv[4], dv[4];
        xr[j].get(xv);
        dr[j].get(dv);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float xh = (xv[k] - mean) * rstd;
          const float gy = dv[k] * gm[j][k];
          s1 += gy;
          s2 += gy * xh;
          ag[j][k] += dv[k] * xh;
          ab[j][k] += dv[k];
        }
      }
    }
    s1 = wave_sum_dpp(s1) / C;
    s2 = wave_sum_dpp(s2) / C;
    T* dxrow = dx + row * C;
    TO* dresrow = dres ? dres + row * C : nullptr;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = (j * 64 + lane) * 4;
      if (c < C) {
        float xv[4], dv[4], o[4];
        xr[j].get(xv);
        dr[j].get(dv);
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = rstd * (dv[k] * gm[j][k] - s1 - (xv[k] - mean) * rstd * s2);
        if (dsum) {  // the residual stream's own gradient joins here (fused add-norm)
          float ds[4];
          sr[j].get(ds);
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] += ds[k];
        }
        st4<T>(dxrow + c, o);
        if (dres) st4<TO>(dresrow + c, o);  // gradient of the added branch
        if (NP == 3) {
#pragma unroll
          for (int k = 0; k < 4; ++k) ar[j][k] += o[k];
        }
      }
    }
    if (PF) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        xr[j] = xn[j];
        dr[j] = dn[j];
        sr[j] = sn[j];
      }
    }
  }
  // block partial: every wave parks its column partials in its own LDS image (16-byte stores,
  // consecutive lanes: whole bank rows), then each thread sums the 4 waves' values of its columns
  // (per-wave images instead of LDS atomics into one: the atomics' per-block cost measured higher
  // than the 4x LDS footprint, bench/ln_probe.py)
  // k-major image: column 4q + k at k (C / 4) + q, so a wave's 4-byte stores cover consecutive
  // words (the 16-byte stores of the natural order measured 60% SQ_LDS_BANK_CONFLICT); the block
  // partial keeps that order and colsum_kernel maps it back (perm_q = C / 4)
  const int cq = C / 4;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = j * 64 + lane;
    if (4 * q < C) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sm[(w * NP) * C + k * cq + q] = ag[j][k];
        sm[(w * NP + 1) * C + k * cq + q] = ab[j][k];
        if (NP == 3) sm[(w * NP + 2) * C + k * cq + q] = ar[j][k];
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NP * C; i += LN_T) {
    float t = 0.f;
#pragma unroll
    for (int ww = 0; ww < LN_W; ++ww) t += sm[ww * NP * C + i];
    part[(int64_t)blockIdx.x * NP * C + i] = t;
  }
}

// column sums of the [nrows][2C] block partials -> dgamma (first C) / dbeta (last C), accumulated.
// Block: 64 columns x 16 row-slices; each thread strides its slice with 4 loads in flight.
// perm_q > 0: each C-wide section of a partial row is stored k-major (position k * perm_q + q holds
// column 4q + k, ln_bwd_kernel's image).
constexpr int CS_T = 1024;
__global__ void __launch_bounds__(CS_T) colsum_kernel(const float* __restrict__ part, int nrows, int C2,
                                                      float* dgamma, float* dbeta, int C, float* dthird = nullptr,
                                                      int perm_q = 0, float* dthird_acc = nullptr) {
  __shared__ float red[CS_T / 64][65];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6, nsl = CS_T / 64;
  const int cc = col < C2 ? col : C2 - 1;
  float t = 0.f;
  int r = sl;
  for (; r + 3 * nsl < nrows; r += 4 * nsl) {
    const float a0 = part[(int64_t)r * C2 + cc], a1 = part[(int64_t)(r + nsl) * C2 + cc];
    const float a2 = part[(int64_t)(r + 2 * nsl) * C2 + cc], a3 = part[(int64_t)(r + 3 * nsl) * C2 + cc];
    t += (a0 + a1) + (a2 + a3);
  }
  for (; r < nrows; r += nsl) t += part[(int64_t)r * C2 + cc];
  red[sl][threadIdx.x & 63] = t;
  __syncthreads();
  if (threadIdx.x < 64 && col < C2) {
    float u = 0.f;
#pragma unroll
    for (int k = 0; k < CS_T / 64; ++k) u += red[k][threadIdx.x];
    const int sec = col / C;
    int oc = col - sec * C;
    if (perm_q > 0) oc = 4 * (oc % perm_q) + oc / perm_q;
    if (sec == 0) {
      if (dgamma) dgamma[oc] += u;
    } else if (sec == 1) {
      if (dbeta) dbeta[oc] += u;
    } else if (dthird) {
      dthird[oc] = u;  // written, not accumulated: the caller needs no zeroed buffer
      if (dthird_acc) dthird_acc[oc] += u;
    }
  }
}

// ---- BatchNorm + ReLU + 3x3/stride-2/pad-1 max-pool (the ImageNet ResNet stem) -------------------
// Forward: one thread per (n, oh, ow, 8-channel vector): the nine window pixels are normalised in
// registers (relu(x*a + b)) and max-reduced; the full-resolution activation never reaches HBM.
// Per channel a 1-byte code records the window tap (kh*3 + kw) of the max, or 0xFF when the max is
// 0 (every tap <= 0: ReLU kills the gradient).  Strict '>' keeps the first max, as max_pool2d does.
// Backward (gather, no atomics): one thread per input pixel vector sums the pooled gradients of
// the <= 2x2 windows whose code names it; the result is the ReLU-masked gradient of the BN output,
// handed to bn_bwd with no mask.  256 % (C/8) == 0 (host check): a thread's channel vector is
// fixed across the grid-stride loop, so the coefficients stay in registers.
constexpr int MP_T = 256;

template <typename T>
__global__ void __launch_bounds__(MP_T) bn_relu_maxpool_kernel(const T* __restrict__ x, const float* __restrict__ scale,
                                                               const float* __restrict__ shift, T* __restrict__ y,
                                                               uint8_t* __restrict__ code, int N, int H, int W, int C,
                                                               int OH, int OW) {
  const int CV = C >> 3;
  const int total = N * OH * OW * CV;  // < 2^31 (host check)
  int q = blockIdx.x * MP_T + threadIdx.x;
  const int cv = q % CV, c = cv * 8;
  float A[8], B[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    A[k] = scale[c + k];
    B[k] = shift[c + k];
  }
  for (; q < total; q += gridDim.x * MP_T) {
    // 32-bit index math (host check: N*H*W*C/8 < 2^31; 64-bit division is a long emulated sequence)
    const int pq = q / CV;  // output pixel
    const int t = pq / OW, ow = pq - t * OW, n = t / OH, oh = t - n * OH;
    const int64_t p = pq;
    float best[8];
    unsigned idx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      best[k] = 0.f;
      idx[k] = 0xFFu;
    }
    const int64_t img = (int64_t)n * H * W;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        V8<T>::load(x + (img + (int64_t)ih * W + iw) * C + c, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float o = v[k] * A[k] + B[k];
          if (o > best[k]) {
            best[k] = o;
            idx[k] = (unsigned)(kh * 3 + kw);
          }
        }
      }
    }
    V8<T>::store(y + p * C + c, best);
    *(uint2*)(code + p * C + c) = make_uint2(idx[0] | (idx[1] << 8) | (idx[2] << 16) | (idx[3] << 24),
                                             idx[4] | (idx[5] << 8) | (idx[6] << 16) | (idx[7] << 24));
  }
}

template <typename T>
__global__ void __launch_bounds__(MP_T) maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ code,
                                                           T* __restrict__ dx, int N, int H, int W, int C, int OH,
                                                           int OW) {
  const int CV = C >> 3;
  const int64_t total = (int64_t)N * H * W * CV;
  for (int q = blockIdx.x * MP_T + threadIdx.x; q < (int)total; q += gridDim.x * MP_T) {
    const int c = (q % CV) * 8;
    const int pq = q / CV;  // input pixel (32-bit index math, host-checked range)
    const int t = pq / W, iw = pq - t * W, n = t / H, ih = t - n * H;
    const int64_t p = pq;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const int oh = (ih + 1) / 2 - dh, kh = ih - 2 * oh + 1;
      if (oh < 0 || oh >= OH || kh > 2) continue;
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int ow = (iw + 1) / 2 - dw, kw = iw - 2 * ow + 1;
        if (ow < 0 || ow >= OW || kw > 2) continue;
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c;
        const uint2 cd = *(const uint2*)(code + o);
        float g[8];
        V8<T>::load(dy + o, g);
        const unsigned t = (unsigned)(kh * 3 + kw);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const unsigned ck = ((k < 4 ? cd.x : cd.y) >> (8 * (k & 3))) & 0xFFu;
          acc[k] += ck == t ? g[k] : 0.f;
        }
      }
    }
    V8<T>::store(dx + p * C + c, acc);
  }
}

int mp_grid(int64_t work) {
  const int64_t b = (work + MP_T - 1) / MP_T;
  return (int)(b < 256 * 16 ? b : 256 * 16);
}

int bn_grid_rows(int64_t R, int C, int* rpb) {
  // ~2048 blocks in total (8 per CU: enough loads in flight to stream HBM); the two-level
  // finalize keeps the serial tail short at any block count
  const int ncol = (C + BN_CT - 1) / BN_CT;
  int64_t rb = 2048 / ncol;
  if (rb < 1) rb = 1;
  if (rb > BN_MAXRB) rb = BN_MAXRB;
  int64_t per = (R + rb - 1) / rb;
  per = (per + BN_ROWQ - 1) / BN_ROWQ * BN_ROWQ;
  *rpb = (int)per;
  return (int)((R + per - 1) / per);
}

}  // namespace

// workspace needed by the BN reductions (floats): block partials + group partials, 2*C each
RK_API int64_t rk_bn_workspace(int64_t R, int C) {
  int rpb;
  const int rb = bn_grid_rows(R, C, &rpb);
  return (int64_t)(rb + (rb + BN_GS - 1) / BN_GS) * 2 * C;
}

// ticket counters needed by one BN reduction launch over C channels (zeroed once, self-resetting)
RK_API int rk_bn_counters(int C) { return (C + BN_CT - 1) / BN_CT * BN_CNT; }

// Stem BatchNorm + ReLU + 3x3/s2/p1 max-pool over NHWC x [N][H][W][C] -> y, code [N][OH][OW][C]
RK_API int rk_bn_relu_maxpool(int dt, const void* x, const float* scale, const float* shift, void* y, void* code, int N,
                              int H, int W, int C, int OH, int OW, hipStream_t s) {
  if (C % 8 || MP_T % (C / 8) || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1) return (int)hipErrorInvalidValue;
  if ((int64_t)N * H * W * (C / 8) >= ((int64_t)1 << 31) - 2 * 256 * 16 * MP_T) return (int)hipErrorInvalidValue;
  const int g = mp_grid((int64_t)N * OH * OW * (C / 8));
  if (dt == BF16)
    bn_relu_maxpool_kernel<uint16_t><<<g, MP_T, 0, s>>>((const uint16_t*)x, scale, shift, (uint16_t*)y,
                                                         (uint8_t*)code, N, H, W, C, OH, OW);
  else if (dt == F16)
    bn_relu_maxpool_kernel<f16_t><<<g, MP_T, 0, s>>>((const f16_t*)x, scale, shift, (f16_t*)y, (uint8_t*)code, N, H,
                                                      W, C, OH, OW);
  else
    bn_relu_maxpool_kernel<float><<<g, MP_T, 0, s>>>((const float*)x, scale, shift, (float*)y, (uint8_t*)code, N, H,
                                                      W, C, OH, OW);
  return (int)hipGetLastError();
}

// gradient of rk_bn_relu_maxpool's pool + ReLU: dy [N][OH][OW][C] -> dx [N][H][W][C] (same dtype)
RK_API int rk_maxpool_bwd(int dt, const void* dy, const void* code, void* dx, int N, int H, int W, int C, int OH,
                          int OW, hipStream_t s) {
  if (C % 8 || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1) return (int)hipErrorInvalidValue;
  if ((int64_t)N * H * W * (C / 8) >= ((int64_t)1 << 31) - 2 * 256 * 16 * MP_T) return (int)hipErrorInvalidValue;
  const int g = mp_grid((int64_t)N * H * W * (C / 8));
  if (dt == BF16)
    maxpool_bwd_kernel<uint16_t><<<g, MP_T, 0, s>>>((const uint16_t*)dy, (const uint8_t*)code, (uint16_t*)dx, N, H,
                                                     W, C, OH, OW);
  else if (dt == F16)
    maxpool_bwd_kernel<f16_t><<<g, MP_T, 0, s>>>((const f16_t*)dy, (const uint8_t*)code, (f16_t*)dx, N, H, W, C,
                                                  OH, OW);
  else
    maxpool_bwd_kernel<float><<<g, MP_T, 0, s>>>((const float*)dy, (const uint8_t*)code, (float*)dx, N, H, W, C,
                                                  OH, OW);
  return (int)hipGetLastError();
}

// x: [R][C] (dt 0 f32 / 1 bf16). Training statistics + fused scale/shift + running stats.
RK_API int rk_bn_stats(int dt, const void* x, int64_t R, int C, const float* gamma, const float* beta, float* mean,
                       float* invstd, float* scale, float* shift, float* run_mean, float* run_var, int64_t* nbt,
                       float momentum, float eps, float* ws, unsigned* counters, hipStream_t s) {
  if (C % 8 || R <= 0) return (int)hipErrorInvalidValue;
  BnStatsArgs a{x, R, C, 0, ws, counters, gamma, beta, mean, invstd, scale, shift, run_mean, run_var, nbt, momentum, eps};
  const int rb = bn_grid_rows(R, C, &a.rpb);
  dim3 grid((C + BN_CT - 1) / BN_CT, rb);
  if (dt == BF16)
    bn_stats_kernel<uint16_t><<<grid, BN_T, 0, s>>>(a);
  else if (dt == F16)
    bn_stats_kernel<f16_t><<<grid, BN_T, 0, s>>>(a);
  else
    bn_stats_kernel<float><<<grid, BN_T, 0, s>>>(a);
  return (int)hipGetLastError();
}

// Tiles per block of the finalize launches (whole passes of BN_RG, at most rb_max row blocks: the
// workspace rk_bn_workspace(R, C) sized).  The partials are small (ResNet-18 CIFAR: <= 2048 tiles x
// 2 x C floats), so the launch is latency-bound: at most BN_GS row blocks per column while each
// thread keeps <= 4 passes of BN_FU tiles makes the ticket tree one level deep (one store / ticket /
// re-read round trip instead of two).  ROCKET_BN_FIN_ONE=0: as many row blocks as the workspace allows.
static int bn_final_per(int ntiles, int rb_max) {
  static const int one = [] {
    const char* e = getenv("ROCKET_BN_FIN_ONE");
    return e ? atoi(e) : 1;
  }();
  int per = (ntiles + rb_max - 1) / rb_max;
  if (one) {
    const int p1 = (ntiles + BN_GS - 1) / BN_GS;
    if (p1 <= 4 * BN_FU * BN_RG) per = max(per, p1);
  }
  return (per + BN_RG - 1) / BN_RG * BN_RG;
}

// Same outputs as rk_bn_stats, from the per-row-tile partials tp ([ntiles][2][C]: tile mean, M2) of
// an R-row activation cut into tiles of tile_rows rows.  ws / counters as for rk_bn_stats(R, C).
RK_API int rk_bn_finalize(const float* tp, int ntiles, int tile_rows, int64_t R, int C, const float* gamma,
                          const float* beta, float* mean, float* invstd, float* scale, float* shift, float* run_mean,
                          float* run_var, int64_t* nbt, float momentum, float eps, float* ws, unsigned* counters,
                          hipStream_t s) {
  if (C % 8 || R <= 0 || ntiles <= 0 || (int64_t)ntiles * tile_rows < R) return (int)hipErrorInvalidValue;
  BnStatsArgs a{nullptr, R, C, 0, ws, counters, gamma, beta, mean, invstd, scale, shift, run_mean, run_var, nbt,
                momentum, eps};
  // tiles per block: whole passes of BN_RG, at most the row blocks rk_bn_workspace(R, C) sized for
  int rpb_rows;
  const int rb_max = bn_grid_rows(R, C, &rpb_rows);
  const int per = bn_final_per(ntiles, rb_max);
  a.rpb = per;
  const int rb = (ntiles + per - 1) / per;
  dim3 grid((C + BN_CT - 1) / BN_CT, rb);
  bn_finalize_kernel<<<grid, BN_T, 0, s>>>(a, tp, ntiles, tile_rows);
  return (int)hipGetLastError();
}

// rows per block for the elementwise passes: ~2048 blocks, whole passes of RPP rows
static int bn_ew_variant();
// the variant for one tensor: nontemporal only for tensors far beyond the Infinity Cache's reuse
// (ResNet-50's >= 103 MB BatchNorm tensors gain 1-10%; ResNet-18's CIFAR-shape 33 MB ones lose 1.9%
// with it: the next pass re-reads them from the cache; scripts/r5/gpu_r18.sh)
static int bn_ew_for(int64_t R, int C) {
  int v = bn_ew_variant();
  if (R * (int64_t)C * 2 < ((int64_t)64 << 20)) v &= ~1;
  return v;
}
static int bn_ew_variant() {
  // default 1 (nontemporal): ResNet-50 10,569-10,579 -> 10,668-10,682 img/s, the fused BN
  // fwd+bwd probe +10% on the 56x56 / 28x28 residual shapes (profiles/r5_bn_ew_ab.md)
  static const int v = getenv("ROCKET_BN_EW") ? atoi(getenv("ROCKET_BN_EW")) & 3 : 1;
  return v;
}
static int bn_elem_rows(int64_t R, int C, int* grid) {
  const int rpp = BN_T / (C / 8);
  int64_t per = (R + 2047) / 2048;
  per = (per + rpp - 1) / rpp * rpp;
  if (per < rpp) per = rpp;
  *grid = (int)((R + per - 1) / per);
  return (int)per;
}
// the elementwise passes' per-block 32-bit byte offsets (at_b) must not wrap
static bool bn_elem_ok(int rpb, int C) { return (int64_t)rpb * C * 4 < (1ll << 32); }

// out[c] += sum_r x[r][c]  (x: [R][C], dt f32 / bf16 / f16, C % 8 == 0); ws: rk_bn_workspace(R, C)
// floats, counters: rk_bn_counters(C) zeroed uints (self-resetting)
// Global average pool (channels-last [N][HW][C] -> [N][C]) and its backward.  dt: x / dx dtype,
// dto: out / dy dtype (F32, BF16 or F16; 16-bit pairs must match).  C % 8 == 0.
RK_API int rk_gap_fwd(int dt, int dto, const void* x, void* out, int N, int HW, int C, hipStream_t s) {
  if (C % 8 || N <= 0 || HW <= 0 || (dt != F32 && dto != F32 && dt != dto)) return (int)hipErrorInvalidValue;
  const int64_t nt = (int64_t)N * (C / 8);
  const int grid = (int)((nt + 255) / 256);
#define RK_GF(T, TO) gap_fwd_kernel<T, TO><<<grid, 256, 0, s>>>((const T*)x, (TO*)out, N, HW, C)
  if (dt == BF16 && dto == BF16) RK_GF(uint16_t, uint16_t);
  else if (dt == F16 && dto == F16) RK_GF(f16_t, f16_t);
  else if (dt == BF16) RK_GF(uint16_t, float);
  else if (dt == F16) RK_GF(f16_t, float);
  else if (dto == BF16) RK_GF(float, uint16_t);
  else if (dto == F16) RK_GF(float, f16_t);
  else RK_GF(float, float);
#undef RK_GF
  return (int)hipGetLastError();
}
RK_API int rk_gap_bwd(int dt, int dto, const void* dy, void* dx, int N, int HW, int C, hipStream_t s) {
  if (C % 8 || N <= 0 || HW <= 0 || (dt != F32 && dto != F32 && dt != dto)) return (int)hipErrorInvalidValue;
  const int64_t nt = (int64_t)N * HW * (C / 8);
  const int grid = (int)((nt + 255) / 256);
#define RK_GB(TG, T) gap_bwd_kernel<TG, T><<<grid, 256, 0, s>>>((const TG*)dy, (T*)dx, N, HW, C)
  if (dt == BF16 && dto == BF16) RK_GB(uint16_t, uint16_t);
  else if (dt == F16 && dto == F16) RK_GB(f16_t, f16_t);
  else if (dt == BF16) RK_GB(float, uint16_t);
  else if (dt == F16) RK_GB(float, f16_t);
  else if (dto == BF16) RK_GB(uint16_t, float);
  else if (dto == F16) RK_GB(f16_t, float);
  else RK_GB(float, float);
#undef RK_GB
  return (int)hipGetLastError();
}

// ViT patchify (see patchify_kernel).  dt: x dtype (F32 / BF16 / F16), dto: out dtype (BF16 / F16).
RK_API int rk_patchify(int dt, int dto, const void* x, void* out, int B, int C, int H, int W, int k, hipStream_t s) {
  if (k <= 0 || k % 8 || H % k || W % k || B <= 0 || C <= 0 || (dto != BF16 && dto != F16) ||
      (dt != F32 && dt != dto))
    return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)B * (H / k) * (W / k) * C * k * k / 8;
  const int grid = (int)((total + 255) / 256);
#define RK_PF(T, TO) patchify_kernel<T, TO><<<grid, 256, 0, s>>>((const T*)x, (TO*)out, B, C, H, W, k)
  if (dt == F32 && dto == BF16) RK_PF(float, uint16_t);
  else if (dt == F32) RK_PF(float, f16_t);
  else if (dto == BF16) RK_PF(uint16_t, uint16_t);
  else RK_PF(f16_t, f16_t);
#undef RK_PF
  return (int)hipGetLastError();
}

RK_API int rk_colsum_acc(int dt, const void* x, int64_t R, int C, float* out, float* ws, unsigned* counters,
                         hipStream_t s) {
  if (C % 8 || R <= 0) return (int)hipErrorInvalidValue;
  int rpb;
  const int rb = bn_grid_rows(R, C, &rpb);
  dim3 grid((C + BN_CT - 1) / BN_CT, rb);
  if (dt == BF16)
    colsum_acc_kernel<uint16_t><<<grid, BN_T, 0, s>>>((const uint16_t*)x, R, C, rpb, ws, counters, out);
  else if (dt == F16)
    colsum_acc_kernel<f16_t><<<grid, BN_T, 0, s>>>((const f16_t*)x, R, C, rpb, ws, counters, out);
  else
    colsum_acc_kernel<float><<<grid, BN_T, 0, s>>>((const float*)x, R, C, rpb, ws, counters, out);
  return (int)hipGetLastError();
}

// dz = dh * gelu'(z) and out[c] += sum_r dz[r][c] (all 16-bit [R][C] of dtype dt, bf16 or fp16,
// except out; C % 8 == 0); ws / counters as rk_colsum_acc
RK_API int rk_gelu_bwd_colsum16(int dt, const void* dh, const void* z, void* dz, int64_t R, int C, float* out,
                                float* ws, unsigned* counters, hipStream_t s) {
  if (C % 8 || R <= 0 || (dt != BF16 && dt != F16)) return (int)hipErrorInvalidValue;
  int rpb;
  const int rb = bn_grid_rows(R, C, &rpb);
  if ((int64_t)rpb * C * 2 >= (1ll << 32)) return (int)hipErrorInvalidValue;
  dim3 grid((C + BN_CT - 1) / BN_CT, rb);
  if (dt == F16)
    gelu_bwd_colsum_kernel<f16_t><<<grid, BN_T, 0, s>>>((const f16_t*)dh, (const f16_t*)z, (f16_t*)dz, R, C, rpb, ws,
                                                        counters, out);
  else
  {
    // ROCKET_GELU_EW (act.hip rk_gelu_fwd): 2 (default) = nontemporal loads / stores here too
    static const int gev = getenv("ROCKET_GELU_EW") ? atoi(getenv("ROCKET_GELU_EW")) : 2;
    if (gev == 2)
      gelu_bwd_colsum_kernel<uint16_t, 1><<<grid, BN_T, 0, s>>>((const uint16_t*)dh, (const uint16_t*)z, (uint16_t*)dz,
                                                                R, C, rpb, ws, counters, out);
    else
      gelu_bwd_colsum_kernel<uint16_t><<<grid, BN_T, 0, s>>>((const uint16_t*)dh, (const uint16_t*)z, (uint16_t*)dz, R, C,
                                                             rpb, ws, counters, out);
  }
  return (int)hipGetLastError();
}
RK_API int rk_gelu_bwd_colsum(const void* dh, const void* z, void* dz, int64_t R, int C, float* out, float* ws,
                              unsigned* counters, hipStream_t s) {
  return rk_gelu_bwd_colsum16(BF16, dh, z, dz, R, C, out, ws, counters, s);
}

// y = relu?(x*scale + shift + res?); dt: x dtype, dto: y/res dtype.  mask (uint8 [R][C/8], may be
// null): the ReLU mask bits for rk_bn_bwd.
RK_API int rk_bn_apply(int dt, int dto, const void* x, const void* res, const float* scale, const float* shift, void* y,
                       void* mask, int64_t R, int C, int relu, hipStream_t s) {
  if (dto == F16 && dt != F16) return (int)hipErrorInvalidValue;  // f16 variants: (f16, f16), (f16, f32)
  if (C % 8 || C > 8 * BN_T || R <= 0) return (int)hipErrorInvalidValue;
  int grid;
  const int rpb = bn_elem_rows(R, C, &grid);
  if (!bn_elem_ok(rpb, C)) return (int)hipErrorInvalidValue;
#define RK_BA2(T, TO, RES, EV)                                                                                 \
  do {                                                                                                          \
    if (relu)                                                                                                   \
      bn_apply_kernel<T, TO, RES, true, EV><<<grid, BN_T, 0, s>>>((const T*)x, (const TO*)res, scale, shift,    \
                                                                  (TO*)y, (uint8_t*)mask, R, C, rpb);           \
    else                                                                                                        \
      bn_apply_kernel<T, TO, RES, false, EV><<<grid, BN_T, 0, s>>>((const T*)x, (const TO*)res, scale, shift,   \
                                                                   (TO*)y, nullptr, R, C, rpb);                 \
  } while (0)
#define RK_BA(T, TO, ...)                                  \
  do {                                                     \
    if (res) RK_BA2(T, TO, true, __VA_OPT__(__VA_ARGS__ +) 0);   \
    else RK_BA2(T, TO, false, __VA_OPT__(__VA_ARGS__ +) 0);      \
  } while (0)
  if (dt == F16 && dto == F16) RK_BA(f16_t, f16_t);
  else if (dt == F16 && dto == F32) RK_BA(f16_t, float);
  else if (dt == BF16 && dto == BF16) {
    switch (bn_ew_for(R, C)) {
      case 1: RK_BA(uint16_t, uint16_t, 1); break;
      case 2: RK_BA(uint16_t, uint16_t, 2); break;
      case 3: RK_BA(uint16_t, uint16_t, 3); break;
      default: RK_BA(uint16_t, uint16_t, 0);
    }
  } else if (dt == BF16) RK_BA(uint16_t, float);
  else if (dto == BF16) RK_BA(float, uint16_t);
  else RK_BA(float, float);
#undef RK_BA
#undef RK_BA2
  return (int)hipGetLastError();
}

// backward. dt: x/dx dtype; dto: dy/dres dtype. mask (fused-ReLU bits from rk_bn_apply) may be
// null, dres may be null.
RK_API int rk_bn_bwd(int dt, int dto, const void* dy, const void* x, const void* mask, int64_t R, int C,
                     const float* mean, const float* invstd, const float* scale, float* dgamma, float* dbeta, void* dx,
                     void* dres, float* ws, float* coef /*[3C]*/, unsigned* counters, hipStream_t s) {
  if (dto == F16 && dt != F16) return (int)hipErrorInvalidValue;  // f16 variants: (f16, f16), (f16, f32)
  if (C % 8 || C > 8 * BN_T || R <= 0) return (int)hipErrorInvalidValue;
  BnBwdArgs a{dy, x, (const uint8_t*)mask, R, C, 0, mean, invstd, ws, counters, dgamma, dbeta, scale, coef};
  const int rb = bn_grid_rows(R, C, &a.rpb);
  dim3 grid((C + BN_CT - 1) / BN_CT, rb);
  int eg;
  const int erpb = bn_elem_rows(R, C, &eg);
  if (!bn_elem_ok(erpb, C)) return (int)hipErrorInvalidValue;
#define RK_BB(T, TO, ...)                                                                                          \
  do {                                                                                                             \
    bn_bwd_reduce_kernel<T, TO><<<grid, BN_T, 0, s>>>(a);                                                          \
    bn_bwd_apply_kernel<T, TO, __VA_OPT__(__VA_ARGS__ +) 0><<<eg, BN_T, 0, s>>>((const TO*)dy, (const T*)x,       \
                                                   (const uint8_t*)mask, coef, (T*)dx, (TO*)dres, R, C, erpb);      \
  } while (0)
  if (dt == F16 && dto == F16) RK_BB(f16_t, f16_t);
  else if (dt == F16 && dto == F32) RK_BB(f16_t, float);
  else if (dt == BF16 && dto == BF16) {
    switch (bn_ew_for(R, C)) {
      case 1: RK_BB(uint16_t, uint16_t, 1); break;
      case 2: RK_BB(uint16_t, uint16_t, 2); break;
      case 3: RK_BB(uint16_t, uint16_t, 3); break;
      default: RK_BB(uint16_t, uint16_t, 0);
    }
  }
  else if (dt == BF16) RK_BB(uint16_t, float);
  else if (dto == BF16) RK_BB(float, uint16_t);
  else RK_BB(float, float);
#undef RK_BB
  return (int)hipGetLastError();
}

// LayerNorm forward over rows of C (C % 4 == 0, C <= 4096).  dt: x dtype, dto: y dtype.
// res (dtype dto) / sum_out (dtype dt) may be null: y = LN(x [+ res]), sum_out = x + res
// BatchNorm backward from the producing dgrad's partials (tp [ntiles][2][C], one row per output
// tile of the dgrad): dy is already ReLU-masked, so the input-gradient pass reads no mask.  dt: x / dx dtype,
// dto: dy / dres dtype.
RK_API int rk_bn_bwd_partials(int dt, int dto, const void* dy, const void* x, const float* tp, int ntiles, int64_t R,
                              int C, const float* mean, const float* invstd, const float* scale, float* dgamma,
                              float* dbeta, void* dx, void* dres, float* ws, float* coef, unsigned* counters,
                              hipStream_t s) {
  if (dto == F16 && dt != F16) return (int)hipErrorInvalidValue;  // f16 variants: (f16, f16), (f16, f32)
  if (C % 8 || C > 8 * BN_T || R <= 0 || ntiles <= 0) return (int)hipErrorInvalidValue;
  BnBwdArgs a{dy, x, nullptr, R, C, 0, mean, invstd, ws, counters, dgamma, dbeta, scale, coef};
  int rpb_rows;
  const int rb_max = bn_grid_rows(R, C, &rpb_rows);  // the workspace rk_bn_workspace(R, C) sized
  const int per = bn_final_per(ntiles, rb_max);
  a.rpb = per;
  dim3 grid((C + BN_CT - 1) / BN_CT, (ntiles + per - 1) / per);
  bn_bwd_finalize_kernel<<<grid, BN_T, 0, s>>>(a, tp, ntiles);
  int eg;
  const int erpb = bn_elem_rows(R, C, &eg);
  if (!bn_elem_ok(erpb, C)) return (int)hipErrorInvalidValue;
#define RK_BP(T, TO, ...)                                                                                       \
  bn_bwd_apply_kernel<T, TO, __VA_OPT__(__VA_ARGS__ +) 0><<<eg, BN_T, 0, s>>>((const TO*)dy, (const T*)x, nullptr, coef, \
                                                                            (T*)dx, (TO*)dres, R, C, erpb)
  if (dt == F16 && dto == F16) RK_BP(f16_t, f16_t);
  else if (dt == F16 && dto == F32) RK_BP(f16_t, float);
  else if (dt == BF16 && dto == BF16) {
    switch (bn_ew_for(R, C)) {
      case 1: RK_BP(uint16_t, uint16_t, 1); break;
      case 2: RK_BP(uint16_t, uint16_t, 2); break;
      case 3: RK_BP(uint16_t, uint16_t, 3); break;
      default: RK_BP(uint16_t, uint16_t, 0);
    }
  }
  else if (dt == BF16) RK_BP(uint16_t, float);
  else if (dto == BF16) RK_BP(float, uint16_t);
  else RK_BP(float, float);
#undef RK_BP
  return (int)hipGetLastError();
}

RK_API int rk_ln_fwd(int dt, int dto, const void* x, const void* res, void* sum_out, const float* g, const float* b,
                     void* y, float* mean, float* rstd, int64_t rows, int C, float eps, hipStream_t s) {
  if ((dt == F16 && dto == BF16) || (dt == BF16 && dto == F16)) return (int)hipErrorInvalidValue;
  if (C % 4 || C > 64 * 4 * LN_MAXV) return (int)hipErrorInvalidValue;
  const int grid = (int)((rows + LN_W - 1) / LN_W);
  const int nv = (C + 255) / 256;
#define RK_LF(T, TO, NV) \
  ln_fwd_kernel<T, TO, NV><<<grid, LN_T, 0, s>>>((const T*)x, (const TO*)res, (T*)sum_out, g, b, (TO*)y, mean, rstd, rows, C, eps)
#define RK_LFN(T, TO)                 \
  if (nv <= 1) RK_LF(T, TO, 1);       \
  else if (nv <= 2) RK_LF(T, TO, 2);  \
  else if (nv <= 3) RK_LF(T, TO, 3);  \
  else if (nv <= 4) RK_LF(T, TO, 4);  \
  else if (nv <= 8) RK_LF(T, TO, 8);  \
  else RK_LF(T, TO, 16);
  if (dt == BF16 && dto == BF16) { RK_LFN(uint16_t, uint16_t) }
  else if (dt == F16 && dto == F16) { RK_LFN(f16_t, f16_t) }
  else if (dt == F16) { RK_LFN(f16_t, float) }
  else if (dto == F16) { RK_LFN(float, f16_t) }
  else if (dt == BF16) { RK_LFN(uint16_t, float) }
  else if (dto == BF16) { RK_LFN(float, uint16_t) }
  else { RK_LFN(float, float) }
#undef RK_LFN
#undef RK_LF
  return (int)hipGetLastError();
}

// Rows per block of ln_bwd_kernel: ONE round of blocks over the chip (3 resident per CU at its
// ~150 VGPRs), each wave walking rows with the next row's loads in flight; at least 16 rows.
int ln_num_cus() {
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
int g_ln_rpb = 64;  // rk_ln_set_bwd_cfg: rows per block (0 = one round of blocks over the chip);
                    // 64: 5.1 TB/s on ViT's 25216 x 768 (bench/ln_probe.py; 16: 4.3, one round: 4.7)
int g_ln_pf = 1;    // next-row prefetch in ln_bwd_kernel
RK_API int rk_ln_set_bwd_cfg(int rpb, int pf) {
  if (rpb < 0 || (rpb > 0 && rpb % LN_W)) return (int)hipErrorInvalidValue;
  g_ln_rpb = rpb;
  g_ln_pf = pf != 0;
  return 0;
}
int ln_bwd_rpb(int64_t rows) {
  if (g_ln_rpb > 0) return g_ln_rpb;
  const int64_t slots = (int64_t)ln_num_cus() * 3;
  int64_t rpb = (rows + slots - 1) / slots;
  rpb = (rpb + LN_W - 1) / LN_W * LN_W;
  return (int)std::max<int64_t>(16, std::min<int64_t>(rpb, 1 << 20));
}

RK_API int64_t rk_ln_workspace(int64_t rows, int C) {
  const int64_t rpb = ln_bwd_rpb(rows);
  return ((rows + rpb - 1) / rpb) * 3 * C;  // up to three column partials per block (rk_ln_bwd)
}

// LayerNorm backward; dgamma/dbeta accumulated (+=). dt: x/dx dtype, dto: dy dtype.
// dsum (dtype dt) / dres (dtype dto) may be null: dx = LN_bwd(dy) [+ dsum], dres = dx
// dres_sum (f32 [C], optional, needs dres): = column sums of dres (the added branch's bias gradient;
// written, not accumulated); dres_acc (f32 [C], optional, needs dres_sum): += the same sums (that
// bias's persistent gradient, so its producer needs no add launch)
RK_API int rk_ln_bwd(int dt, int dto, const void* dy, const void* x, const float* g, const float* mean,
                     const float* rstd, void* dx, const void* dsum, void* dres, float* dgamma, float* dbeta,
                     float* dres_sum, float* dres_acc, int64_t rows, int C, float* ws, unsigned* counter,
                     hipStream_t s) {
  if ((dt == F16 && dto == BF16) || (dt == BF16 && dto == F16)) return (int)hipErrorInvalidValue;
  if (C % 4 || C > 64 * 4 * LN_MAXV || (dres_sum && !dres) || (dres_acc && !dres_sum)) return (int)hipErrorInvalidValue;
  const int rpb = ln_bwd_rpb(rows);
  const int grid = (int)((rows + rpb - 1) / rpb);
  const int nv = (C + 255) / 256;
  const int np = dres_sum ? 3 : 2;
  const size_t smem = (size_t)LN_W * np * C * sizeof(float);
#define RK_LB(T, TO, NV)                                                                                               \
  if (np == 3)                                                                                                         \
    ln_bwd_kernel<T, TO, NV, 3><<<grid, LN_T, smem, s>>>((const TO*)dy, (const T*)x, g, mean, rstd, (T*)dx,             \
                                                         (const T*)dsum, (TO*)dres, ws, rows, C, rpb, g_ln_pf);      \
  else                                                                                                                 \
    ln_bwd_kernel<T, TO, NV, 2><<<grid, LN_T, smem, s>>>((const TO*)dy, (const T*)x, g, mean, rstd, (T*)dx,             \
                                                         (const T*)dsum, (TO*)dres, ws, rows, C, rpb, g_ln_pf)
#define RK_LBN(T, TO)                 \
  if (nv <= 1) RK_LB(T, TO, 1);       \
  else if (nv <= 2) RK_LB(T, TO, 2);  \
  else if (nv <= 3) RK_LB(T, TO, 3);  \
  else if (nv <= 4) RK_LB(T, TO, 4);  \
  else if (nv <= 8) RK_LB(T, TO, 8);  \
  else RK_LB(T, TO, 16);
  if (dt == BF16 && dto == BF16) { RK_LBN(uint16_t, uint16_t) }
  else if (dt == F16 && dto == F16) { RK_LBN(f16_t, f16_t) }
  else if (dt == F16) { RK_LBN(f16_t, float) }
  else if (dto == F16) { RK_LBN(float, f16_t) }
  else if (dt == BF16) { RK_LBN(uint16_t, float) }
  else if (dto == BF16) { RK_LBN(float, uint16_t) }
  else { RK_LBN(float, float) }
#undef RK_LBN
#undef RK_LB
  if (dgamma || dbeta || dres_sum)
    colsum_kernel<<<(np * C + 63) / 64, CS_T, 0, s>>>(ws, grid, np * C, dgamma, dbeta, C, dres_sum, C / 4, dres_acc);
  (void)counter;
  return (int)hipGetLastError();
}
