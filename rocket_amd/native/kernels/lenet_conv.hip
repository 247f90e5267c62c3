// LeNet feature extractor on MFMA: conv(1->6,5x5,p2)+ReLU+pool2 -> conv(6->16,5x5)+ReLU+pool2,
// forward and backward, one wave per sample (replaces MIOpen igemm
// fwd/bwd/wrw + max_pool fwd/bwd + threshold_backward: 8 launches/step -> 2).
//
// Both convolutions are implicit GEMMs on v_mfma_f32_16x16x32_bf16 with the im2col operand
// gathered from an LDS-resident copy of the sample.  The M dimension (conv output
// positions) is ordered window-major: rows 4w..4w+3 of a 16-row tile are the four positions
// of pooling window w.  The MFMA C layout gives lane l rows (l>>4)*4 .. +3 of column l&15,
// so every lane holds one complete 2x2 window of one output channel and the max-pool,
// argmax, bias and ReLU happen in registers — the pre-pool activation never exists.
//
// Backward (one kernel): the pooled gradient is expanded through the 1-byte argmax/ReLU
// codes while building MFMA operands.
//   conv2 dgrad  dX2[pos,r] = dConv2[pos,co] . W2[co,r]   (16x16x16 MFMA, K = co = 16)
//                col2im by LDS f32 atomics into a per-wave dX2 image;
//   conv2 wgrad  dW2[co,r] += dConv2^T[co,pos] . im2col(a1)[pos,r]
//   conv1 wgrad  dW1[co,r] += dConv1^T[co,pos] . im2col(img)[pos,r], dConv1 = dX2 routed
//                through code1 — conv1's input gradient is never needed.
// Weight gradients accumulate in registers across the samples of a wave, are reduced across
// the block's waves through LDS and added to the persistent f32 gradients with one atomic
// per element per block.
#include "rk_common.h"

using namespace rk;

namespace {

constexpr int IMG = 28, PADI = 32, C1 = 6, KS = 5, Q1 = 14, C2 = 16, Q2 = 5;
constexpr int A1N = C1 * Q1 * Q1;  // 1176 conv1 pooled outputs per sample
constexpr int A2N = C2 * Q2 * Q2;  // 400
constexpr int R1 = KS * KS;        // 25  conv1 reduction
constexpr int R2 = C1 * KS * KS;   // 150 conv2 reduction

__device__ __forceinline__ __bf16 tobf(float v) { return (__bf16)v; }

// Intra-wave LDS producer/consumer ordering: drain this wave's LDS ops and stop the compiler
// from moving memory accesses across (lanes read what other lanes of the same wave wrote).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------------------ layout
// A block = 16 waves = 4 samples x 4 waves (sub-wave sw = wave & 3 splits each sample's
// tiles / k-steps), so 256 blocks of a 1024-sample batch put 4 waves on every SIMD.
// All gathers are branch-free: an invalid element reads a dedicated zero slot (a conditional
// load makes hipcc branch around it and wait lgkmcnt(0) per element).
constexpr int SPB = 4;               // samples per block
constexpr int WPS = 4;               // waves per sample
constexpr int NTHR = 64 * SPB * WPS; // 1024
constexpr int IMGZ = PADI * PADI;    // zero slot index in img

// padded-image offset of conv1 output position (window w of the 14x14 pool grid, quadrant q)
__device__ __forceinline__ int pos1(int w, int q) {
  const int wr = w / Q1, wc = w - wr * Q1;
  return (2 * wr + (q >> 1)) * PADI + 2 * wc + (q & 1);
}
// a1 offset of conv2 output position (window w of the 5x5 pool grid, quadrant q)
__device__ __forceinline__ int pos2(int w, int q) {
  const int wr = w / Q2, wc = w - wr * Q2;
  return (2 * wr + (q >> 1)) * Q1 + 2 * wc + (q & 1);
}

// ------------------------------------------------------------------------------ forward
struct FwdSmem {
  float img[SPB][PADI * PADI + 4];
  uint16_t a1[SPB][A1N + 8];  // zero slot at A1N, trash at A1N+4
  uint8_t c1[SPB][A1N + 8];
  uint16_t a2[SPB][A2N + 8];  // trash at A2N
  uint8_t c2[SPB][A2N + 8];
};

__global__ void __launch_bounds__(NTHR) lenet_conv_fwd(const float* __restrict__ x, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, uint16_t* __restrict__ a1g,
                                                       uint8_t* __restrict__ code1, uint16_t* __restrict__ a2g,
                                                       uint8_t* __restrict__ code2, int N) {
  __shared__ __attribute__((aligned(16))) FwdSmem sm;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = wave / WPS, sw = wave % WPS, st = threadIdx.x % (64 * WPS);  // st: thread in sample group
  const int n = blockIdx.x * SPB + slot;
  const bool live = n < N;
  const int nc = live ? n : 0;
  float* img = sm.img[slot];
  uint16_t* a1 = sm.a1[slot];
  uint8_t* c1 = sm.c1[slot];

  for (int i = st; i < PADI * PADI + 4; i += 64 * WPS) {
    const int r = (i >> 5) - 2, c = (i & 31) - 2;
    const bool in = i < PADI * PADI && r >= 0 && r < IMG && c >= 0 && c < IMG;
    const float v = x[(int64_t)nc * IMG * IMG + (in ? r * IMG + c : 0)];
    img[i] = in ? v : 0.f;
  }
  if (st < 8) a1[A1N + st] = 0;
  const int hi = lane >> 4, lo = lane & 15;
  bf16x8 bw1;
  int koff1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = 8 * hi + j;
    const bool ok = lo < C1 && r < R1;
    const float v = w1[ok ? lo * R1 + r : 0];
    bw1[j] = tobf(ok ? v : 0.f);
    koff1[j] = r < R1 ? (r / KS) * PADI + (r % KS) : -100000;
  }
  const float bias1 = b1[lo < C1 ? lo : 0];
  __syncthreads();

  // ---- conv1: 49 tiles of 16 rows (4 windows x 4 positions), split over the sample's 4 waves
  for (int t = sw; t < 49; t += WPS) {
    const int pos = pos1(4 * t + (lo >> 2), lo & 3);
    bf16x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = tobf(img[koff1[j] >= 0 ? pos + koff1[j] : IMGZ]);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw1, acc, 0, 0, 0);
    float m = acc[0];
    int arg = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      const bool gt = acc[i] > m;
      m = gt ? acc[i] : m;
      arg = gt ? i : arg;
    }
    m += bias1;
    const bool on = m > 0.f;
    const int o = lo < C1 ? lo * (Q1 * Q1) + 4 * t + hi : A1N + 4;
    a1[o] = f2bf(on ? m : 0.f);
    c1[o] = on ? (uint8_t)arg : 0xFF;
  }
  // conv2 operands (loaded here so their latency overlaps the barrier)
  bf16x8 bw2[5];
  int koff2[5][8];
#pragma unroll
  for (int s = 0; s < 5; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = 32 * s + 8 * hi + j;
      const float v = w2[lo * R2 + (r < R2 ? r : 0)];
      bw2[s][j] = tobf(r < R2 ? v : 0.f);
      koff2[s][j] = r < R2 ? (r / R1) * (Q1 * Q1) + ((r / KS) % KS) * Q1 + (r % KS) : -100000;
    }
  const float bias2 = b2[lo];
  __syncthreads();
  if (live) {
    for (int i = st * 8; i < A1N; i += 64 * WPS * 8) {
      *(uint4*)(a1g + (int64_t)n * A1N + i) = *(const uint4*)(a1 + i);
      *(uint2*)(code1 + (int64_t)n * A1N + i) = *(const uint2*)(c1 + i);
    }
  }

  // ---- conv2: 25 windows -> 7 tiles, split over the 4 waves
  for (int t = sw; t < 7; t += WPS) {
    const int w = 4 * t + (lo >> 2);
    const bool wvalid = w < Q2 * Q2;
    const int pos = pos2(wvalid ? w : 0, lo & 3);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ko = koff2[s][j];
        a[j] = __builtin_bit_cast(__bf16, a1[(wvalid && ko >= 0) ? pos + ko : A1N]);
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw2[s], acc, 0, 0, 0);
    }
    const int wq = 4 * t + hi;
    float m = acc[0];
    int arg = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      const bool gt = acc[i] > m;
      m = gt ? acc[i] : m;
      arg = gt ? i : arg;
    }
    m += bias2;
    const bool on = m > 0.f;
    const int o = wq < Q2 * Q2 ? lo * (Q2 * Q2) + wq : A2N;  // flatten order (C, H, W)
    sm.a2[slot][o] = f2bf(on ? m : 0.f);
    sm.c2[slot][o] = on ? (uint8_t)arg : 0xFF;
  }
  __syncthreads();
  if (live) {
    for (int i = st * 8; i < A2N; i += 64 * WPS * 8) {
      *(uint4*)(a2g + (int64_t)n * A2N + i) = *(const uint4*)(sm.a2[slot] + i);
      *(uint2*)(code2 + (int64_t)n * A2N + i) = *(const uint2*)(sm.c2[slot] + i);
    }
  }
}

// ------------------------------------------------------------------------------ backward
struct BwdSmem {
  float img[SPB][PADI * PADI + 4];  // + zero slot
  float dx2[SPB][A1N + 4];          // dL/d a1 (conv2 input gradient) + trash slot at A1N
  uint16_t a1[SPB][A1N + 8];        // + zero slot at A1N
  uint8_t c1[SPB][A1N + 8];         // + never-matching slot at A1N
  uint16_t da2[SPB][A2N + 8];
  uint8_t c2[SPB][A2N + 8];
  float gw2[C2 * R2 + 4];           // block-level weight-gradient accumulators (LDS atomics) + trash
  float gw1[C1 * R1 + 4];
  float gb2[C2];
  float gb1[C1 + 2];
  bf16x4 wfr[10 * 64];
};

__global__ void __launch_bounds__(NTHR) lenet_conv_bwd(const float* __restrict__ x, const uint16_t* __restrict__ a1g,
                                                       const uint8_t* __restrict__ code1g,
                                                       const uint16_t* __restrict__ da2g,
                                                       const uint8_t* __restrict__ code2g,
                                                       const float* __restrict__ w2, float* __restrict__ dw1,
                                                       float* __restrict__ db1, float* __restrict__ dw2,
                                                       float* __restrict__ db2, int N, int rounds) {
  __shared__ __attribute__((aligned(16))) BwdSmem sm;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = wave / WPS, sw = wave % WPS, st = threadIdx.x % (64 * WPS);
  const int hi = lane >> 4, lo = lane & 15;
  float* img = sm.img[slot];
  float* dx2 = sm.dx2[slot];
  uint16_t* a1 = sm.a1[slot];
  uint8_t* c1 = sm.c1[slot];
  uint16_t* da2 = sm.da2[slot];
  uint8_t* c2 = sm.c2[slot];

  for (int i = threadIdx.x; i < C2 * R2; i += NTHR) sm.gw2[i] = 0.f;
  for (int i = threadIdx.x; i < C1 * R1; i += NTHR) sm.gw1[i] = 0.f;
  if (threadIdx.x < C2) sm.gb2[threadIdx.x] = 0.f;
  if (threadIdx.x < C1) sm.gb1[threadIdx.x] = 0.f;
  if (st < 4) {
    img[PADI * PADI + st] = 0.f;
    a1[A1N + st] = 0;
    c1[A1N + st] = 0xFE;
    da2[A2N + st] = 0;
    c2[A2N + st] = 0xFE;
  }

  // conv2 dgrad operand B[k=co][col=r] = w2[co][r] (10 column tiles of 16, K = co = 16) kept in
  // LDS as bf16 in MFMA-fragment order: wfr[u][lane] = 4 consecutive co for column 16u + (lane&15)
  for (int i = threadIdx.x; i < 10 * 64; i += NTHR) {
    const int u = i >> 6, l = i & 63, r = 16 * u + (l & 15);
    bf16x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float f = w2[(4 * (l >> 4) + j) * R2 + (r < R2 ? r : 0)];
      v[j] = tobf(r < R2 ? f : 0.f);
    }
    sm.wfr[i] = v;
  }
  auto cofs_of = [&](int u) {
    const int r = 16 * u + lo;
    return r < R2 ? (r / R1) * (Q1 * Q1) + ((r / KS) % KS) * Q1 + (r % KS) : -100000;
  };
  int cw1[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = 16 * u + lo;
    cw1[u] = r < R1 ? (r / KS) * PADI + (r % KS) : -100000;
  }
  float sb2 = 0.f, sb1 = 0.f;

  for (int rd = 0; rd < rounds; ++rd) {
    const int n = (blockIdx.x * rounds + rd) * SPB + slot;
    const bool live = n < N;
    const int nc = live ? n : 0;
    __syncthreads();  // previous round's readers are done with the staging buffers
    // ---- stage (dead samples stage zero gradients: every wave runs the same barriers)
    for (int i = st; i < PADI * PADI; i += 64 * WPS) {
      const int r = (i >> 5) - 2, c = (i & 31) - 2;
      const bool in = r >= 0 && r < IMG && c >= 0 && c < IMG;
      const float v = x[(int64_t)nc * IMG * IMG + (in ? r * IMG + c : 0)];
      img[i] = in ? v : 0.f;
    }
    for (int i = st * 8; i < A1N; i += 64 * WPS * 8) {
      *(uint4*)(a1 + i) = *(const uint4*)(a1g + (int64_t)nc * A1N + i);
      *(uint2*)(c1 + i) = *(const uint2*)(code1g + (int64_t)nc * A1N + i);
    }
    for (int i = st; i < A1N + 4; i += 64 * WPS) dx2[i] = 0.f;
    for (int i = st * 8; i < A2N; i += 64 * WPS * 8) {
      uint4 d = *(const uint4*)(da2g + (int64_t)nc * A2N + i);
      if (!live) d = make_uint4(0, 0, 0, 0);
      *(uint4*)(da2 + i) = d;
      *(uint2*)(c2 + i) = *(const uint2*)(code2g + (int64_t)nc * A2N + i);
    }
    __syncthreads();

    // ---- conv2 dgrad: tiles t of 16 positions (4 windows); A[pos][co] = dConv2 (K = co = 16)
    for (int t = sw; t < 7; t += WPS) {
      const int w = 4 * t + (lo >> 2), q = lo & 3;
      const int wcl = w < Q2 * Q2 ? w : -1;
      bf16x4 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int idx = wcl >= 0 ? (4 * hi + j) * 25 + wcl : A2N;
        const float v = bf2f(da2[idx]);
        a[j] = tobf(c2[idx] == q ? v : 0.f);
      }
      const int wq = 4 * t + hi;
      const bool qvalid = wq < Q2 * Q2;
      const int base = pos2(qvalid ? wq : 0, 0);
#pragma unroll 2
      for (int u = 0; u < 10; ++u) {
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
        c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, sm.wfr[u * 64 + lane], c, 0, 0, 0);
        const int co = cofs_of(u);
        const bool ok = qvalid && co >= 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          atomicAdd(&dx2[ok ? base + (i >> 1) * Q1 + (i & 1) + co : A1N], c[i]);
      }
    }
    // ---- conv2 wgrad, k-step ks = sw (positions 32ks..32ks+31 = windows 8ks..8ks+7)
    {
      const int ks = sw;
      // this lane's 8 positions are windows wa = 8ks+2hi (j<4) and wa+1 (j>=4), quadrant j&3
      const int wa = 8 * ks + 2 * hi, wb = wa + 1;
      const bool va = wa < Q2 * Q2, vb = wb < Q2 * Q2;
      const int ia = va ? lo * 25 + wa : A2N, ib = vb ? lo * 25 + wb : A2N;
      const float da = bf2f(da2[ia]), db = bf2f(da2[ib]);
      const uint8_t ca = c2[ia], cb = c2[ib];
      const int pa = va ? pos2(wa, 0) : -100000, pb = vb ? pos2(wb, 0) : -100000;
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = j < 4 ? (ca == (j & 3) ? da : 0.f) : (cb == (j & 3) ? db : 0.f);
        a[j] = tobf(v);
        sb2 += v;
      }
#pragma unroll 2
      for (int u = 0; u < 10; ++u) {
        bf16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ofs = (j < 4 ? pa : pb) + ((j & 3) >> 1) * Q1 + (j & 1) + cofs_of(u);
          b[j] = __builtin_bit_cast(__bf16, a1[ofs >= 0 ? ofs : A1N]);
        }
        f32x4 g = {0.f, 0.f, 0.f, 0.f};
        g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, g, 0, 0, 0);
        const int col = 16 * u + lo;  // C rows = co (4hi+i), cols r = 16u + lo
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(&sm.gw2[col < R2 ? (4 * hi + i) * R2 + col : C2 * R2], g[i]);
      }
    }
    __syncthreads();  // all dX2 atomics of this sample are complete
    // ---- conv1 wgrad: k-steps ks = sw, sw+4, ... (windows 8ks..8ks+7 of 196)
    f32x4 g1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    for (int ks = sw; ks < 25; ks += WPS) {
      const int wa = 8 * ks + 2 * hi, wb = wa + 1;
      const bool va = lo < C1 && wa < Q1 * Q1, vb = lo < C1 && wb < Q1 * Q1;
      const int ia = va ? lo * 196 + wa : A1N, ib = vb ? lo * 196 + wb : A1N;
      const float da = dx2[ia], db = dx2[ib];
      const uint8_t ca = c1[ia], cb = c1[ib];
      const int pa = wa < Q1 * Q1 ? pos1(wa, 0) : -100000, pb = wb < Q1 * Q1 ? pos1(wb, 0) : -100000;
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = j < 4 ? (ca == (j & 3) ? da : 0.f) : (cb == (j & 3) ? db : 0.f);
        a[j] = tobf(v);
        sb1 += v;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        bf16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ofs = (j < 4 ? pa : pb) + ((j & 3) >> 1) * PADI + (j & 1) + cw1[u];
          b[j] = tobf(img[ofs >= 0 ? ofs : IMGZ]);
        }
        g1[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, g1[u], 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int col = 16 * u + lo;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = col < R1 && 4 * hi + i < C1;
        atomicAdd(&sm.gw1[ok ? (4 * hi + i) * R1 + col : C1 * R1], g1[u][i]);
      }
    }
  }

  // ---- block reduction in LDS (f32 atomics), then one global atomic per element
  sb2 += __shfl_xor(sb2, 16, 64);
  sb2 += __shfl_xor(sb2, 32, 64);
  sb1 += __shfl_xor(sb1, 16, 64);
  sb1 += __shfl_xor(sb1, 32, 64);
  if (hi == 0) {
    atomicAdd(&sm.gb2[lo], sb2);
    if (lo < C1) atomicAdd(&sm.gb1[lo], sb1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C2 * R2; i += NTHR) atomicAdd(dw2 + i, sm.gw2[i]);
  for (int i = threadIdx.x; i < C1 * R1; i += NTHR) atomicAdd(dw1 + i, sm.gw1[i]);
  if (threadIdx.x < C2 && db2) atomicAdd(db2 + threadIdx.x, sm.gb2[threadIdx.x]);
  if (threadIdx.x < C1 && db1) atomicAdd(db1 + threadIdx.x, sm.gb1[threadIdx.x]);
}

}  // namespace

RK_API int rk_lenet_conv_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                             void* a1, void* code1, void* a2, void* code2, int N, hipStream_t s) {
  const int grid = (N + SPB - 1) / SPB;
  lenet_conv_fwd<<<grid, NTHR, 0, s>>>(x, w1, b1, w2, b2, (uint16_t*)a1, (uint8_t*)code1, (uint16_t*)a2,
                                       (uint8_t*)code2, N);
  return (int)hipGetLastError();
}

// Gradients are ACCUMULATED (atomics) into dw1/db1/dw2/db2 (zeroed or persistent f32 buffers).
// `rounds`: samples groups of 4 processed per block (more rounds -> fewer global atomics).
RK_API int rk_lenet_conv_bwd(const float* x, const void* a1, const void* code1, const void* da2, const void* code2,
                             const float* w2, float* dw1, float* db1, float* dw2, float* db2, int N, int rounds,
                             hipStream_t s) {
  if (rounds < 1) rounds = 1;
  const int per_block = SPB * rounds;
  const int grid = (N + per_block - 1) / per_block;
  lenet_conv_bwd<<<grid, NTHR, 0, s>>>(x, (const uint16_t*)a1, (const uint8_t*)code1, (const uint16_t*)da2,
                                       (const uint8_t*)code2, w2, dw1, db1, dw2, db2, N, rounds);
  return (int)hipGetLastError();
}
