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

#include <cstdlib>

using namespace rk;

// 16-bit format of every activation / fragment / weight-gradient operand: bf16 (default) or, when
// this file is compiled with RK_LENET_H = 1 (the *_h.hip wrapper TU), IEEE fp16 for autocast fp16;
// the fp16 build's entry points carry an "_h" suffix.
#ifndef RK_LENET_H
#define RK_LENET_H 0
#endif
#if RK_LENET_H
#define RKL_NAME(n) n##_h
#else
#define RKL_NAME(n) n
#endif

namespace {

constexpr bool kH16 = RK_LENET_H;
__device__ __forceinline__ uint16_t c16(float v) { return kH16 ? f2h(v) : f2bf(v); }
__device__ __forceinline__ float d16(uint16_t v) { return kH16 ? h2f(v) : bf2f(v); }
__device__ __forceinline__ __bf16 e16(float v) { return __builtin_bit_cast(__bf16, c16(v)); }
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  typedef __attribute__((ext_vector_type(8))) _Float16 h8;
  if constexpr (kH16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

constexpr int IMG = 28, PADI = 32, C1 = 6, KS = 5, Q1 = 14, C2 = 16, Q2 = 5;
constexpr int A1N = C1 * Q1 * Q1;  // 1176 conv1 pooled outputs per sample
constexpr int A2N = C2 * Q2 * Q2;  // 400
constexpr int R1 = KS * KS;        // 25  conv1 reduction
constexpr int R2 = C1 * KS * KS;   // 150 conv2 reduction
constexpr int K1P = KS * 6;        // 30: conv1 reduction with kw padded to 6 (fused path: pair reads)

// Optional phase timeline (diagnostics): thread 0 of every block stamps s_memrealtime (100 MHz)
// at phase boundaries into trace[block][0..15]; RK_TRW stamps lane 0 of EVERY wave into
// trace[block][base + wave] (per-wave view of a phase).  A null trace pointer costs one uniform branch.
constexpr int kTraceStride = 48;
#define RK_TR(tr, k)                                                                              \
  do {                                                                                            \
    if ((tr) != nullptr && threadIdx.x == 0)                                                      \
      (tr)[(int64_t)blockIdx.x * kTraceStride + (k)] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#define RK_TRW(tr, base)                                                                          \
  do {                                                                                            \
    if ((tr) != nullptr && (threadIdx.x & 63) == 0)                                               \
      (tr)[(int64_t)blockIdx.x * kTraceStride + (base) + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// Elements (x, x+1) of a bf16 row held twice (c0[i] = v[i], c1[i] = v[i+1]): one aligned 4-byte
// LDS read from c0 at even x, from c1 at x - 1 for odd x.
__device__ __forceinline__ uint32_t pair_at(const uint16_t* c0, const uint16_t* c1, int x) {
  const uint16_t* p = (x & 1) ? c1 + (x - 1) : c0 + x;
  return *(const uint32_t*)p;
}

// Block barrier for LDS hand-offs only: waits for this wave's LDS ops, not its global loads
// (__syncthreads() also drains vmcnt, exposing the latency of prefetched operands at every phase
// boundary).  Global memory is never exchanged between the waves of a block here.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

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
// LDS row stride of the padded image, and the distance between its two copies (even / odd pair
// starts): 35 and IMGN + 16 make conv1's A-operand and the dW1 B-operand pair reads 1.4-way / 1.8-way
// by a model of the ds_read_b32 lane groups (33 and IMGN + 8: 2.4-way / 2.5-way)
constexpr int IMGS = PADI + 3;
constexpr int IMGN = PADI * IMGS;    // 1120
constexpr int IMGC = IMGN + 16;      // element distance of the two image copies
constexpr int NBC = IMGS - IMG;      // border columns of an interior row: 0, 1, 30 .. IMGS-1
constexpr int NBORD = 4 * IMGS + IMG * NBC;  // border elements (rows 0, 1, 30, 31 + interior columns)
constexpr int IMGZ = IMGN;           // zero slot index in img

// padded-image offset of conv1 output position (window w of the 14x14 pool grid, quadrant q)
__device__ __forceinline__ int pos1(int w, int q) {
  const int wr = w / Q1, wc = w - wr * Q1;
  return (2 * wr + (q >> 1)) * IMGS + 2 * wc + (q & 1);
}
// a1 offset of conv2 output position (window w of the 5x5 pool grid, quadrant q)
__device__ __forceinline__ int pos2(int w, int q) {
  const int wr = w / Q2, wc = w - wr * Q2;
  return (2 * wr + (q >> 1)) * Q1 + 2 * wc + (q & 1);
}

// ------------------------------------------------------------------------------ classifier
// fc1 400->120, fc2 120->84, fc3 84->10 fused into the conv kernels (one block = 4 samples, so an
// MFMA tile uses rows 0..3; the FLOPs are negligible, the point is one launch and no HBM round
// trip of the features).  Weights come from a fragment table built once per step by lenet_prep
// from the fp32 master weights: one 16-byte load per lane per MFMA, no per-block conversion.
//   forward  fragment (nt, ks)[lane] = W[16nt + lo][32ks + 8hi + j]     (B[k][n] = W[n][k])
//   dgrad    fragment (it, ks)[lane] = W[32ks + 8hi + j][16it + lo]     (B[k][n] = W[k][n])
constexpr int F0 = 400, F1 = 120, F2 = 84, F3 = 10;
constexpr int OFF_F1 = 0;                  // fc1 fwd: 8 n-tiles x 13 k-steps
constexpr int OFF_F2 = OFF_F1 + 8 * 13;    // fc2 fwd: 6 x 4
constexpr int OFF_F3 = OFF_F2 + 6 * 4;     // fc3 fwd: 1 x 3
constexpr int OFF_B3 = OFF_F3 + 1 * 3;     // fc3 dgrad: 6 n-tiles (84) x 1 k-step (10)
constexpr int OFF_B2 = OFF_B3 + 6 * 1;     // fc2 dgrad: 8 (120) x 3 (84)
constexpr int OFF_B1 = OFF_B2 + 8 * 3;     // fc1 dgrad: 25 (400) x 4 (120)
constexpr int OFF_C1 = OFF_B1 + 25 * 4;    // conv1 fwd B: 1 k-step (25 taps)
constexpr int OFF_C2 = OFF_C1 + 1;         // conv2 fwd B: 7 k-steps (25 taps x 8 padded channels)
constexpr int OFF_D2 = OFF_C2 + 7;         // conv2 dgrad weights, plain [tap 25][ci 8][co 16] (400 x 16 B of 13 x 1 KB)
constexpr int NFRAG = OFF_D2 + 13;         // 282 fragments x 64 lanes x 16 B
constexpr int A2P = 432;                   // LDS row of pooled conv2 output: data 0..399, zero 400..415, trash 424
constexpr int A2TRASH = 424;
constexpr int H1P = 136, H2P = 104, DYP = 40;

__global__ void __launch_bounds__(64) lenet_prep_kernel(const float* __restrict__ w1, const float* __restrict__ w2,
                                                        const float* __restrict__ w3, const float* __restrict__ cw1,
                                                        const float* __restrict__ cw2, bf16x8* __restrict__ frag) {
  const int f = blockIdx.x, lane = threadIdx.x, lo = lane & 15, hi = lane >> 4;
  bf16x8 v;
  if (f >= OFF_C1) {  // conv B fragments (the layouts the conv phases used to gather per block)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = 0.f;
      if (f == OFF_C1) {  // B[k = (kh, kw) = (k / 6, k % 6), kw padded 5 -> 6][col = co lo], k = 8hi + j
        const int k = 8 * hi + j, kh = k / 6, kw = k % 6;
        if (lo < C1 && k < K1P && kw < KS) x = cw1[lo * R1 + kh * KS + kw];
      } else if (f < OFF_D2) {  // B[k = (tap kk = 4s + hi, ci = j)][col = co lo]
        const int kk = 4 * (f - OFF_C2) + hi;
        if (kk < R1 && j < C1) x = cw2[(lo * C1 + j) * R1 + kk];
      } else {  // dgrad weights [kk][ci][co]: 16-byte unit u = (kk, ci, co half), see d2frag
        const int u = (f - OFF_D2) * 64 + lane, kk = u >> 4, ci = (u >> 1) & 7, co = 8 * (u & 1) + j;
        if (kk < R1 && ci < C1) x = cw2[(co * C1 + ci) * R1 + kk];
      }
      v[j] = e16(x);
    }
    frag[f * 64 + lane] = v;
    return;
  }
  const float* W;
  int nout, nin, tile, ks, bwd;
  if (f < OFF_F2) { W = w1; nout = F1; nin = F0; tile = (f - OFF_F1) / 13; ks = (f - OFF_F1) % 13; bwd = 0; }
  else if (f < OFF_F3) { W = w2; nout = F2; nin = F1; tile = (f - OFF_F2) / 4; ks = (f - OFF_F2) % 4; bwd = 0; }
  else if (f < OFF_B3) { W = w3; nout = F3; nin = F2; tile = 0; ks = f - OFF_F3; bwd = 0; }
  else if (f < OFF_B2) { W = w3; nout = F3; nin = F2; tile = f - OFF_B3; ks = 0; bwd = 1; }
  else if (f < OFF_B1) { W = w2; nout = F2; nin = F1; tile = (f - OFF_B2) / 3; ks = (f - OFF_B2) % 3; bwd = 1; }
  else { W = w1; nout = F1; nin = F0; tile = (f - OFF_B1) / 4; ks = (f - OFF_B1) % 4; bwd = 1; }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int a = bwd ? 32 * ks + 8 * hi + j : 16 * tile + lo;  // output-feature row of W
    const int b = bwd ? 16 * tile + lo : 32 * ks + 8 * hi + j;  // input-feature column of W
    const bool ok = a < nout && b < nin;
    v[j] = e16(ok ? W[a * nin + b] : 0.f);
  }
  frag[f * 64 + lane] = v;
}

// one MFMA tile of a 4-row classifier layer: rows = the block's samples (lanes lo < 4 read `act`,
// the rest a zero row), K-steps KS from LDS, B fragments from the table (all loads issued first)
template <int KS>
__device__ __forceinline__ f32x4 cls_tile(const uint16_t* act, int stride, const uint16_t* zrow,
                                          const bf16x8* __restrict__ frag, int fbase, int lane) {
  const int lo = lane & 15, hi = lane >> 4;
  const uint16_t* row = lo < SPB ? act + lo * stride : zrow;
  bf16x8 b[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) b[ks] = frag[(fbase + ks) * 64 + lane];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    acc = mfma16(*(const bf16x8*)(row + 32 * ks + 8 * hi), b[ks], acc);
  return acc;
}

// same with the B fragments already in registers (prefetched early by the caller)
template <int KS>
__device__ __forceinline__ f32x4 cls_tile_pre(const uint16_t* act, int stride, const uint16_t* zrow,
                                              const bf16x8 (&b)[KS], int lane) {
  const int lo = lane & 15, hi = lane >> 4;
  const uint16_t* row = lo < SPB ? act + lo * stride : zrow;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    acc = mfma16(*(const bf16x8*)(row + 32 * ks + 8 * hi), b[ks], acc);
  return acc;
}

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  return make_uint2((uint32_t)c16(a) | ((uint32_t)c16(b) << 16), (uint32_t)c16(c) | ((uint32_t)c16(d) << 16));
}

// Fused batch gather (a deferred device-loader batch, runtime/data.py PendingRows): sample n of
// the batch is dataset row rows[n] (staged by the previous step's tail / the loader); the step
// kernel reads the image / label rows through it and writes them into the batch buffers (x, ydst)
// for every later reader.  rows == null: x / the targets ARE the batch.
struct RowSrc {
  const int64_t* rows;
  const float* xsrc;    // dataset images [rows][784]
  const int64_t* ysrc;  // dataset labels [rows]
  int64_t* ydst;        // the batch's label buffer [N]
  const int64_t* target;  // labels of a batch that is not gathered (rows == null); keep != 0 only
  int keep;             // whole-step kernel: also stage the backward's inputs in KeepSmem (labels, dgrad fragments)
};

// ------------------------------------------------------------------------------ forward
constexpr int A1CL = Q1 * Q1 * 8;  // channel-last conv1 output: [pixel][8 channels], 6 used

// conv2 dgrad as an implicit GEMM whose 16 B columns are (d, ci) = (lo >> 3, lo & 7): TWO output
// pixels (ih, iw0 + d), iw0 even, per A row, so the A rows are the 98 pixel pairs of a sample and the
// K index runs over a 5 x 6 window (dy, dx) of dConv2 pixels x 16 channels: 480 -> 15 k-steps
// (with one output pixel per row and 16 columns for 6 channels: 13 tiles x 13 k-steps per sample;
// this form is 7 x 15, -38% MFMAs and A-operand LDS reads).  B[(dy, dx, co)][(d, ci)] =
// w2[co][ci][4 - dy][4 + d - dx] (0 where that kw is outside 0..4 or ci >= 6).
constexpr int K2P = 15;
constexpr int DGT = 7;              // dgrad row tiles per sample (98 pixel pairs -> 112 rows)

// B fragment element group of conv2-dgrad k-step s, lane l from the plain [kk][ci][co] table (16-byte
// units): lane (lo, hi) holds k = 32s + 8hi + j -> window position pi = 2s + hi/2 = (dy, dx) =
// (pi / 6, pi % 6), co = 8(hi & 1) + j; column lo = (d, ci).  Returns -1 for an all-zero fragment.
__device__ __forceinline__ int d2unit(int s, int l) {
  const int h = l >> 4, c = l & 15, pi = 2 * s + (h >> 1), dy = pi / 6, dx = pi % 6;
  const int d = c >> 3, ci = c & 7, kh = 4 - dy, kw = 4 + d - dx;
  return (kw >= 0 && kw < KS && ci < C1) ? ((kh * KS + kw) * 8 + ci) * 2 + (h & 1) : -1;
}

// The forward state the backward reuses.  Both phase layouts (FwdSmem, BwdSmem) START with it, so in
// the whole-step kernel (TrainSmem, a union of the two) the backward finds the staged image, the
// pooled conv1 output a1 and both argmax/ReLU code maps still in LDS: no global round trip (and no
// global copy of a1 / codes at all, which also shrinks the dirty bytes the kernel boundary writes back).
struct KeepSmem {
  uint16_t imgb[SPB][2][IMGC];      // bf16 image, two copies for pair reads (see BwdSmem)
  uint16_t a1[SPB][A1N + 8];        // fwd: zero slot at A1N, trash at A1N+4; bwd: zero / ones pairs there
  uint8_t c1[SPB][A1N + 8];         // bwd: never-matching slot at A1N
  uint8_t c2[SPB][A2P];             // same row pitch as a2: the trash slot A2TRASH must stay inside the row
  uint16_t h1[SPB][H1P];            // classifier activations (bf16; the backward's ReLU masks), zero K pads
  uint16_t h2[SPB][H2P];
  float logit[SPB][16];             // fp32 logits (the fused cross-entropy's input)
  int64_t label[SPB];               // the samples' targets
  bf16x8 wfr[K2P * 64];             // conv2-dgrad B fragments (loaded during the forward by the whole-step kernel)
};

struct FwdSmem {
  KeepSmem k;
  uint16_t a1cl[SPB][A1CL + 16];  // zero pixel at A1CL (8 zeros), trash lanes at A1CL+8
  uint16_t a2[SPB][A2P];  // data 0..399, zero pad 400..415, trash at A2TRASH
  uint16_t zrow[A2P];
};
static_assert(offsetof(FwdSmem, a1cl) % 16 == 0 && offsetof(FwdSmem, a2) % 16 == 0, "16-byte operand reads stay aligned");

struct ClsFwd {  // classifier operands of the fused forward
  const bf16x8* frag;
  const float *fb1, *fb2, *fb3;
  uint16_t *a2T, *h1T, *h2T;  // transposed activations [features][N] for the weight gradients
  float* logits;              // [N][10]
  uint64_t* trace;            // optional phase timeline [blocks][kTraceStride]
};

// The classifier backward's B fragments (fc3 / fc2 / fc1 dgrad), per wave.  The whole-step kernel
// issues their loads inside the forward, after fc1 (whose fragments are then dead), so their
// memory latency hides under fc2 / fc3 instead of opening the backward.
struct ClsBwdFrags {
  bf16x8 fb3, fb2[3], fb1[2][4];
};
__device__ __forceinline__ void load_cls_bwd23(const bf16x8* __restrict__ frag, int wave, int lane, ClsBwdFrags& f) {
  if (wave < 6) f.fb3 = frag[(OFF_B3 + wave) * 64 + lane];
  if (wave < 8) {
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) f.fb2[ks] = frag[(OFF_B2 + wave * 3 + ks) * 64 + lane];
  }
}
// fc1's (100 of the 130 KB per block): issued after fc3, so the 100 KB do not share fc2's phase
// with its own operand traffic (the vector-memory pipe, ~64 B/clk/CU, set fc2's length)
__device__ __forceinline__ void load_cls_bwd1(const bf16x8* __restrict__ frag, int wave, int lane, ClsBwdFrags& f) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = wave + 16 * u;
    if (t < 25) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) f.fb1[u][ks] = frag[(OFF_B1 + t * 4 + ks) * 64 + lane];
    }
  }
}

template <bool MLP>
__device__ __forceinline__ void fwd_body(FwdSmem& sm, const float* __restrict__ x, const float* __restrict__ w1,
                                         const float* __restrict__ b1, const float* __restrict__ w2,
                                         const float* __restrict__ b2, uint16_t* __restrict__ a1g,
                                         uint8_t* __restrict__ code1, uint16_t* __restrict__ a2g,
                                         uint8_t* __restrict__ code2, int N, ClsFwd cf, const RowSrc& rs,
                                         ClsBwdFrags* pre = nullptr, const bf16x8* bfrag = nullptr) {
  RK_TR(cf.trace, 0);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // conv B operands: the fused path loads the prep kernel's fragments first thing (one 16-byte
  // load per k-step, latency hidden behind the image staging); the generic path gathers them
  bf16x8 bw1, bw2[7];
  bf16x8 fr1[13], fr2[4], fr3[3];  // classifier B fragments (fused path), prefetched: their global
                                   // latency hides under the convolutions instead of after a barrier
  if constexpr (MLP) {
    bw1 = cf.frag[OFF_C1 * 64 + lane];
#pragma unroll
    for (int s = 0; s < 7; ++s) bw2[s] = cf.frag[(OFF_C2 + s) * 64 + lane];
  }
  const int slot = wave / WPS, sw = wave % WPS, st = threadIdx.x % (64 * WPS);  // st: thread in sample group
  const int n = blockIdx.x * SPB + slot;
  const bool live = n < N;
  const int nc = live ? n : 0;
  uint16_t* img0 = sm.k.imgb[slot][0];
  uint16_t* img1 = sm.k.imgb[slot][1];
  uint16_t* a1 = sm.k.a1[slot];
  uint8_t* c1 = sm.k.c1[slot];

  // the sample's 784 pixels as 196 float4 loads (one per thread), written at their padded
  // position (row stride IMGS, 2-pixel zero border) into both image copies; the 280 border /
  // zero-slot elements are written by the other threads (disjoint addresses: no ordering needed)
  {
    static_assert(64 * WPS >= IMG * IMG / 4, "one vector per thread");
    // fused gather: the sample's dataset row through the epoch table (two dependent loads), and
    // the row is written back into the batch buffer for the backward phase and later readers
    const int64_t srow = rs.rows ? rs.rows[nc] : (int64_t)nc;
    const float4* xs = (const float4*)((rs.rows ? rs.xsrc : x) + srow * IMG * IMG);
    float4 v4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (st < IMG * IMG / 4) {
      v4 = xs[st];
      // the batch buffer is only for later readers (the backward reuses the LDS image): streamed
      // out non-temporally, so it does not sit dirty in L2 at the kernel boundary
      if (rs.rows && live) {
        f32x4* const xd = (f32x4*)(const_cast<float*>(x) + (int64_t)n * IMG * IMG) + st;
        if (rs.keep & 2) *xd = f32x4{v4.x, v4.y, v4.z, v4.w};  // A/B knob ROCKET_LENET_X_PLAIN=1
        else __builtin_nontemporal_store(f32x4{v4.x, v4.y, v4.z, v4.w}, xd);
      }
    }
    if (st == IMG * IMG / 4 && (rs.rows || rs.keep)) {
      const int64_t lab = rs.rows ? rs.ysrc[srow] : (rs.target ? rs.target[nc] : 0);
      if (rs.rows && live) __builtin_nontemporal_store(lab, rs.ydst + n);
      if (rs.keep) sm.k.label[slot] = lab;
    }
    if constexpr (MLP) {
      if (rs.keep)  // the backward's conv2-dgrad fragments (its phase A then waits on no global load)
        for (int i = threadIdx.x; i < K2P * 64; i += NTHR) {
          const int u = d2unit(i >> 6, i & 63);
          sm.k.wfr[i] = u >= 0 ? cf.frag[OFF_D2 * 64 + u] : bf16x8{};
        }
    }
    for (int b = st; b < NBORD + 8; b += 64 * WPS) {  // border / zero-slot elements
      int bi;
      if (b < 4 * IMGS) {  // rows 0, 1, 30, 31
        const int r = b / IMGS;
        bi = (r < 2 ? r : r + IMG) * IMGS + b % IMGS;
      } else if (b < NBORD) {  // columns 0, 1, 30 .. IMGS-1 of rows 2..29
        const int u = b - 4 * IMGS, c5 = u % NBC;
        bi = (2 + u / NBC) * IMGS + (c5 < 2 ? c5 : c5 + IMG);
      } else {
        bi = IMGN + (b - NBORD);  // zero slots past the image
      }
      img0[bi] = 0;
      if (bi > 0) img1[bi - 1] = 0;
    }
    if (st < IMG * IMG / 4) {
      const int p = 4 * st, r = p / IMG, c = p - r * IMG;
      const int i = (r + 2) * IMGS + c + 2;
      const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint16_t u = c16(live ? vv[j] : 0.f);
        img0[i + j] = u;
        img1[i + j - 1] = u;
      }
    }
  }
  if (st < 8) a1[A1N + st] = 0;
  if (st < 16) sm.a1cl[slot][A1CL + st] = 0;
  if (MLP) {
    if (st < 32) sm.a2[slot][400 + st] = 0;  // K pad of fc1 (400..431; trash at 424 rewritten by conv2)
    for (int i = threadIdx.x; i < A2P; i += NTHR) sm.zrow[i] = 0;
  }
  const int hi = lane >> 4, lo = lane & 15;
  int koff1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = 8 * hi + j;
    if constexpr (!MLP) {
      const bool ok = lo < C1 && r < R1;
      const float v = w1[ok ? lo * R1 + r : 0];
      bw1[j] = e16(ok ? v : 0.f);
    }
    koff1[j] = r < R1 ? (r / KS) * IMGS + (r % KS) : -100000;
  }
  int koffp[4];  // fused path: pair q covers taps k = 8hi + 2q, +1 of the kw-padded-to-6 order
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 8 * hi + 2 * q;
    koffp[q] = k < K1P ? (k / 6) * IMGS + (k % 6) : -100000;
  }
  const float bias1 = b1[(lo & 7) < C1 ? (lo & 7) : 0];  // (lo & 7: the fused path's merged tile pairs)
  // every later layer's bias, issued now: its global-load latency hides behind conv1 instead of
  // stalling the conv2 / classifier epilogues (~1 us each after a barrier)
  const float bias2 = b2[lo];
  float fbias1 = 0.f, fbias2 = 0.f, fbias3 = 0.f;  // fc1 on waves 0-7, fc2 on 0-5, fc3 on wave 0
  if constexpr (MLP) {
    const int col = 16 * wave + lo;
    if (wave < 8) fbias1 = cf.fb1[col < F1 ? col : 0];
    if (wave < 6) fbias2 = cf.fb2[col < F2 ? col : 0];
    if (wave == 0) fbias3 = cf.fb3[lo < F3 ? lo : 0];
  }
  lds_barrier();
  RK_TR(cf.trace, 1);

  // ---- conv1: 49 tiles of 16 rows (4 windows x 4 positions), split over the sample's 4 waves;
  // U1 tiles per iteration: all their LDS gathers, then their MFMAs, then their epilogues (four
  // independent chains in flight instead of one read -> MFMA -> max -> store chain at a time)
  constexpr int U1 = 4;
  if constexpr (MLP) {
    // VALU-issue-bound phase (4 waves per SIMD): tiles are laid out so that every per-tile address
    // step is wave-uniform.  Wave sw owns pool-window columns 4sw .. 4sw+3 of all 14 pool rows (one
    // tile per row; columns 14, 15 of wave 3 are padding lanes whose outputs are not stored): moving
    // one pool row down is +2 image rows for every lane, so the 14 tiles' LDS reads and stores are
    // the lane's base address plus immediate offsets — no per-tile address arithmetic.  (The
    // 49-tile walk over consecutive windows spent ~15 VALU instructions per tile on window
    // wrap-around and addresses, half of the phase.)  56 tiles instead of 49; the epilogue is ~14
    // VALU instructions per tile.
    const int q4 = lo & 3;
    const int par = ((q4 >> 1) ^ q4) & 1;
    const int wl = 4 * sw + (lo >> 2);  // this lane's A row: window column wl, quadrant q4
    const int pos0 = (q4 >> 1) * IMGS + 2 * wl + (q4 & 1);  // pool row 0
    const char* pbq[4];  // per pair: the lane's LDS address in pool row 0
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // padded taps (k >= K1P) have zero B rows: any finite pair will do (the window's first pair)
      const int kp = koffp[q] >= 0 ? koffp[q] : 0;
      const int xp = par ^ (kp & 1);  // parity of pos + kp (pos0's parity is par; rows step by 66)
      pbq[q] = (const char*)(xp ? img1 - 1 + kp : img0 + kp) + 2 * pos0;
    }
    // Epilogue on merged tile PAIRS: an MFMA tile's columns are 16 channels of which 6 are real, so
    // the pool / ReLU / store sequence ran on 6 of 16 lanes.  Rows r and r + 1 are merged into one
    // register set first — lanes 8..15 take tile r + 1's channels 0..7 by one DPP row shift per
    // accumulator (row_shr:8 into banks 2-3) — and the sequence then runs once per pair.
    const int wo = 4 * sw + hi;  // this lane's output window column (C rows 4hi + i: its 4 quadrants)
    const int ch = lo & 7, rb = lo >> 3;  // merged lane: channel ch of pool row r + rb
    const bool st1 = ch < C1 && wo < Q1, st2 = wo < Q1;
    uint16_t* const a1p = a1 + (ch < C1 ? ch : 0) * (Q1 * Q1) + wo + rb * Q1;
    uint8_t* const c1p = c1 + (ch < C1 ? ch : 0) * (Q1 * Q1) + wo + rb * Q1;
    uint16_t* const clp = sm.a1cl[slot] + (wo + rb * Q1) * 8 + ch;
    const float bias1z = ch < C1 ? bias1 : 0.f;  // channels 6, 7 of the channel-last copy: relu(0) = 0
    static_assert(Q1 % 2 == 0 && U1 % 2 == 0, "pool rows in whole pairs");
#pragma unroll
    for (int r0 = 0; r0 < Q1; r0 += U1) {
      bf16x8 a[U1];
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        if (r0 + u < Q1) {
          const int ro = (r0 + u) * 2 * IMGS * 2;  // bytes: two image rows per pool row
          uint32_t w4[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) w4[q] = *(const uint32_t*)(pbq[q] + ro);
          a[u] = __builtin_bit_cast(bf16x8, make_uint4(w4[0], w4[1], w4[2], w4[3]));
        }
      }
      f32x4 acc[U1];
#pragma unroll
      for (int u = 0; u < U1; ++u)
        if (r0 + u < Q1) acc[u] = mfma16(a[u], bw1, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int u = 0; u < U1; u += 2) {
        if (r0 + u >= Q1) break;
        const int r = r0 + u;  // the pair's first pool row
        // (whole-vector bit casts: hipcc folds a bit cast of ONE element of a vector to element 0)
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const i32x4 ai = __builtin_bit_cast(i32x4, acc[u]), bi = __builtin_bit_cast(i32x4, acc[u + 1]);
        i32x4 mi;
#pragma unroll
        for (int i = 0; i < 4; ++i) mi[i] = __builtin_amdgcn_update_dpp(ai[i], bi[i], 0x118, 0xf, 0xc, false);
        const f32x4 mg = __builtin_bit_cast(f32x4, mi);
        // max over the window's 4 quadrants; code = first quadrant attaining it (strict > as before)
        float m = mg[0];
        int arg = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i) {
          const bool gt = mg[i] > m;
          m = gt ? mg[i] : m;
          arg = gt ? i : arg;
        }
        m += bias1z;
        const bool on = m > 0.f;
        const uint16_t v = c16(on ? m : 0.f);
        if (st1) {
          a1p[r * Q1] = v;
          c1p[r * Q1] = on ? (uint8_t)arg : 0xFF;
        }
        if (st2) clp[r * Q1 * 8] = v;
      }
    }
  } else {
    for (int t0 = sw; t0 < 49; t0 += U1 * WPS) {
      bf16x8 a[U1];
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        const int t = min(t0 + u * WPS, 48);  // past the end: a duplicate of tile 48, never stored
        const int pos = pos1(4 * t + (lo >> 2), lo & 3);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[u][j] = __builtin_bit_cast(__bf16, img0[koff1[j] >= 0 ? pos + koff1[j] : IMGZ]);
      }
      f32x4 acc[U1];
#pragma unroll
      for (int u = 0; u < U1; ++u) acc[u] = mfma16(a[u], bw1, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        const int t = t0 + u * WPS;
        if (t >= 49) break;  // wave-uniform
        float m = acc[u][0];
        int arg = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i) {
          const bool gt = acc[u][i] > m;
          m = gt ? acc[u][i] : m;
          arg = gt ? i : arg;
        }
        m += bias1;
        const bool on = m > 0.f;
        const int o = lo < C1 ? lo * (Q1 * Q1) + 4 * t + hi : A1N + 4;
        const uint16_t v = c16(on ? m : 0.f);
        a1[o] = v;
        c1[o] = on ? (uint8_t)arg : 0xFF;
        sm.a1cl[slot][lo < 8 ? (4 * t + hi) * 8 + lo : A1CL + 8] = lo < C1 ? v : (uint16_t)0;
      }
    }
  }
  RK_TRW(cf.trace, 16);  // per wave: conv1 tiles done
  if constexpr (MLP) {  // fc1 fragments (bw1 is dead now)
    if (wave < 8) {
#pragma unroll
      for (int ks = 0; ks < 13; ++ks) fr1[ks] = cf.frag[(OFF_F1 + wave * 13 + ks) * 64 + lane];
    }
  }
  // conv2 operands, reduction ordered k = (kh*5 + kw)*8 + ci (ci padded 6 -> 8): a lane's 8
  // consecutive k are the 8 channels of one pixel of the channel-last image = ONE 16-byte read.
  // 200 -> 7 k-steps; lane (hi) covers (kh,kw) pair kk = 4s + hi.
  RK_TR(cf.trace, 2);
  if constexpr (!MLP) {
#pragma unroll
    for (int s = 0; s < 7; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = 4 * s + hi;
        const bool ok = kk < R1 && j < C1;
        const float v = w2[ok ? (lo * C1 + j) * R1 + kk : 0];
        bw2[s][j] = e16(ok ? v : 0.f);
      }
  }
  lds_barrier();
  RK_TR(cf.trace, 3);
  if (live && a1g) {  // (null in the whole-step kernel: its backward reads them from LDS)
    for (int i = st * 8; i < A1N; i += 64 * WPS * 8) {
      *(uint4*)(a1g + (int64_t)n * A1N + i) = *(const uint4*)(a1 + i);
      *(uint2*)(code1 + (int64_t)n * A1N + i) = *(const uint2*)(c1 + i);
    }
  }

  RK_TR(cf.trace, 4);
  // ---- conv2: 25 windows -> 7 tiles, split over the 4 waves; a wave's two tiles (sw, sw + 4)
  // run as two interleaved 7-MFMA chains
  {
    const uint16_t* acl = sm.a1cl[slot];
    const bool two = sw + WPS < 7;  // wave-uniform
    // A rows of windows past the grid and k-steps of the padded taps (kk >= 25: zero B rows) read
    // some in-grid pixel instead of the zero pixel: those rows are never stored and those products
    // are zero, so no per-k-step select — the address is the lane's window base plus a per-k-step
    // lane constant (the selects and tap divisions were ~8 VALU instructions per MFMA)
    const uint16_t* wb[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = u ? (two ? sw + WPS : sw) : sw;
      const int w = 4 * t + (lo >> 2);
      wb[u] = acl + pos2(w < Q2 * Q2 ? w : 0, lo & 3) * 8;  // conv2 output position = pixel of a1
    }
    int toff2[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int kk = 4 * s + hi;
      toff2[s] = kk < R1 ? ((kk / KS) * Q1 + (kk % KS)) * 8 : 0;
    }
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 7; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[u] = mfma16(*(const bf16x8*)(wb[u] + toff2[s]), bw2[s], acc[u]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      const int t = sw + u * WPS;
      const int wq = 4 * t + hi;
      float m = acc[u][0];
      int arg = 0;
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        const bool gt = acc[u][i] > m;
        m = gt ? acc[u][i] : m;
        arg = gt ? i : arg;
      }
      m += bias2;
      const bool on = m > 0.f;
      const int o = wq < Q2 * Q2 ? lo * (Q2 * Q2) + wq : (MLP ? A2TRASH : A2N);  // flatten order (C, H, W)
      sm.a2[slot][o] = c16(on ? m : 0.f);
      sm.k.c2[slot][o] = on ? (uint8_t)arg : 0xFF;
    }
  }
  RK_TRW(cf.trace, 32);  // per wave: conv2 tiles done
  if constexpr (MLP) {  // fc2 / fc3 fragments (bw2 is dead now; fc1 hides their latency)
    if (wave < 6) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) fr2[ks] = cf.frag[(OFF_F2 + wave * 4 + ks) * 64 + lane];
    }
    if (wave == 0) {
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) fr3[ks] = cf.frag[(OFF_F3 + ks) * 64 + lane];
    }
  }
  lds_barrier();
  RK_TR(cf.trace, 5);
  if (live && code2) {
    for (int i = st * 8; i < A2N; i += 64 * WPS * 8) {
      if (!MLP) *(uint4*)(a2g + (int64_t)n * A2N + i) = *(const uint4*)(sm.a2[slot] + i);
      *(uint2*)(code2 + (int64_t)n * A2N + i) = *(const uint2*)(sm.k.c2[slot] + i);
    }
  }
  if constexpr (MLP) {
    // the host guarantees N % 8 == 0, so every block holds 4 live samples
    const int n0 = blockIdx.x * SPB;
    if (wave < 8) {  // fc1: n-tile = wave, 13 k-steps
      const f32x4 acc = cls_tile_pre<13>(&sm.a2[0][0], A2P, sm.zrow, fr1, lane);
      if (hi == 0) {
        const int col = 16 * wave + lo;
        const float bb = fbias1;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = col < F1 ? fmaxf(acc[i] + bb, 0.f) : 0.f;
          sm.k.h1[i][col] = c16(v[i]);
        }
        if (col < F1) *(uint2*)(cf.h1T + (int64_t)col * N + n0) = pack4(v[0], v[1], v[2], v[3]);
      }
    } else {  // meanwhile: a2^T for the fc1 weight gradient
      for (int f = threadIdx.x - 512; f < F0; f += 512)
        *(uint2*)(cf.a2T + (int64_t)f * N + n0) = make_uint2(
            (uint32_t)sm.a2[0][f] | ((uint32_t)sm.a2[1][f] << 16), (uint32_t)sm.a2[2][f] | ((uint32_t)sm.a2[3][f] << 16));
      if (threadIdx.x - 512 < SPB * 8) sm.k.h1[(threadIdx.x - 512) >> 3][128 + ((threadIdx.x - 512) & 7)] = 0;
    }
    lds_barrier();
    RK_TR(cf.trace, 6);
    if (wave < 6) {  // fc2: 6 n-tiles x 4 k-steps
      const f32x4 acc = cls_tile_pre<4>(&sm.k.h1[0][0], H1P, sm.zrow, fr2, lane);
      if (hi == 0) {
        const int col = 16 * wave + lo;
        const float bb = fbias2;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = col < F2 ? fmaxf(acc[i] + bb, 0.f) : 0.f;
          sm.k.h2[i][col] = c16(v[i]);
        }
        if (col < F2) *(uint2*)(cf.h2T + (int64_t)col * N + n0) = pack4(v[0], v[1], v[2], v[3]);
      }
    }
    // the backward's classifier fragments, issued once fc2 no longer waits on its own operands
    // (issued before fc2 they put vmcnt waits into fc2's chain: +0.8 us)
    if (pre) load_cls_bwd23(bfrag, wave, lane, *pre);
    lds_barrier();
    RK_TR(cf.trace, 7);
    if (wave == 0) {  // fc3: 1 n-tile x 3 k-steps -> fp32 logits
      const f32x4 acc = cls_tile_pre<3>(&sm.k.h2[0][0], H2P, sm.zrow, fr3, lane);
      if (hi == 0 && lo < F3) {
        const float bb = fbias3;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          cf.logits[(int64_t)(n0 + i) * F3 + lo] = acc[i] + bb;
          sm.k.logit[i][lo] = acc[i] + bb;
        }
      }
    }
    if (pre) load_cls_bwd1(bfrag, wave, lane, *pre);
    RK_TR(cf.trace, 8);
  }
}

template <bool MLP>
__global__ void __launch_bounds__(NTHR) lenet_conv_fwd(const float* __restrict__ x, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, uint16_t* __restrict__ a1g,
                                                       uint8_t* __restrict__ code1, uint16_t* __restrict__ a2g,
                                                       uint8_t* __restrict__ code2, int N, ClsFwd cf) {
  __shared__ __attribute__((aligned(16))) FwdSmem sm;
  fwd_body<MLP>(sm, x, w1, b1, w2, b2, a1g, code1, a2g, code2, N, cf, RowSrc{});
}

// ------------------------------------------------------------------------------ backward
// Output-owned decomposition (no LDS float atomics on shared addresses):
//  phase A  stage 4 samples; expand the pooled conv2 gradient into a dense, zero-ringed
//           dConv2 image [16][18][18] (bf16) through the argmax/ReLU codes
//  phase B  conv2 dgrad as a GATHER implicit GEMM: dX2[pixel][ci] = sum_{co,kh,kw}
//           dConv2[co][ih+4-kh][iw+4-kw] . W2[co][ci][kh][kw]  (7 pixel-pair tiles x 15 k-steps per
//           sample, see K2P, all 16 waves); every output element is written by exactly one lane
//  phase C  dW2: waves 0..9 one 16-column tile each (issued alongside phase B — it needs no dX2),
//           reducing over the 4 samples' positions in registers; then dW1 (2 column tiles) on all
//           16 waves over a share of the 4 x 784 positions
//  phase D  block totals -> one row of a per-block gradient slab (fused path; summed by the
//           weight-gradient launch) or global f32 atomics (generic path)
constexpr int DC = 18;             // dConv2 image side: 10 + 2*4 zero ring
// channel-last [y][x][co] with a row pitch of 19 pixels (608 B = 38 16-B slots, 6 mod 16): with the
// phase-B row order below every ds_read_b128 lane group of the dgrad A operand hits 16 distinct
// bank slots (18-pixel rows, 4 mod 16: 2.7-way on average, by a model of the b128 lane groups)
constexpr int DCR = (DC + 1) * C2;  // 304 elements per ring row
constexpr int DCN = DC * DCR;       // 5472
// (Measured round 5: two 8-channel planes with one-pixel-row tiles — conflict-free 256-byte operand
// reads — made phase B slower, 5.48 -> 5.72 us: the 4 extra tiles cost more than the conflicts.)
// row stride of dConv2^T [co][position] (100 used, zero padded): 288 B = 18 16-B slots (2 mod 16), so
// the dW2 A read's b128 lane groups (16 rows at one or two hi) hit 16 distinct slots (272 B: 2-way)
constexpr int DTS = 144;
// fused path: per-block conv-gradient slab row [dW1 150 | db1 6 | dW2 2400 | db2 16] (+pad)
constexpr int SL_W1 = 0, SL_B1 = SL_W1 + C1 * R1, SL_W2 = SL_B1 + C1, SL_B2 = SL_W2 + C2 * R2;
constexpr int SLABN = SL_B2 + C2;  // 2572
constexpr int SLABW = 2576;

// dx2 channel row: the 196 windows + zeros (phase C's last k-step reads up to 199); 202 = 10 mod 32
// keeps phase B's dx2 stores (rows = 2 image rows apart, channel lanes) and phase C's 8-byte reads
// conflict-free (200: 2.75-way stores)
constexpr int DX2S = Q1 * Q1 + 6;
// phase C's ones image: the ones column's B reads at the lane's offsets + the unrolled rows' immediates
constexpr int PC_ONES = 880;
struct BwdSmem {
  // k.imgb: bf16 image in two copies: [0][i] = img[i], [1][i] = img[i + 1], so any pair (x, x+1) is
  // ONE aligned 4-byte read (copy x & 1 at x & ~1) — the dW1 B operand is 4 pair reads per fragment.
  // Zero pair at [0][IMGZ].  k.a1 (+ zero slot at A1N), k.c1 (+ never-matching slot at A1N), k.c2.
  KeepSmem k;
  float dx2[SPB][C1 * DX2S];        // dL/d a1 (conv2 input gradient), channel rows of DX2S (zero tail)
  uint16_t ones[PC_ONES];           // phase C: 16-bit 1.0 everywhere (the db1 "ones column" reads it)
  uint16_t posT2[32];               // phase B (dW2): pos2(w, 0) of conv2 window w (w >= 25: clamped)
  uint16_t pad_a1o[78];             // places a1o at 46 mod 64 elements from a1 (see static_assert below)
  uint16_t a1o[SPB][A1N + 8];       // a1 shifted by one element (pair reads for the dW2 B operand)
  // (16-byte aligned: the pad before a1o must not shift the b128-read arrays from here on)
  alignas(16) uint16_t dc2[SPB][DCN + 16];  // dense channel-last dConv2 with zero ring
                                    // (after phase B: the 16 waves' dW1 partials [16][2][256] f32)
  uint16_t dcT[SPB][C2 * DTS];      // dConv2^T [co][p = 4*window + quadrant] (wgrad2 A operand)
  // fused classifier backward (MLP=true): gradients of the 4 samples as MFMA A rows
  uint16_t dyl[SPB][DYP];           // dlogits, K pad 10..39 zero
  uint16_t d2l[SPB][H2P];           // d(fc2 out) masked, pad 84..
  uint16_t d1l[SPB][H1P];           // d(fc1 out) masked, pad 120..
  uint16_t da2[SPB][A2N];           // d(pooled conv2 output)
  uint16_t zrow[H1P];
  float dyf[SPB][F3];               // fused CE: fp32 d(logits) of the block's samples
  float red[NTHR / 64];
  float lossp[SPB];
  float cecnt[NTHR / 64];  // fused CE: [0] the block's valid-target count
  int flag;
};
static_assert(sizeof(((BwdSmem*)nullptr)->dc2) >= (NTHR / 64) * 2 * 256 * sizeof(float),
              "dW1 partials alias dc2");
// The dW2 B operand reads pairs from a1 (even offsets) and a1o (odd ones) in one ds_read_b32: the
// distance between the two copies mod 64 elements (32 banks) sets how the two halves of a lane group
// collide; 46 measured best of all even distances by a model of the b32 lane groups (2.2-way -> 1.7-way).
static_assert(((offsetof(BwdSmem, a1o) - offsetof(BwdSmem, k.a1)) / 2) % 64 == 46, "a1o bank placement");
static_assert(offsetof(BwdSmem, dc2) % 16 == 0 && offsetof(BwdSmem, dcT) % 16 == 0 && offsetof(BwdSmem, dyl) % 16 == 0 &&
              offsetof(BwdSmem, d2l) % 16 == 0 && offsetof(BwdSmem, d1l) % 16 == 0 && offsetof(BwdSmem, da2) % 16 == 0 &&
              offsetof(BwdSmem, dx2) % 16 == 0 && offsetof(KeepSmem, wfr) % 16 == 0,
              "16-byte operand reads stay aligned");

struct ClsBwd {
  const bf16x8* frag;
  const float* dy;                  // dlogits [N][10] (already scaled by the upstream gradient)
  const uint16_t *h1T, *h2T;        // forward activations (ReLU masks)
  uint16_t *dyT, *d2T, *d1T;        // transposed gradients for the weight-gradient launch
  // fused softmax cross-entropy (ce != 0): d(logits) is derived here from the saved logits and
  // the targets instead of being read from `dy`; the mean loss is reduced across blocks
  // (last-block ticket) and folded into the Loss capsule's device accumulator / report ring.
  int ce;
  const float* logits;
  const int64_t* target;
  int64_t ignore_index;
  float grad_scale;
  float* partials;                  // [2][gridDim.x]: loss sums, valid-target counts
  unsigned* counter;
  float* loss_out;                  // [2]: loss, nvalid
  int defer_loss;                   // 1: store block partials + nvalid only; the wgrad launch finalises
  float *acc, *ring;
  int64_t* slot;
  int ring_size;
  float acc_scale;
  int sync;
  uint64_t* trace;                  // optional phase timeline [blocks][kTraceStride]
  float* slab;                      // [blocks][SLABW] conv weight/bias gradient partials
  const int64_t* row_table;         // fused gather: target of sample i = row_labels[row_table[i]]
  const int64_t* row_labels;
  const float* gscale_dev;          // optional device factor on d(logits) (the fp16 loss scale)
};

// RES (whole-step kernel only): the forward of this block left the image, a1 and both code maps in
// sm.k (KeepSmem), so phase A stages nothing from global memory and a1g / code1g / code2g are unused.
template <bool MLP, bool RES = false>
__device__ __forceinline__ void bwd_body(BwdSmem& sm, const float* __restrict__ x, const uint16_t* __restrict__ a1g,
                                         const uint8_t* __restrict__ code1g, const uint16_t* __restrict__ da2g,
                                         const uint8_t* __restrict__ code2g, const float* __restrict__ w2,
                                         float* __restrict__ dw1, float* __restrict__ db1, float* __restrict__ dw2,
                                         float* __restrict__ db2, int N, int rounds, ClsBwd cb,
                                         const ClsBwdFrags* pre = nullptr) {
  RK_TR(cb.trace, 0);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hi = lane >> 4, lo = lane & 15;

  // conv2-dgrad B operand (two output pixels per A row, see K2P): 15 k-steps kept in LDS in
  // fragment order (wfr[s*64 + lane]), one ds_read_b128 per k-step
  if constexpr (RES) {
    // staged by the forward (KeepSmem)
  } else if constexpr (MLP) {
    for (int i = threadIdx.x; i < K2P * 64; i += NTHR) {
      const int u = d2unit(i >> 6, i & 63);
      sm.k.wfr[i] = u >= 0 ? cb.frag[OFF_D2 * 64 + u] : bf16x8{};
    }
  } else
  for (int i = threadIdx.x; i < K2P * 64; i += NTHR) {
    const int u = d2unit(i >> 6, i & 63), kk = u >> 4, ci = (u >> 1) & 7;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int co = 8 * (u & 1) + j;
      const float f = w2[u >= 0 ? (co * C1 + ci) * R1 + kk : 0];
      v[j] = e16(u >= 0 ? f : 0.f);
    }
    sm.k.wfr[i] = v;
  }


  if (MLP)
    for (int i = threadIdx.x; i < H1P; i += NTHR) sm.zrow[i] = 0;
  if (MLP && cb.ce && threadIdx.x == 0) sm.lossp[0] = sm.cecnt[0] = 0.f;
  // fused path: the classifier dgrad B fragments and ReLU masks are loaded now, so the chain below
  // runs on registers and LDS only (each was one global round trip after a barrier)
  ClsBwdFrags fl;
  if constexpr (MLP) {
    if (pre) fl = *pre;
    else {
      load_cls_bwd23(cb.frag, wave, lane, fl);
      load_cls_bwd1(cb.frag, wave, lane, fl);
    }
  }
  const bf16x8& fb3 = fl.fb3;
  const bf16x8 (&fb2)[3] = fl.fb2;
  const bf16x8 (&fb1)[2][4] = fl.fb1;
  uint2 mk2 = make_uint2(0u, 0u), mk1 = make_uint2(0u, 0u);
  if constexpr (MLP) {
    const int nb = blockIdx.x * rounds * SPB;
    if (wave < 6) {
      const int col = 16 * wave + lo;
      if (RES) {
        if (hi == 0)
          mk2 = make_uint2((uint32_t)sm.k.h2[0][col] | ((uint32_t)sm.k.h2[1][col] << 16),
                           (uint32_t)sm.k.h2[2][col] | ((uint32_t)sm.k.h2[3][col] << 16));
      } else if (hi == 0) mk2 = *(const uint2*)(cb.h2T + (int64_t)(col < F2 ? col : 0) * N + nb);
    }
    if (wave < 8) {
      const int col = 16 * wave + lo;
      if (RES) {
        if (hi == 0)
          mk1 = make_uint2((uint32_t)sm.k.h1[0][col] | ((uint32_t)sm.k.h1[1][col] << 16),
                           (uint32_t)sm.k.h1[2][col] | ((uint32_t)sm.k.h1[3][col] << 16));
      } else if (hi == 0) mk1 = *(const uint2*)(cb.h1T + (int64_t)(col < F1 ? col : 0) * N + nb);
    }
  }

  const int nrounds = MLP ? 1 : rounds;  // fused variant: one round (no loop-invariant state to keep live)
  for (int rd = 0; rd < nrounds; ++rd) {
    const int nbase = (blockIdx.x * rounds + rd) * SPB;
    // fused cross-entropy operands, issued ahead of the conv staging loads (in-order vmcnt):
    // wave 0 holds one logit per lane (lane = 16 * sample + class).  The mean's 1/(valid targets)
    // is NOT applied here: d(logits) is scaled by 1/N only, every block reports its own valid
    // count, and the weight-gradient launch (which sums the counts) applies N / count to the
    // gradients and divides the loss — no block reads the whole batch's targets.
    int64_t ce_t = 0;
    float ce_x = 0.f;
    if (MLP && cb.ce) {
      if (wave == 0) {
        const int n = nbase + (lane >> 4), o = lane & 15;
        if constexpr (RES) {
          ce_t = sm.k.label[lane >> 4];
          ce_x = sm.k.logit[lane >> 4][o < F3 ? o : 0];
        } else {
          ce_t = cb.row_table ? cb.row_labels[cb.row_table[n]] : cb.target[n];
          ce_x = cb.logits[(int64_t)n * F3 + (o < F3 ? o : 0)];
        }
      }
    }
    if constexpr (MLP) lds_barrier();
    else __syncthreads();
    RK_TR(cb.trace, 1);
    // ---- phase A: stage.  Fused path: the image and a1 / code1 loads go to registers here and are
    // written to LDS after the classifier chain (their latency hides under it); the image border
    // and the dc2 / dcT zero fills need no loads and are written now.
    float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
    uint4 a1v = make_uint4(0u, 0u, 0u, 0u);
    uint2 c1v = make_uint2(0u, 0u);
    if constexpr (RES) {
      // everything is in LDS already (the image border zeros and zero slots included)
    } else if constexpr (MLP) {
      static_assert(SPB * IMG * IMG / 4 <= NTHR && SPB * (A1N / 8) <= NTHR, "one vector per thread");
      if (threadIdx.x < SPB * IMG * IMG / 4) {
        const int sl = threadIdx.x / (IMG * IMG / 4), v = threadIdx.x % (IMG * IMG / 4);
        xv = *(const float4*)(x + (int64_t)(nbase + sl) * IMG * IMG + 4 * v);
      }
      if (threadIdx.x < SPB * (A1N / 8)) {
        const int sl = threadIdx.x / (A1N / 8), e = (threadIdx.x % (A1N / 8)) * 8;
        a1v = *(const uint4*)(a1g + (int64_t)(nbase + sl) * A1N + e);
        c1v = *(const uint2*)(code1g + (int64_t)(nbase + sl) * A1N + e);
      }
      for (int t = threadIdx.x; t < SPB * NBORD; t += NTHR) {  // border of the padded image (rows/cols)
        const int sl = t / NBORD, b = t % NBORD;
        int bi;
        if (b < 4 * IMGS) {
          const int r = b / IMGS;
          bi = (r < 2 ? r : r + IMG) * IMGS + b % IMGS;
        } else {
          const int u = b - 4 * IMGS, c5 = u % NBC;
          bi = (2 + u / NBC) * IMGS + (c5 < 2 ? c5 : c5 + IMG);
        }
        sm.k.imgb[sl][0][bi] = 0;
        if (bi > 0) sm.k.imgb[sl][1][bi - 1] = 0;
      }
    } else
    for (int i = threadIdx.x; i < SPB * IMGN; i += NTHR) {
      const int sl = i / IMGN, e = i % IMGN;
      const int n = nbase + sl;
      const int r = e / IMGS - 2, c = e % IMGS - 2;
      const bool in = n < N && r >= 0 && r < IMG && c >= 0 && c < IMG;
      const float v = x[(int64_t)(n < N ? n : 0) * IMG * IMG + (in ? r * IMG + c : 0)];
      const uint16_t u = c16(in ? v : 0.f);
      sm.k.imgb[sl][0][e] = u;
      if (e > 0) sm.k.imgb[sl][1][e - 1] = u;
    }
    if (!MLP)
    for (int i = threadIdx.x; i < SPB * (A1N / 8); i += NTHR) {
      const int sl = i / (A1N / 8), e = (i % (A1N / 8)) * 8;
      const int n = nbase + sl, nc = n < N ? n : 0;
      const uint4 v = *(const uint4*)(a1g + (int64_t)nc * A1N + e);
      *(uint4*)(sm.k.a1[sl] + e) = v;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // a1o[e - 1 + j] = a1[e + j]
        if (e + 2 * k > 0) sm.a1o[sl][e + 2 * k - 1] = (uint16_t)(w[k] & 0xffff);
        sm.a1o[sl][e + 2 * k] = (uint16_t)(w[k] >> 16);
      }
      *(uint2*)(sm.k.c1[sl] + e) = *(const uint2*)(code1g + (int64_t)nc * A1N + e);
    }
    // zero dc2 / dcT (16-byte stores over each array as one flat range: no per-store division);
    // with the fused cross-entropy, waves 1.. do it while wave 0 runs the softmax below
    static_assert(sizeof(sm.dc2) % 16 == 0 && sizeof(sm.dcT) % 16 == 0, "whole 16-byte stores");
    {
      const bool ce_wave0 = MLP && cb.ce;
      if (!ce_wave0 || wave > 0) {
        const int t0 = ce_wave0 ? (int)threadIdx.x - 64 : (int)threadIdx.x, nt = ce_wave0 ? NTHR - 64 : NTHR;
        for (int i = t0; i < (int)(sizeof(sm.dc2) / 16); i += nt) ((uint4*)&sm.dc2[0][0])[i] = make_uint4(0, 0, 0, 0);
        for (int i = t0; i < (int)(sizeof(sm.dcT) / 16); i += nt) ((uint4*)&sm.dcT[0][0])[i] = make_uint4(0, 0, 0, 0);
      }
    }
    RK_TR(cb.trace, 2);
    // the classifier chain runs while the conv operands above are still in flight
    if constexpr (MLP) {
      // ---- classifier input-gradient chain (host guarantees N % 8 == 0: 4 live samples)
      if (cb.ce) {
        // softmax cross-entropy backward in-kernel; d(logits) kept unnormalised in LDS until the
        // valid-target count (reduced by the other waves meanwhile) is known
        if (wave == 0) {
          const int sl = lane >> 4, o = lane & 15;
          const bool valid = ce_t != cb.ignore_index, oc = o < F3;
          // row reductions on the DPP network (each sample's 16 logits are one 16-lane row): the
          // ds_bpermute shuffles were ten LDS round trips in a row on the step's critical path
          const float mx = row16_max(oc ? ce_x : -INFINITY);
          const float e = oc ? __expf(ce_x - mx) : 0.f;
          const float se = row16_sum(e), xt = row16_sum((oc && (int64_t)o == ce_t) ? ce_x : 0.f);
          if (oc) sm.dyf[sl][o] = valid ? e / se - ((int64_t)o == ce_t ? 1.f : 0.f) : 0.f;
          // lanes 0/16/32/48: a sample's loss and valid count -> the block's sums (wave-uniform)
          const float li = rows4_sum((o == 0 && valid) ? mx + __logf(se) - xt : 0.f);
          const float ci = rows4_sum((o == 0 && valid) ? 1.f : 0.f);
          if (lane == 0) {  // block running sums over rounds (LDS: no live register)
            sm.lossp[0] += li;
            sm.cecnt[0] += ci;
          }
        }
        lds_barrier();
        RK_TR(cb.trace, 3);
        if (threadIdx.x < SPB * DYP || (threadIdx.x >= 256 && threadIdx.x < 256 + F3)) {
          // pre-normalised by the batch size (keeps the gradients' magnitudes, and so their bf16
          // rounding, those of the mean); the weight-gradient launch applies N / (valid count)
          const float sc = cb.grad_scale / (float)N * (cb.gscale_dev ? *cb.gscale_dev : 1.f);
          if (threadIdx.x < SPB * DYP) {
            const int sl = threadIdx.x / DYP, o = threadIdx.x % DYP;
            sm.dyl[sl][o] = c16(o < F3 ? sc * sm.dyf[sl][o] : 0.f);
          } else {
            const int o = threadIdx.x - 256;
            *(uint2*)(cb.dyT + (int64_t)o * N + nbase) =
                pack4(sc * sm.dyf[0][o], sc * sm.dyf[1][o], sc * sm.dyf[2][o], sc * sm.dyf[3][o]);
          }
        }
        lds_barrier();
      } else {
        if (threadIdx.x < SPB * DYP) {
          const int sl = threadIdx.x / DYP, o = threadIdx.x % DYP;
          sm.dyl[sl][o] = c16(o < F3 ? cb.dy[(int64_t)(nbase + sl) * F3 + o] : 0.f);
        } else if (threadIdx.x >= 256 && threadIdx.x < 256 + F3) {
          const int o = threadIdx.x - 256;
          const float* d = cb.dy + (int64_t)nbase * F3 + o;
          *(uint2*)(cb.dyT + (int64_t)o * N + nbase) = pack4(d[0], d[F3], d[2 * F3], d[3 * F3]);
        }
        lds_barrier();
      RK_TR(cb.trace, 4);
      }
      if (wave < 6) {  // fc3 dgrad: d2 = (dy W3) * [h2 > 0]
        const bf16x8 fb3a[1] = {fb3};
        const f32x4 acc = cls_tile_pre<1>(&sm.dyl[0][0], DYP, sm.zrow, fb3a, lane);
        if (hi == 0) {
          const int col = 16 * wave + lo;
          const uint2 m = mk2;
          const float mk[4] = {d16(m.x & 0xffff), d16(m.x >> 16), d16(m.y & 0xffff), d16(m.y >> 16)};
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = (col < F2 && mk[i] > 0.f) ? acc[i] : 0.f;
            sm.d2l[i][col] = c16(v[i]);
          }
          if (col < F2) *(uint2*)(cb.d2T + (int64_t)col * N + nbase) = pack4(v[0], v[1], v[2], v[3]);
        }
      }
      lds_barrier();
      RK_TR(cb.trace, 5);
      if (wave < 8) {  // fc2 dgrad: d1 = (d2 W2) * [h1 > 0]
        const f32x4 acc = cls_tile_pre<3>(&sm.d2l[0][0], H2P, sm.zrow, fb2, lane);
        if (hi == 0) {
          const int col = 16 * wave + lo;
          const uint2 m = mk1;
          const float mk[4] = {d16(m.x & 0xffff), d16(m.x >> 16), d16(m.y & 0xffff), d16(m.y >> 16)};
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = (col < F1 && mk[i] > 0.f) ? acc[i] : 0.f;
            sm.d1l[i][col] = c16(v[i]);
          }
          if (col < F1) *(uint2*)(cb.d1T + (int64_t)col * N + nbase) = pack4(v[0], v[1], v[2], v[3]);
        }
      }
      lds_barrier();
      RK_TR(cb.trace, 6);
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // fc1 dgrad: da2 = d1 W1 (400 outputs = 25 tiles)
        const int t = wave + 16 * u;
        if (t < 25) {
          const f32x4 acc = cls_tile_pre<4>(&sm.d1l[0][0], H1P, sm.zrow, fb1[u], lane);
          if (hi == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) sm.da2[i][16 * t + lo] = c16(acc[i]);
          }
        }
      }
      if constexpr (RES) {
        // a1o (a1 shifted by one element) from the LDS-resident a1
        if (threadIdx.x < SPB * (A1N / 8)) {
          const int sl = threadIdx.x / (A1N / 8), e = (threadIdx.x % (A1N / 8)) * 8;
          const uint4 v = *(const uint4*)(sm.k.a1[sl] + e);
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {  // a1o[e - 1 + j] = a1[e + j]
            if (e + 2 * k > 0) sm.a1o[sl][e + 2 * k - 1] = (uint16_t)(w[k] & 0xffff);
            sm.a1o[sl][e + 2 * k] = (uint16_t)(w[k] >> 16);
          }
        }
      } else {
      // the staged conv operands, loaded before the chain
      if (threadIdx.x < SPB * IMG * IMG / 4) {
        const int sl = threadIdx.x / (IMG * IMG / 4), p = 4 * (threadIdx.x % (IMG * IMG / 4));
        const int r = p / IMG, c = p - r * IMG;
        const int i = (r + 2) * IMGS + c + 2;
        const float vv[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint16_t u = c16(vv[j]);
          sm.k.imgb[sl][0][i + j] = u;
          sm.k.imgb[sl][1][i + j - 1] = u;
        }
      }
      if (threadIdx.x < SPB * (A1N / 8)) {
        const int sl = threadIdx.x / (A1N / 8), e = (threadIdx.x % (A1N / 8)) * 8;
        *(uint4*)(sm.k.a1[sl] + e) = a1v;
        const uint32_t w[4] = {a1v.x, a1v.y, a1v.z, a1v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // a1o[e - 1 + j] = a1[e + j]
          if (e + 2 * k > 0) sm.a1o[sl][e + 2 * k - 1] = (uint16_t)(w[k] & 0xffff);
          sm.a1o[sl][e + 2 * k] = (uint16_t)(w[k] >> 16);
        }
        *(uint2*)(sm.k.c1[sl] + e) = c1v;
      }
      }
    }
    lds_barrier();
    RK_TR(cb.trace, 7);
    if (threadIdx.x < SPB * C1 * 4)  // dx2 zero tails (phase B writes windows < 196 only)
      sm.dx2[threadIdx.x / (C1 * 4)][(threadIdx.x / 4) % C1 * DX2S + Q1 * Q1 + (threadIdx.x & 3)] = 0.f;
    if (threadIdx.x >= NTHR - 32) {  // phase B's (dW2) window -> a1 offset table
      const int w = threadIdx.x - (NTHR - 32);
      sm.posT2[w] = (uint16_t)pos2(min(w, Q2 * Q2 - 1), 0);
    }
    for (int i = threadIdx.x; i < PC_ONES; i += NTHR) sm.ones[i] = (uint16_t)(kH16 ? 0x3C00 : 0x3F80);
    // scatter the pooled gradients: thread e owns pooled element (co, w) of all SPB samples, so its
    // index arithmetic (divisions by 25 and 5) is done once, not once per (sample, element)
    static_assert(A2N <= NTHR, "one pooled element per thread");
    if (threadIdx.x < A2N) {
      const int e = threadIdx.x, co = e / 25, w = e % 25;
      const int d0 = (2 * (w / Q2) + 4) * DCR + (2 * (w % Q2) + 4) * C2 + co, t0 = co * DTS + 4 * w;
#pragma unroll
      for (int sl = 0; sl < SPB; ++sl) {
        const int n = nbase + sl, nc = n < N ? n : 0;
        const uint16_t g = MLP ? sm.da2[sl][e] : da2g[(int64_t)nc * A2N + e];
        const uint8_t cd = RES ? sm.k.c2[sl][e] : code2g[(int64_t)nc * A2N + e];
        if (n < N && cd < 4) {
          sm.dc2[sl][d0 + (cd >> 1) * DCR + (cd & 1) * C2] = g;
          sm.dcT[sl][t0 + cd] = g;
        }
      }
    }
    if (threadIdx.x < SPB * 8) {
      const int sl = threadIdx.x >> 3, k = threadIdx.x & 7;
      // zero pair at [0..1], 16-bit ones pair at [2..3]: the B operand of the "ones column" whose
      // MFMA output is the bias gradient (row sums of the A operand)
      const uint16_t zo = (k == 2 || k == 3) ? (uint16_t)(kH16 ? 0x3C00 : 0x3F80) : (uint16_t)0;  // 16-bit 1.0
      sm.k.a1[sl][A1N + k] = zo;
      sm.a1o[sl][A1N - 1 + k] = 0;
      sm.k.c1[sl][A1N + k] = 0xFE;
      sm.k.imgb[sl][0][IMGN + k] = zo;
      sm.k.imgb[sl][1][IMGN - 1 + k] = 0;
    }
    lds_barrier();
    RK_TR(cb.trace, 8);

    // ---- phase B: conv2 dgrad (4 samples x 7 pixel-pair tiles) and dW2 (10 column tiles), which
    // needs only dcT and a1: 38 work items (the dW2 tiles, then the dgrad tiles) dealt round-robin,
    // item w + 16i to wave w: waves 0..5 a dW2 tile + 2 dgrad tiles, 6..9 a dW2 tile + 1, 10..15 2.  Per-lane address offsets are hoisted out of the tile loops (the phase is
    // VALU-issue-bound, not MFMA- or LDS-bound), and the bias gradients come out of the MFMAs as
    // "ones columns" (B column r = R2 of dW2 / r = R1 of dW1 is all ones -> C = row sums of A).
    f32x4 g2 = {0.f, 0.f, 0.f, 0.f};         // waves 0..9: dW2 tile u = wave (col r = 150: db2)
    if (wave < 10) {
      // dW2 tile u = wave: rows co (16), cols r = 16u + lo; K = positions of 4 samples (4 x 4 k-steps)
      const int u = wave;
      const int r = 16 * u + lo;
      // B element j of k-step ks at a1 offset (j<4 ? pa : pb) + ((j&3)>>1)*Q1 + (j&1): 4 pairs,
      // each one aligned 4-byte read from a1 (even x) or a1o (odd x), relative to sample 0's a1.
      // pos2(w, 0) and Q1 are even, so a pair's copy (x & 1) is that of the lane's column offset
      // alone: x = posT2[w] + a lane constant per (k & 1).  Columns r > 150 are never stored and
      // windows >= 25 meet zero A values (dcT's zero padding), so they read any in-range pair; the
      // ones column r = 150 (db2) reads the ones pair whatever the window (multiplier 0).
      constexpr int A1O = (int)(offsetof(BwdSmem, a1o) - offsetof(BwdSmem, k.a1)) / 2;
      const int rc = r < R2 ? r : R2 - 1;
      const int cof = (rc / R1) * (Q1 * Q1) + ((rc / KS) % KS) * Q1 + (rc % KS);
      const int wmul = r == R2 ? 0 : 1;
      int cst2[2];
#pragma unroll
      for (int k1 = 0; k1 < 2; ++k1) {
        const int c = cof + k1 * Q1;
        cst2[k1] = r == R2 ? A1N + 2 : ((c & 1) ? A1O + c - 1 : c);
      }
      const uint16_t* pt2 = sm.posT2 + 2 * hi;
      int pofs[4][4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int k = 0; k < 4; ++k) pofs[ks][k] = (int)pt2[8 * ks + (k >> 1)] * wmul + cst2[k & 1];
      const uint16_t* a1b = &sm.k.a1[0][0];
      // 16 k-steps (4 samples x 4), operands of step i + 1 read before step i's MFMA
      auto ld_a = [&](int i) {  // A[co = lo][p]
        return *(const bf16x8*)(sm.dcT[i >> 2] + lo * DTS + 32 * (i & 3) + 8 * hi);
      };
      auto ld_b = [&](int i) {
        const uint16_t* a1s = a1b + (i >> 2) * (A1N + 8);
        const int ks = i & 3;
        return make_uint4(*(const uint32_t*)(a1s + pofs[ks][0]), *(const uint32_t*)(a1s + pofs[ks][1]),
                          *(const uint32_t*)(a1s + pofs[ks][2]), *(const uint32_t*)(a1s + pofs[ks][3]));
      };
      bf16x8 a_cur = ld_a(0);
      uint4 b_cur = ld_b(0);
#pragma unroll
      for (int i = 0; i < 4 * SPB; ++i) {
        bf16x8 a_nxt = a_cur;
        uint4 b_nxt = b_cur;
        if (i + 1 < 4 * SPB) {
          a_nxt = ld_a(i + 1);
          b_nxt = ld_b(i + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        g2 = mfma16(a_cur, __builtin_bit_cast(bf16x8, b_cur), g2);
        a_cur = a_nxt;
        b_cur = b_nxt;
      }
    }
    RK_TRW(cb.trace, 16);  // per wave: dW2 tile done
    {
      constexpr int NDG = SPB * DGT;  // dgrad tiles = work items 10 .. 37
      const int t_begin = wave >= 10 ? wave - 10 : wave + 6;
      // fused path: this lane's B fragments read from LDS once per wave, not once per tile (the
      // generic multi-round variant keeps re-reading them: registers would spill there)
      bf16x8 wr[MLP ? K2P : 1];
      if constexpr (MLP) {
#pragma unroll
        for (int s = 0; s < K2P; ++s) wr[s] = sm.k.wfr[s * 64 + lane];
      }
      // A row = pixel pair (ih, iw0 = 2jx .. +1) reads the (ring) dConv2 pixels (ih + dy, iw0 + dx):
      // k-step s covers window positions 2s, 2s + 1 = (dy, dx) = (s / 3, 2(s % 3) + hi / 2), channels
      // 8(hi & 1) ..: the lane part is 8hi elements, the rest an immediate per k-step
      auto toff = [](int s) { return (s / 3) * DCR + 2 * (s % 3) * C2; };
      // Tile t = pair column jx = t (iw0 = 2t); row r -> ih: rows {0-3, 12-15} -> 0..7, rows 4..11 ->
      // 8..15 (14, 15: pad rows, re-reading 6, 7, never stored).  A b128 lane group is one of those
      // row classes at one hi: 8 rows at slots 6ih + const mod 16 (distinct even slots for 8
      // consecutive ih) and 8 rows of the other class at odd ones.
      auto row_ih = [](int r) { return (r >= 4 && r < 12) ? r + 4 : (r < 4 ? r : r - 8); };
      for (int tt = t_begin; tt < NDG; tt += 16) {
        const int sl = tt / DGT, t = tt % DGT;
        const int ihr = row_ih(lo), ih = ihr < Q1 ? ihr : ihr - 8;
        const uint16_t* ab = sm.dc2[sl] + ih * DCR + 2 * t * C2 + 8 * hi;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        // A operands in chunks of 4 k-steps, the next chunk's LDS reads issued before this
        // chunk's MFMAs (one read + wait per MFMA would expose the LDS latency every step)
        constexpr int CH = 4, NCH = (K2P + CH - 1) / CH;
        bf16x8 abuf[2][CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) abuf[0][q] = *(const bf16x8*)(ab + toff(q));
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          if (c + 1 < NCH) {
#pragma unroll
            for (int q = 0; q < CH; ++q)
              if ((c + 1) * CH + q < K2P) abuf[(c + 1) & 1][q] = *(const bf16x8*)(ab + toff((c + 1) * CH + q));
          }
          __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this chunk's MFMAs
#pragma unroll
          for (int q = 0; q < CH; ++q) {
            const int s = c * CH + q;
            if (s < K2P) {
              if constexpr (MLP) acc = mfma16(abuf[c & 1][q], wr[s], acc);
              else acc = mfma16(abuf[c & 1][q], sm.k.wfr[s * 64 + lane], acc);
            }
          }
        }
        // C[row 4hi + i][col = (d, ci) = (lo >> 3, lo & 7)] -> pixel (ih(row), 2t + d)
        if ((lo & 7) < C1) {
          float* dst = sm.dx2[sl] + (lo & 7) * DX2S + (lo >> 3) + 2 * t;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = row_ih(4 * hi + i);
            if (r < Q1) dst[r * Q1] = acc[i];
          }
        }
      }
    }
    RK_TRW(cb.trace, 32);  // per wave: dgrad tiles done
    lds_barrier();
    RK_TR(cb.trace, 9);

    // ---- phase C: dW1 on all 16 waves over the positions of the 14x14 pool grid; column r = 25 of
    // tile u = 1 is the ones column (db1)
    f32x4 g1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    {
      // Wave = (sample wave & 3, h0 = wave / 4): k-step j covers pool row r0 + 2j (r0 = h0 >> 1) and
      // the 8 window columns 8*half + 2hi, +1 of lane group hi (half = h0 & 1; columns 14, 15 are
      // padding: zero A).  Every address is then a lane constant plus a compile-time offset of the
      // unrolled row loop — no per-step address arithmetic (the window-major order spent ~45 VALU
      // instructions per k-step, 12 of them address adds; 28 k-steps instead of 25, the slowest wave
      // still 7).
      // A (row co = lo, k = the 4 positions of windows wa, wa + 1): the pooled gradient placed at its
      // argmax position by a 64-bit shift (code >= 4: ReLU off, or padding -> zero); lanes co >= 6
      // duplicate channel 0 (their C rows are never stored).
      // B (k, col r = 16u + lo): 4 pair reads at the windows' image offsets + a column constant; the
      // ones column r = 25 reads the ones image at the same offsets; r > 25 are never stored.
      const int sl = wave & (SPB - 1), h0 = wave / SPB, half = h0 & 1, r0 = h0 >> 1;
      const int c0 = 8 * half + 2 * hi;
      const bool padl = c0 >= Q1;
      const int cw = padl ? 0 : c0;  // padding lanes read window column 0 (any finite value; code forced)
      const uint32_t cpad = padl ? 4u : 0u;
      const int co = lo < C1 ? lo : 0;
      const float* dxr = &sm.dx2[sl][co * DX2S + r0 * Q1 + cw];
      const uint8_t* cr = &sm.k.c1[sl][co * (Q1 * Q1) + r0 * Q1 + cw];
      const bool onecol = lo == R1 - 16;  // u = 1 lane of the ones column
      const char* ib = (const char*)&sm.k.imgb[sl][0][0] + 2 * (2 * r0 * IMGS + 2 * cw);  // window (r0, cw)
      const char* bb[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = min(16 * u + lo, R1 - 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int x = (k & 1) * IMGS + (r / KS) * IMGS + (r % KS);
          const int cst = 2 * ((x & 1) ? IMGC + x - 1 : x) + (k >> 1) * 4;  // bytes; window wa + 1: +2 pixels
          bb[u][k] = (u == 1 && onecol) ? (const char*)sm.ones + (k >> 1) * 4 : ib + cst;
        }
      }
      static_assert(NTHR / 64 == 4 * SPB, "4 waves per sample in phase C");
      static_assert(6 * 8 * IMGS + 8 + 4 <= 2 * PC_ONES, "ones image covers the unrolled rows");
#pragma unroll
      for (int j = 0; j < 7; ++j) {  // pool rows r0 + 2j
        const float2 dd = *(const float2*)(dxr + 2 * j * Q1);
        const uint32_t cc = *(const uint16_t*)(cr + 2 * j * Q1);
        const uint32_t ca = (cc & 0xffu) | cpad, cb2 = (cc >> 8) | cpad;
        const uint32_t ab = pack16t<kH16>(dd.x, dd.y);
        const uint64_t ea = ca < 4 ? (uint64_t)(ab & 0xffffu) << (16 * ca) : 0ull;
        const uint64_t eb = cb2 < 4 ? (uint64_t)(ab >> 16) << (16 * cb2) : 0ull;
        const bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4((uint32_t)ea, (uint32_t)(ea >> 32), (uint32_t)eb,
                                                               (uint32_t)(eb >> 32)));
        const int ro = j * 8 * IMGS;  // bytes: two pool rows = four image rows
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint4 w = make_uint4(*(const uint32_t*)(bb[u][0] + ro), *(const uint32_t*)(bb[u][1] + ro),
                                     *(const uint32_t*)(bb[u][2] + ro), *(const uint32_t*)(bb[u][3] + ro));
          g1[u] = mfma16(a, __builtin_bit_cast(bf16x8, w), g1[u]);
        }
      }
    }

    RK_TR(cb.trace, 13);
    // ---- phase D: block totals -> the fused path stores them as one row of the [blocks][SLABW]
    // gradient slab (summed by the weight-gradient launch that follows: no contended atomics);
    // the generic path adds them to the gradients with global atomics
    float* srow = MLP ? cb.slab + (int64_t)blockIdx.x * SLABW : nullptr;
    if (wave < 10) {  // C[row = co 4hi + i][col = r]; column r = R2 holds db2
      const int u = wave, col = 16 * u + lo;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (col < R2) {
          if (MLP) srow[SL_W2 + (4 * hi + i) * R2 + col] = g2[i];
          else atomicAdd(dw2 + (4 * hi + i) * R2 + col, g2[i]);
        } else if (col == R2) {
          if (MLP) srow[SL_B2 + 4 * hi + i] = g2[i];
          else if (db2) atomicAdd(db2 + 4 * hi + i, g2[i]);
        }
      }
    }
    {  // dW1 partials of all 16 waves -> LDS (aliasing dc2: dead since phase B's barrier)
      float (*red1)[2][256] = (float (*)[2][256])&sm.dc2[0][0];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) red1[wave][u][(4 * hi + i) * 16 + lo] = g1[u][i];
    }
    lds_barrier();
    RK_TR(cb.trace, 10);
    for (int e = threadIdx.x; e < 2 * 256; e += NTHR) {  // column r = R1 (u = 1, lane 9) holds db1
      const int u = e >> 8, row = (e & 255) >> 4, col = 16 * u + (e & 15);
      if (row < C1 && col <= R1) {
        const float (*red1)[2][256] = (const float (*)[2][256])&sm.dc2[0][0];
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < NTHR / 64; ++w) v += red1[w][u][e & 255];
        if (col < R1) {
          if (MLP) srow[SL_W1 + row * R1 + col] = v;
          else atomicAdd(dw1 + row * R1 + col, v);
        } else {
          if (MLP) srow[SL_B1 + row] = v;
          else if (db1) atomicAdd(db1 + row, v);
        }
      }
    }
  RK_TR(cb.trace, 11);
  }
  if constexpr (MLP) {
    if (cb.ce && cb.defer_loss) {  // loss / valid-count partials; the next (wgrad) launch reduces them
      if (threadIdx.x == 0) {
        cb.partials[blockIdx.x] = sm.lossp[0];
        cb.partials[gridDim.x + blockIdx.x] = sm.cecnt[0];
      }
    } else if (cb.ce) {  // batch loss: block partials -> last block -> loss + Loss-capsule bookkeeping
      // (this path is only for unit-scale callers: the gradients it leaves are unnormalised)
      if (threadIdx.x == 0) {
        st_sc1(cb.partials + blockIdx.x, sm.lossp[0]);
        st_sc1(cb.partials + gridDim.x + blockIdx.x, sm.cecnt[0]);
      }
      if (last_block_arrived(cb.counter, &sm.flag)) {
        float t = 0.f, c = 0.f;
        for (int i = threadIdx.x; i < (int)gridDim.x; i += NTHR) {
          t += ld_sc1(cb.partials + i);
          c += ld_sc1(cb.partials + gridDim.x + i);
        }
        t = block_sum(t, sm.red);
        c = block_sum(c, sm.red);
        if (threadIdx.x == 0) {
          const float nv = c;
          const float l = nv > 0.f ? t / nv : NAN;
          cb.loss_out[0] = l;
          cb.loss_out[1] = nv;
          if (cb.acc) {
            float v = cb.acc[0] + l * cb.acc_scale;
            if (cb.sync) {
              const int64_t k = cb.slot[0];
              cb.ring[k] = v;
              cb.slot[0] = (k + 1) % cb.ring_size;
              v = 0.f;
            }
            cb.acc[0] = v;
          }
        }
        reset_counter(cb.counter);
      }
    }
    if (cb.ce) RK_TR(cb.trace, 12);
  }
}

template <bool MLP>
__global__ void __launch_bounds__(NTHR) lenet_conv_bwd(const float* __restrict__ x, const uint16_t* __restrict__ a1g,
                                                       const uint8_t* __restrict__ code1g, const uint16_t* __restrict__ da2g,
                                                       const uint8_t* __restrict__ code2g, const float* __restrict__ w2,
                                                       float* __restrict__ dw1, float* __restrict__ db1, float* __restrict__ dw2,
                                                       float* __restrict__ db2, int N, int rounds, ClsBwd cb) {
  __shared__ __attribute__((aligned(16))) BwdSmem sm;
  bwd_body<MLP>(sm, x, a1g, code1g, da2g, code2g, w2, dw1, db1, dw2, db2, N, rounds, cb);
}

// ------------------------------------------------------------------------------ whole step
// Forward + fused cross-entropy + backward of the block's 4 samples in ONE launch: nothing in the
// backward of a sample depends on another block (the cross-entropy's mean count is derived from the
// targets alone, every block counts them), so the forward -> backward kernel boundary (a dependent
// dispatch, ~3.4 us of idle GPU per step, profiles/r3_lenet_step_timeline.json) is not needed.  The
// two phases share the LDS (union) except the KeepSmem prefix (image, a1, code maps), which the
// backward reads in place; the forward's other outputs it needs (logits, ReLU masks) come back from
// this block's own global stores, which the barrier orders (workgroup scope: one CU, coherent L1).
union TrainSmem {
  FwdSmem f;
  BwdSmem b;
};

__global__ void __launch_bounds__(NTHR) lenet_train_kernel(const float* __restrict__ x, const float* __restrict__ b1,
                                                          const float* __restrict__ b2, uint16_t* __restrict__ a1g,
                                                          uint8_t* __restrict__ code1, uint8_t* __restrict__ code2,
                                                          int N, ClsFwd cf, ClsBwd cb, RowSrc rs) {
  __shared__ __attribute__((aligned(16))) TrainSmem sm;
  // a1 / codes stay in LDS (sm.f.k == sm.b.k): no global copies (a regular backward after a missed
  // speculation re-runs rk_lenet_fwd for them, ops/lenet.py)
  ClsBwdFrags pre;
  fwd_body<true>(sm.f, x, nullptr, b1, nullptr, b2, nullptr, nullptr, nullptr, nullptr, N, cf, rs, &pre, cb.frag);
  // LDS reuse only: this backward (RES) reads nothing the forward wrote to global memory (logits,
  // labels, masks and a1 / codes are in LDS), so the forward's stores need not have landed — a
  // __syncthreads() here would wait for all of them (vmcnt(0))
  lds_barrier();
  if (rs.rows) {  // the block's targets through the rows (as its own label stores, which it just made)
    cb.row_table = rs.rows;
    cb.row_labels = rs.ysrc;
  }
  bwd_body<true, true>(sm.b, x, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, N, 1,
                       cb, &pre);
}

}  // namespace

RK_API int RKL_NAME(rk_lenet_conv_fwd)(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                             void* a1, void* code1, void* a2, void* code2, int N, hipStream_t s) {
  if ((uintptr_t)x & 15) return (int)hipErrorInvalidValue;  // float4 image loads
  const int grid = (N + SPB - 1) / SPB;
  lenet_conv_fwd<false><<<grid, NTHR, 0, s>>>(x, w1, b1, w2, b2, (uint16_t*)a1, (uint8_t*)code1, (uint16_t*)a2,
                                              (uint8_t*)code2, N, ClsFwd{});
  return (int)hipGetLastError();
}

// fc + conv weights (fp32 masters) -> bf16 MFMA fragment table (NFRAG x 64 x 16 B)
RK_API int RKL_NAME(rk_lenet_prep)(const float* fc1w, const float* fc2w, const float* fc3w, const float* conv1w,
                         const float* conv2w, void* frag, hipStream_t s) {
  lenet_prep_kernel<<<NFRAG, 64, 0, s>>>(fc1w, fc2w, fc3w, conv1w, conv2w, (bf16x8*)frag);
  return (int)hipGetLastError();
}

#if !RK_LENET_H
RK_API int rk_lenet_frag_bytes() { return NFRAG * 64 * 16; }
#endif

// Whole LeNet forward (conv stack + classifier) for N % 8 == 0: logits [N][10] fp32, plus the
// saved state of the fused backward (a1, codes) and the transposed activations of the wgrads.
// Diagnostics: phase timelines of the fused launches ([blocks][48] u64 each, or null = off).
// (one pair of pointers, shared by the bf16 and fp16 builds of this file)
#if RK_LENET_H
extern uint64_t* g_fwd_trace;
extern uint64_t* g_bwd_trace;
#else
uint64_t* g_fwd_trace = nullptr;
uint64_t* g_bwd_trace = nullptr;
RK_API void rk_lenet_set_trace(void* fwd, void* bwd) {
  g_fwd_trace = (uint64_t*)fwd;
  g_bwd_trace = (uint64_t*)bwd;
}
#endif

RK_API int RKL_NAME(rk_lenet_fwd)(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                        const void* frag, const float* fb1, const float* fb2, const float* fb3, void* a1,
                        void* code1, void* code2, void* a2T, void* h1T, void* h2T, float* logits, int N,
                        hipStream_t s) {
  if (N % 8 || ((uintptr_t)x & 15)) return (int)hipErrorInvalidValue;
  ClsFwd cf{(const bf16x8*)frag, fb1, fb2, fb3, (uint16_t*)a2T, (uint16_t*)h1T, (uint16_t*)h2T, logits, g_fwd_trace};
  lenet_conv_fwd<true><<<N / SPB, NTHR, 0, s>>>(x, w1, b1, w2, b2, (uint16_t*)a1, (uint8_t*)code1, nullptr,
                                                (uint8_t*)code2, N, cf);
  return (int)hipGetLastError();
}

// Gradients are ACCUMULATED (atomics) into dw1/db1/dw2/db2 (zeroed or persistent f32 buffers).
// `rounds`: samples groups of 4 processed per block (more rounds -> fewer global atomics).
RK_API int RKL_NAME(rk_lenet_conv_bwd)(const float* x, const void* a1, const void* code1, const void* da2, const void* code2,
                             const float* w2, float* dw1, float* db1, float* dw2, float* db2, int N, int rounds,
                             hipStream_t s) {
  if (rounds < 1) rounds = 1;
  const int per_block = SPB * rounds;
  const int grid = (N + per_block - 1) / per_block;
  lenet_conv_bwd<false><<<grid, NTHR, 0, s>>>(x, (const uint16_t*)a1, (const uint8_t*)code1, (const uint16_t*)da2,
                                              (const uint8_t*)code2, w2, dw1, db1, dw2, db2, N, rounds, ClsBwd{});
  return (int)hipGetLastError();
}

// Fused backward for N % 8 == 0 (one block per 4 samples): classifier input-gradient chain from
// dlogits, then the conv stack; writes dy^T, d2^T, d1^T and the conv-gradient slab for
// rk_mlp3_wgrad, which accumulates all ten weight/bias gradients.
struct LenetCE {  // host-side description of the fused cross-entropy (see ClsBwd)
  const float* logits;
  const int64_t* target;
  int64_t ignore_index;
  float grad_scale;
  float* partials;
  unsigned* counter;
  float* loss_out;
  float *acc, *ring;
  int64_t* slot;
  int ring_size;
  float acc_scale;
  int sync;
  int defer_loss;  // 1: rk_mlp3_wgrad_loss finalises the loss (no last-block ticket in this launch)
  const float* gscale_dev;  // nullable: d(logits) also scaled by *gscale_dev (device loss scale)
};

static ClsBwd cls_bwd(const void* frag, const float* dy, const void* h1T, const void* h2T, void* dyT, void* d2T,
                      void* d1T, float* slab, const LenetCE* ce) {
  ClsBwd cb{};
  cb.trace = g_bwd_trace;
  cb.slab = slab;
  cb.frag = (const bf16x8*)frag;
  cb.dy = dy;
  cb.h1T = (const uint16_t*)h1T;
  cb.h2T = (const uint16_t*)h2T;
  cb.dyT = (uint16_t*)dyT;
  cb.d2T = (uint16_t*)d2T;
  cb.d1T = (uint16_t*)d1T;
  if (ce) {
    cb.ce = 1;
    cb.logits = ce->logits;
    cb.target = ce->target;
    cb.ignore_index = ce->ignore_index;
    cb.grad_scale = ce->grad_scale;
    cb.partials = ce->partials;
    cb.counter = ce->counter;
    cb.loss_out = ce->loss_out;
    cb.acc = ce->acc;
    cb.ring = ce->ring;
    cb.slot = ce->slot;
    cb.ring_size = ce->ring_size;
    cb.acc_scale = ce->acc_scale;
    cb.sync = ce->sync;
    cb.defer_loss = ce->defer_loss;
    cb.gscale_dev = ce->gscale_dev;
  }
  return cb;
}

// The conv weight/bias gradients are NOT accumulated here: each block writes its totals to
// slab[block][rk_lenet_slab_width()] (N/4 rows), which rk_mlp3_wgrad then sums into dw1/db1/dw2/db2.
#if !RK_LENET_H
RK_API int rk_lenet_slab_width() { return SLABW; }
RK_API int rk_lenet_slab_cols() { return SLABN; }
#endif

RK_API int RKL_NAME(rk_lenet_bwd)(const float* x, const void* a1, const void* code1, const void* code2, const float* w2,
                        const void* frag, const float* dy, const void* h1T, const void* h2T, void* dyT, void* d2T,
                        void* d1T, float* slab, int N, int rounds, const LenetCE* ce, hipStream_t s) {
  rounds = 1;  // the fused kernel handles one group of SPB samples per block (argument kept for ABI)
  if (N % 8 || N > 65536 || ((uintptr_t)x & 15)) return (int)hipErrorInvalidValue;  // float4 image loads
  if (!slab) return (int)hipErrorInvalidValue;
  const ClsBwd cb = cls_bwd(frag, dy, h1T, h2T, dyT, d2T, d1T, slab, ce);
  lenet_conv_bwd<true><<<N / (SPB * rounds), NTHR, 0, s>>>(x, (const uint16_t*)a1, (const uint8_t*)code1, nullptr,
                                                           (const uint8_t*)code2, w2, nullptr, nullptr, nullptr,
                                                           nullptr, N, rounds, cb);
  return (int)hipGetLastError();
}

// Whole fused LeNet training step of the batch but the weight gradients, in ONE launch
// (lenet_train_kernel): the rk_lenet_fwd outputs (logits, a1, codes, transposed activations) and
// the rk_lenet_bwd outputs (transposed gradients, conv-gradient slab, loss partials) for a
// softmax cross-entropy on `ce` (required; its d(logits) scale is ce->grad_scale).  rows (may be
// null): the batch is gathered by this launch (RowSrc): x / ce->target are the batch buffers it fills.
RK_API int RKL_NAME(rk_lenet_train)(const float* x, const float* b1, const float* b2, const void* frag, const float* fb1,
                          const float* fb2, const float* fb3, void* a1, void* code1, void* code2, void* a2T, void* h1T,
                          void* h2T, float* logits, void* dyT, void* d2T, void* d1T, float* slab, int N,
                          const LenetCE* ce, const RowSrc* rows, hipStream_t s) {
  if (N % 8 || N > 65536 || ((uintptr_t)x & 15) || !slab || !ce || ce->logits != logits) return (int)hipErrorInvalidValue;
  RowSrc rs = rows ? *rows : RowSrc{};
  rs.target = ce->target;
  static const int x_plain = getenv("ROCKET_LENET_X_PLAIN") ? atoi(getenv("ROCKET_LENET_X_PLAIN")) : 0;
  rs.keep = 1 | (x_plain ? 2 : 0);
  if (rs.rows && (!rs.xsrc || !rs.ysrc || !rs.ydst || ((uintptr_t)rs.xsrc & 15))) return (int)hipErrorInvalidValue;
  const ClsFwd cf{(const bf16x8*)frag, fb1, fb2, fb3, (uint16_t*)a2T, (uint16_t*)h1T, (uint16_t*)h2T, logits, g_fwd_trace};
  const ClsBwd cb = cls_bwd(frag, nullptr, h1T, h2T, dyT, d2T, d1T, slab, ce);
  lenet_train_kernel<<<N / SPB, NTHR, 0, s>>>(x, b1, b2, (uint16_t*)a1, (uint8_t*)code1, (uint8_t*)code2, N, cf, cb, rs);
  return (int)hipGetLastError();
}

