// Classifier heads whose class count is not a multiple of 8 (CIFAR-10's 10 classes, CIFAR-100's 100
// beyond the MFMA routes' N % 8 rule): y = x W^T + b with fp32 W / b / y and a 16-bit or fp32 x,
// and the whole backward (dx, dW, db) in ONE launch.
//
// These products are tiny (ResNet-18 CIFAR: 256 x 10 x 512 = 1.3 MFLOP): the library route costs
// a dozen launches around three GEMMs (weight / bias casts to bf16, the fp32 casts of the logits
// and of both gradients, autograd's accumulation adds, a bias column sum), each at the ~5 us floor
// of a kernel boundary.  Here: one forward launch, one backward launch, fp32 logits handed to the
// cross-entropy directly (no cast), gradients accumulated into the persistent fp32 grads.
//
// Forward: one block per row m, threads over k (coalesced x and W rows, every load of a round in
// flight), 16 class accumulators per pass, butterfly + LDS reductions.  Backward: blocks [0, KB)
// form dW / db — a block owns 64 k-columns (one per lane), its 4 waves split the rows, LDS
// combines them in a fixed order (deterministic); the remaining blocks form dx, one element per
// thread.  Both are latency-bound launches: the loads are issued in rounds, not row by row.
#include "rk_common.h"

using namespace rk;

namespace {

constexpr int HT = 256;      // forward: threads per block (one block per row)
constexpr int HW = HT / 64;  // forward: waves per block
// backward: small blocks (4 waves, ~21 KB LDS), so a block always fits next to co-resident
// persistent kernels (the spinning P2P all-reduce blocks of DP ranks sharing a GPU)
constexpr int BT = 256;      // backward: threads per block
constexpr int BW = BT / 64;  // backward: waves per block
constexpr int HNC = 16;      // classes per accumulator pass
constexpr int HNMAX = 128;   // largest class count served
constexpr int SR = 64;       // backward: dy rows staged in LDS per pass (16 per wave, their x loads in one round)

template <int DT>
__device__ __forceinline__ float ldx(const void* p, int64_t i) {
  if constexpr (DT == F32) return ((const float*)p)[i];
  else if constexpr (DT == F16) return h2f(((const uint16_t*)p)[i]);
  else return bf2f(((const uint16_t*)p)[i]);
}
template <int DT>
__device__ __forceinline__ void stx(void* p, int64_t i, float v) {
  if constexpr (DT == F32) ((float*)p)[i] = v;
  else if constexpr (DT == F16) ((uint16_t*)p)[i] = f2h(v);
  else ((uint16_t*)p)[i] = f2bf(v);
}

template <int DT>
__device__ __forceinline__ float rnd(float v) {  // the value a DT store then load would give
  if constexpr (DT == F32) return v;
  else if constexpr (DT == F16) return h2f(f2h(v));
  else return bf2f(f2bf(v));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one block per row: each thread 4 k's per round (all x / W loads of the round in flight), the
// block's partial dot products reduced by butterflies then across the 4 waves in LDS (fixed order).
// hw > 1: x is the channels-last activation [M][hw][K] and the row is its global average pool
// (fp32 sum, rounded to the activation dtype like rk_gap_fwd's output), also stored to xpool
// [M][K] for the backward.
template <int DT>
__global__ void __launch_bounds__(HT) head_fwd_kernel(const void* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ b, float* __restrict__ y, int M,
                                                      int N, int K, int hw, void* __restrict__ xpool) {
  __shared__ float red[HW][HNC];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int m = blockIdx.x;
  const float inv_hw = 1.f / (float)hw;
  for (int n0 = 0; n0 < N; n0 += HNC) {
    float acc[HNC];
#pragma unroll
    for (int j = 0; j < HNC; ++j) acc[j] = 0.f;
    for (int k0 = 0; k0 < K; k0 += 4 * HT) {
      float xv[4], wr[4][HNC];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * HT + (int)threadIdx.x;
        if (hw == 1) {
          xv[u] = k < K ? ldx<DT>(x, (int64_t)m * K + k) : 0.f;
        } else {
          float sum = 0.f;
          if (hw <= 16) {  // ResNet's 4x4 / 7x7-class heads: every pixel load of the round in flight
            float pv[16];
#pragma unroll
            for (int p = 0; p < 16; ++p) pv[p] = (p < hw && k < K) ? ldx<DT>(x, ((int64_t)m * hw + p) * K + k) : 0.f;
#pragma unroll
            for (int p = 0; p < 16; ++p) sum += pv[p];
          } else {
#pragma unroll 8
            for (int p = 0; p < hw; ++p) sum += k < K ? ldx<DT>(x, ((int64_t)m * hw + p) * K + k) : 0.f;
          }
          xv[u] = rnd<DT>(sum * inv_hw);  // the pooled row as rk_gap_fwd stores it: the value the head consumes
          if (k < K) stx<DT>(xpool, (int64_t)m * K + k, xv[u]);
        }
#pragma unroll
        for (int j = 0; j < HNC; ++j) wr[u][j] = (k < K && n0 + j < N) ? w[(int64_t)(n0 + j) * K + k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < HNC; ++j) acc[j] += xv[u] * wr[u][j];
    }
#pragma unroll
    for (int j = 0; j < HNC; ++j) {
      const float v = wave_sum(acc[j]);
      if (lane == 0) red[wv][j] = v;
    }
    __syncthreads();
    if (threadIdx.x < HNC && n0 + (int)threadIdx.x < N) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < HW; ++q) v += red[q][threadIdx.x];
      y[(int64_t)m * N + n0 + threadIdx.x] = v + (b ? b[n0 + threadIdx.x] : 0.f);
    }
    __syncthreads();
  }
}

// blocks [0, kb * mb): dW / db partials of 64 k-columns (one per lane) over one chunk of SR rows
// (16 rows per wave, all their x loads in flight; dy staged in LDS, read as broadcasts), the 4
// waves' sums combined in LDS in wave order and stored as the chunk's partial; the last chunk block
// of a column group (ticket, no waiting) sums the mb partials in chunk order (deterministic) into
// dW / db.  The rest of the grid: dx, one element per thread.
template <int DT>
__global__ void __launch_bounds__(BT) head_bwd_kernel(const float* __restrict__ dy, const void* __restrict__ x,
                                                      const float* __restrict__ w, void* __restrict__ dx,
                                                      float* __restrict__ dw, float* __restrict__ db, int acc_w,
                                                      int acc_b, int M, int N, int K, int kb, int mb,
                                                      float* __restrict__ part, unsigned* __restrict__ cnt, int hw) {
  // the staged dy rows and the cross-wave partials share one LDS region (~17 KB in all: the block
  // must fit next to whatever else is resident, see BT)
  __shared__ float lds_u[BW * HNC * (64 + 1)];
  __shared__ float redb[BW][HNC];
  __shared__ int last;
  float (*sdy)[HNC] = reinterpret_cast<float (*)[HNC]>(lds_u);
  float (*red)[HNC][64 + 1] = reinterpret_cast<float (*)[HNC][64 + 1]>(lds_u);
  static_assert(SR * HNC <= BW * HNC * (64 + 1), "staged rows fit the shared region");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if ((int)blockIdx.x < kb * mb) {  // partial dW[n][k] = sum_m dy[m][n] x[m][k] over rows [mc, mc + SR)
    const int kbi = (int)blockIdx.x % kb, mbi = (int)blockIdx.x / kb;
    const int k = kbi * 64 + lane, mc = mbi * SR;
    const bool kok = k < K;
    float* pw = part + (int64_t)mbi * N * K;          // [mb][N][K]
    float* pb = part + (int64_t)mb * N * K + mbi * N;  // [mb][N]
    for (int n0 = 0; n0 < N; n0 += HNC) {
      float acc[HNC], accb[HNC];
      __syncthreads();  // the previous class chunk's reads of the shared region are done
#pragma unroll
      for (int t = 0; t < SR * HNC / BT; ++t) {
        const int i = (int)threadIdx.x + t * BT, r = i / HNC, j = i % HNC;
        sdy[r][j] = (mc + r < M && n0 + j < N) ? dy[(int64_t)(mc + r) * N + n0 + j] : 0.f;
      }
      __syncthreads();
      float xv[SR / BW];
#pragma unroll
      for (int t = 0; t < SR / BW; ++t) {
        const int m = mc + wv + BW * t;
        xv[t] = (kok && m < M) ? ldx<DT>(x, (int64_t)m * K + k) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < HNC; ++j) acc[j] = accb[j] = 0.f;
#pragma unroll 2
      for (int t = 0; t < SR / BW; ++t)
#pragma unroll
        for (int j = 0; j < HNC; ++j) {
          const float g = sdy[wv + BW * t][j];
          acc[j] += g * xv[t];
          accb[j] += g;
        }
      __syncthreads();  // the sdy reads are done before red overwrites the region
#pragma unroll
      for (int j = 0; j < HNC; ++j) red[wv][j][lane] = acc[j];
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < HNC; ++j) redb[wv][j] = accb[j];
      }
      __syncthreads();
      for (int j = wv; j < HNC; j += BW) {  // wave wv: classes wv, wv + 4, ...; partials in wave order
        float sum = 0.f;
#pragma unroll
        for (int q = 0; q < BW; ++q) sum += red[q][j][lane];
        if (kok && n0 + j < N) st_sc1(pw + (int64_t)(n0 + j) * K + k, sum);
      }
      if (kbi == 0 && threadIdx.x < HNC && n0 + (int)threadIdx.x < N) {
        float sum = 0.f;
#pragma unroll
        for (int q = 0; q < BW; ++q) sum += redb[q][threadIdx.x];
        st_sc1(pb + n0 + threadIdx.x, sum);
      }
    }
    // ticket (rk_common.h protocol: partials stored / read with sc1, every wave's stores drained
    // before lane 0's ticket): the last of the column group's mb chunk blocks combines and resets
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(cnt + kbi, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = t == (unsigned)(mb - 1);
    }
    __syncthreads();
    if (!last) return;
    reset_counter(cnt + kbi);
    for (int j = wv; j < N; j += BW) {
      if (!kok) break;
      float sum = 0.f;
      for (int q = 0; q < mb; ++q) sum += ld_sc1(part + ((int64_t)q * N + j) * K + k);
      float* o = dw + (int64_t)j * K + k;
      *o = acc_w ? *o + sum : sum;
    }
    if (db != nullptr && kbi == 0) {
      for (int j = threadIdx.x; j < N; j += BT) {
        float sum = 0.f;
        for (int q = 0; q < mb; ++q) sum += ld_sc1(part + (int64_t)mb * N * K + q * N + j);
        float* o = db + j;
        *o = acc_b ? *o + sum : sum;
      }
    }
    return;
  }
  if (dx == nullptr) return;
  // dx[m][k] = sum_n dy[m][n] W[n][k]: each chunk's 16 dy / W loads in flight together
  const int64_t e = (int64_t)(blockIdx.x - kb * mb) * BT + threadIdx.x;
  if (e >= (int64_t)M * K) return;
  const int m = (int)(e / K), k = (int)(e % K);
  const float* d = dy + (int64_t)m * N;
  float s = 0.f;
  for (int n0 = 0; n0 < N; n0 += HNC) {
    float dv[HNC], wr[HNC];
#pragma unroll
    for (int j = 0; j < HNC; ++j) {
      dv[j] = n0 + j < N ? d[n0 + j] : 0.f;
      wr[j] = n0 + j < N ? w[(int64_t)(n0 + j) * K + k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < HNC; ++j) s += dv[j] * wr[j];
  }
  if (hw == 1) {
    stx<DT>(dx, e, s);
    return;
  }
  // pooled head: the input gradient of the average pool, dy / hw broadcast over the row's pixels of
  // the channels-last activation (the pooled gradient rounded first, as rk_gap_bwd reads it)
  const float g = rnd<DT>(s) * (1.f / (float)hw);
  for (int p = 0; p < hw; ++p) stx<DT>(dx, ((int64_t)m * hw + p) * K + k, g);
}

}  // namespace

// y[M][N] f32 = x[M][K] (dt) W[N][K]^T (f32) + b[N] (f32, may be null); N <= 128
// hw > 1: x is a channels-last activation [M][hw][K] pooled first (its pooled rows -> xpool [M][K]).
RK_API int rk_head_fwd(int dt, const void* x, const float* w, const float* b, float* y, int M, int N, int K, int hw,
                       void* xpool, hipStream_t s) {
  if (M <= 0 || N <= 0 || N > HNMAX || K <= 0 || hw <= 0 || (int64_t)M * hw * K >= ((int64_t)1 << 31))
    return (int)hipErrorInvalidValue;
  if (hw > 1 && xpool == nullptr) return (int)hipErrorInvalidValue;
  const int grid = M;
  if (dt == BF16) head_fwd_kernel<BF16><<<grid, HT, 0, s>>>(x, w, b, y, M, N, K, hw, xpool);
  else if (dt == F16) head_fwd_kernel<F16><<<grid, HT, 0, s>>>(x, w, b, y, M, N, K, hw, xpool);
  else if (dt == F32) head_fwd_kernel<F32><<<grid, HT, 0, s>>>(x, w, b, y, M, N, K, hw, xpool);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// One launch: dx[M][K] (dt, may be null) = dy W; dW[N][K] f32 (+)= dy^T x (may be null);
// db[N] f32 (+)= column sums of dy (may be null).  dy: f32 [M][N].  part: f32 scratch of
// rk_head_bwd_scratch(M, N, K) floats; cnt: ceil(K / 64) zeroed counters (left zeroed).
RK_API int64_t rk_head_bwd_scratch(int M, int N, int K) {
  const int64_t mb = (M + SR - 1) / SR;
  return mb * N * (int64_t)K + mb * N;
}

// hw > 1: x is the pooled input [M][K] (rk_head_fwd's xpool) and dx the channels-last activation
// gradient [M][hw][K] (the pool's backward in the same launch).
RK_API int rk_head_bwd(int dt, const float* dy, const void* x, const float* w, void* dx, float* dw, float* db,
                       int acc_w, int acc_b, int M, int N, int K, float* part, unsigned* cnt, int hw, hipStream_t s) {
  if (M <= 0 || N <= 0 || N > HNMAX || K <= 0 || hw <= 0 || (int64_t)M * hw * K >= ((int64_t)1 << 31))
    return (int)hipErrorInvalidValue;
  if (db != nullptr && dw == nullptr) return (int)hipErrorInvalidValue;  // db rides on the dW blocks
  if (dw != nullptr && (part == nullptr || cnt == nullptr)) return (int)hipErrorInvalidValue;
  const int kb = dw != nullptr ? (K + 63) / 64 : 0;
  const int mb = (M + SR - 1) / SR;
  if ((int64_t)kb * mb >= ((int64_t)1 << 30)) return (int)hipErrorInvalidValue;
  const int xb = dx != nullptr ? (int)(((int64_t)M * K + BT - 1) / BT) : 0;
  const int wb = kb * mb;
  if (wb + xb == 0) return 0;
#define RK_HB(D) head_bwd_kernel<D><<<wb + xb, BT, 0, s>>>(dy, x, w, dx, dw, db, acc_w, acc_b, M, N, K, wb ? kb : 1, \
                                                         wb ? mb : 0, part, cnt, hw)
  if (dt == BF16) RK_HB(BF16);
  else if (dt == F16) RK_HB(F16);
  else if (dt == F32) RK_HB(F32);
  else return (int)hipErrorInvalidValue;
#undef RK_HB
  return (int)hipGetLastError();
}
