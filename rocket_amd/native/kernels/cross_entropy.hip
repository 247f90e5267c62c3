// Fused softmax cross-entropy (replaces _log_softmax + nll_loss fwd/bwd).
//
// Forward: one pass over the logits computes max, log-sum-exp, the target logit
// and (for label smoothing) the row mean, writes nothing per element, and
// reduces the batch loss in-launch (block partials + last-arriving block), so
// the whole loss is ONE launch and no per-row tensor round-trips HBM.
// Backward: recomputes the softmax from the logits (cheaper than storing it)
// and writes dlogits = g * w * (softmax - (1-eps)*onehot - eps/C), where g is the
// incoming grad (read from device memory: no host sync, graph-safe) and
// w = 1/num_valid (mean) or 1 (sum).  Ignored targets get zero rows.
//
// Mapping (wave64): for C <= 64 one thread owns a row (LeNet: C = 10, 1024 rows
// -> 4 blocks); for larger C one wave owns a row and strides over the classes
// with 64 lanes, reducing with __shfl_xor over all 64 lanes.
#include "rk_common.h"

using namespace rk;

namespace {

struct RowStats {
  float lse, xt, xmean;
};

template <typename T, bool WAVE>
__device__ __forceinline__ RowStats row_stats(const T* x, int C, int64_t t, int lane) {
  float m = -INFINITY;
  if (WAVE) {
    for (int j = lane; j < C; j += 64) m = fmaxf(m, Ld<T>::get(x, j));
    m = wave_max(m);
    float s = 0.f, sx = 0.f;
    for (int j = lane; j < C; j += 64) {
      float v = Ld<T>::get(x, j);
      s += __expf(v - m);
      sx += v;
    }
    s = wave_sum(s);
    sx = wave_sum(sx);
    float xt = (t >= 0 && t < C) ? Ld<T>::get(x, t) : 0.f;
    return {m + __logf(s), xt, sx / C};
  } else {
    for (int j = 0; j < C; ++j) m = fmaxf(m, Ld<T>::get(x, j));
    float s = 0.f, sx = 0.f;
    for (int j = 0; j < C; ++j) {
      float v = Ld<T>::get(x, j);
      s += __expf(v - m);
      sx += v;
    }
    float xt = (t >= 0 && t < C) ? Ld<T>::get(x, t) : 0.f;
    return {m + __logf(s), xt, sx / C};
  }
}

template <typename T, bool WAVE>
__global__ void __launch_bounds__(256) ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                     int N, int C, int64_t ignore_index, float smoothing,
                                                     float* partials, unsigned* counter, float* out /*[loss, nvalid]*/,
                                                     int mean) {
  __shared__ float red[8];
  __shared__ int flag;
  const int lane = threadIdx.x & 63;
  const int rows_per_block = WAVE ? (blockDim.x >> 6) : blockDim.x;
  const int row = blockIdx.x * rows_per_block + (WAVE ? (threadIdx.x >> 6) : threadIdx.x);
  float loss = 0.f, valid = 0.f;
  if (row < N) {
    int64_t t = target[row];
    if (t != ignore_index) {
      RowStats st = row_stats<T, WAVE>(logits + (int64_t)row * C, C, t, lane);
      float nll = st.lse - st.xt;
      loss = (1.f - smoothing) * nll + smoothing * (st.lse - st.xmean);
      valid = 1.f;
    }
    if (WAVE && lane != 0) loss = valid = 0.f;  // one contribution per row
  }
  float bl = block_sum(loss, red);
  float bv = block_sum(valid, red);
  if (threadIdx.x == 0) {
    st_sc1(partials + 2 * blockIdx.x, bl);
    st_sc1(partials + 2 * blockIdx.x + 1, bv);
  }
  if (last_block_arrived(counter, &flag)) {
    float s = 0.f, v = 0.f;
    for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x) {
      s += ld_sc1(partials + 2 * b);
      v += ld_sc1(partials + 2 * b + 1);
    }
    s = block_sum(s, red);
    v = block_sum(v, red);
    if (threadIdx.x == 0) {
      out[0] = mean ? (v > 0.f ? s / v : NAN) : s;
      out[1] = v;
    }
    reset_counter(counter);
  }
}

template <typename T, bool WAVE>
__global__ void __launch_bounds__(256) ce_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                     T* __restrict__ dlogits, int N, int C, int64_t ignore_index,
                                                     float smoothing, const float* grad_out, const float* stats,
                                                     int mean) {
  const int lane = threadIdx.x & 63;
  const int rows_per_block = WAVE ? (blockDim.x >> 6) : blockDim.x;
  const int row = blockIdx.x * rows_per_block + (WAVE ? (threadIdx.x >> 6) : threadIdx.x);
  if (row >= N) return;
  const T* x = logits + (int64_t)row * C;
  T* dx = dlogits + (int64_t)row * C;
  int64_t t = target[row];
  float g = grad_out[0];
  if (mean) g = stats[1] > 0.f ? g / stats[1] : 0.f;
  const int j0 = WAVE ? lane : 0, js = WAVE ? 64 : 1;
  if (t == ignore_index) {
    for (int j = j0; j < C; j += js) Ld<T>::put(dx, j, 0.f);
    return;
  }
  RowStats st = row_stats<T, WAVE>(x, C, t, lane);
  const float off = smoothing / C;
  for (int j = j0; j < C; j += js) {
    float p = __expf(Ld<T>::get(x, j) - st.lse);
    float d = p - off - (j == t ? (1.f - smoothing) : 0.f);
    Ld<T>::put(dx, j, g * d);
  }
}

// Training-step variant (one launch instead of fwd + loss bookkeeping + bwd): every block
// counts the valid targets of the whole batch itself (N <= 65536, a few L2-resident loads per
// thread) so it can write its rows' d(logits) = grad_scale * w * (softmax - target dist)
// immediately; the last block reduces the loss and folds it into the Loss capsule's device
// accumulator / report ring (acc may be null).
struct CeTrainAcc {
  float* acc;
  float* ring;
  int64_t* slot;
  int ring_size;
  float scale;
  int sync;
};

template <typename T, bool WAVE>
__global__ void __launch_bounds__(256) ce_train_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                       T* __restrict__ dlogits, int N, int C, int64_t ignore_index,
                                                       float smoothing, float grad_scale, float* partials,
                                                       unsigned* counter, float* out, int mean, CeTrainAcc la) {
  __shared__ float red[8];
  __shared__ int flag;
  float cnt = 0.f;
  for (int i = threadIdx.x; i < N; i += blockDim.x) cnt += target[i] != ignore_index ? 1.f : 0.f;
  const float nvalid = block_sum(cnt, red);
  const float w = grad_scale * (mean ? (nvalid > 0.f ? 1.f / nvalid : 0.f) : 1.f);
  const int lane = threadIdx.x & 63;
  const int rows_per_block = WAVE ? (blockDim.x >> 6) : blockDim.x;
  const int row = blockIdx.x * rows_per_block + (WAVE ? (threadIdx.x >> 6) : threadIdx.x);
  float loss = 0.f;
  if (row < N) {
    const T* x = logits + (int64_t)row * C;
    T* dx = dlogits + (int64_t)row * C;
    const int64_t t = target[row];
    const int j0 = WAVE ? lane : 0, js = WAVE ? 64 : 1;
    if (t == ignore_index) {
      for (int j = j0; j < C; j += js) Ld<T>::put(dx, j, 0.f);
    } else {
      const RowStats st = row_stats<T, WAVE>(x, C, t, lane);
      loss = (1.f - smoothing) * (st.lse - st.xt) + smoothing * (st.lse - st.xmean);
      const float off = smoothing / C;
      for (int j = j0; j < C; j += js) {
        const float p = __expf(Ld<T>::get(x, j) - st.lse);
        Ld<T>::put(dx, j, w * (p - off - (j == t ? (1.f - smoothing) : 0.f)));
      }
    }
    if (WAVE && lane != 0) loss = 0.f;
  }
  const float bl = block_sum(loss, red);
  if (threadIdx.x == 0) st_sc1(partials + blockIdx.x, bl);
  if (last_block_arrived(counter, &flag)) {
    float sum = 0.f;
    for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x) sum += ld_sc1(partials + b);
    sum = block_sum(sum, red);
    if (threadIdx.x == 0) {
      const float l = mean ? (nvalid > 0.f ? sum / nvalid : NAN) : sum;
      out[0] = l;
      out[1] = nvalid;
      if (la.acc) {
        float v = la.acc[0] + l * la.scale;
        if (la.sync) {
          const int64_t k = la.slot[0];
          la.ring[k] = v;
          la.slot[0] = (k + 1) % la.ring_size;
          v = 0.f;
        }
        la.acc[0] = v;
      }
    }
    reset_counter(counter);
  }
}

template <typename T>
hipError_t launch_fwd(const void* logits, const int64_t* target, int N, int C, int64_t ignore, float eps,
                      float* partials, unsigned* counter, float* out, int mean, hipStream_t s) {
  const bool wave = C > 64;
  const int threads = 256;
  const int rows = wave ? threads / 64 : threads;
  const int grid = (N + rows - 1) / rows;
  if (wave)
    ce_fwd_kernel<T, true><<<grid, threads, 0, s>>>((const T*)logits, target, N, C, ignore, eps, partials, counter, out, mean);
  else
    ce_fwd_kernel<T, false><<<grid, threads, 0, s>>>((const T*)logits, target, N, C, ignore, eps, partials, counter, out, mean);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_bwd(const void* logits, const int64_t* target, void* dlogits, int N, int C, int64_t ignore,
                      float eps, const float* g, const float* stats, int mean, hipStream_t s) {
  const bool wave = C > 64;
  const int threads = 256;
  const int rows = wave ? threads / 64 : threads;
  const int grid = (N + rows - 1) / rows;
  if (wave)
    ce_bwd_kernel<T, true><<<grid, threads, 0, s>>>((const T*)logits, target, (T*)dlogits, N, C, ignore, eps, g, stats, mean);
  else
    ce_bwd_kernel<T, false><<<grid, threads, 0, s>>>((const T*)logits, target, (T*)dlogits, N, C, ignore, eps, g, stats, mean);
  return hipGetLastError();
}

}  // namespace

// partials: >= 2*ceil(N/rows_per_block) floats; counter: one zeroed uint; out: 2 floats.
RK_API int rk_ce_fwd(const void* logits, int dtype, const int64_t* target, int N, int C, int64_t ignore_index,
                     float smoothing, float* partials, unsigned* counter, float* out, int mean, hipStream_t s) {
  if (N <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  return (int)(dtype == BF16 ? launch_fwd<uint16_t>(logits, target, N, C, ignore_index, smoothing, partials, counter, out, mean, s)
               : dtype == F16 ? launch_fwd<f16_t>(logits, target, N, C, ignore_index, smoothing, partials, counter, out, mean, s)
                              : launch_fwd<float>(logits, target, N, C, ignore_index, smoothing, partials, counter, out, mean, s));
}

RK_API int rk_ce_bwd(const void* logits, int dtype, const int64_t* target, void* dlogits, int N, int C,
                     int64_t ignore_index, float smoothing, const float* grad_out, const float* stats, int mean,
                     hipStream_t s) {
  if (N <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  return (int)(dtype == BF16 ? launch_bwd<uint16_t>(logits, target, dlogits, N, C, ignore_index, smoothing, grad_out, stats, mean, s)
               : dtype == F16 ? launch_bwd<f16_t>(logits, target, dlogits, N, C, ignore_index, smoothing, grad_out, stats, mean, s)
                              : launch_bwd<float>(logits, target, dlogits, N, C, ignore_index, smoothing, grad_out, stats, mean, s));
}

RK_API int rk_ce_train(const void* logits, int dtype, const int64_t* target, void* dlogits, int N, int C,
                       int64_t ignore_index, float smoothing, float grad_scale, float* partials, unsigned* counter,
                       float* out, int mean, float* acc, float* ring, int64_t* slot, int ring_size, float acc_scale,
                       int sync, hipStream_t s) {
  if (N <= 0 || C <= 0 || N > 65536) return (int)hipErrorInvalidValue;
  const bool wave = C > 64;
  const int rows = wave ? 4 : 256;
  const int grid = (N + rows - 1) / rows;
  CeTrainAcc la{acc, ring, slot, ring_size, acc_scale, sync};
#define RK_CT(T, W) ce_train_kernel<T, W><<<grid, 256, 0, s>>>((const T*)logits, target, (T*)dlogits, N, C, ignore_index, \
                                                               smoothing, grad_scale, partials, counter, out, mean, la)
  if (dtype == BF16) {
    if (wave) RK_CT(uint16_t, true); else RK_CT(uint16_t, false);
  } else if (dtype == F16) {
    if (wave) RK_CT(f16_t, true); else RK_CT(f16_t, false);
  } else {
    if (wave) RK_CT(float, true); else RK_CT(float, false);
  }
#undef RK_CT
  return (int)hipGetLastError();
}

RK_API int rk_ce_partials_needed(int N, int C) {
  const int rows = C > 64 ? 4 : 256;
  return 2 * ((N + rows - 1) / rows);
}
