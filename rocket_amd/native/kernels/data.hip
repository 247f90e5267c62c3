// Small data-path kernels that replace chains of PyTorch launches.
//
// rk_gather_rows  – batch assembly for HBM-resident datasets: out_t[r] = src_t[idx[r]] for up
//                   to 4 aligned tensors in ONE launch (a LeNet batch is a 3 KB image row and
//                   an 8 B label row per sample; torch needs one index_select per tensor).
//                   Rows are copied with 16 B vectors when size/alignment allow.
// rk_loss_accum   – the Loss capsule's per-micro-step bookkeeping on the device:
//                   acc += loss * scale; on a gradient-sync step ring[slot] = acc, slot advances,
//                   acc = 0.  One single-thread launch instead of five elementwise kernels,
//                   and graph-capturable (the ring slot lives in device memory).
#include "rk_common.h"
#include "rows_common.h"

#include <algorithm>

#include <hip/hip_ext.h>

namespace {

constexpr int kMaxGather = 4;

struct GatherArgs {
  const char* src[kMaxGather];
  char* dst[kMaxGather];
  int64_t row_bytes[kMaxGather];
  int64_t src_rows[kMaxGather];
  int ntensors;
  uint64_t* trace;  // diagnostics: [blocks][2] start / end stamps (s_memrealtime), or null
  int pieces[kMaxGather];  // wave work items per row of tensor t (ceil(row_bytes / kPiece))
};

// grid: x = row blocks (kRowsPerBlock rows each), y = tensor.  One wave copies one row; each lane
// issues all of its (up to kUnroll) vector loads before the first store, so a row costs one HBM
// round trip instead of one per 1 KB chunk (a 3 KB LeNet image row: 4 -> 1).
constexpr int kThreads = 256;
constexpr int kRowsPerBlock = kThreads / 64;
// rows longer than this are cut into pieces copied by different waves (a 3x224x224 bf16 image row is
// 294 KiB: one wave per row left a 128-row ViT batch on 32 CUs, 0.6 TB/s)
constexpr int64_t kPiece = 16384;
constexpr int kUnroll = 4;  // the register pin below names 4 values
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename V>
__device__ __forceinline__ void copy_row(const V* __restrict__ src, V* __restrict__ dst, int n, int lane) {
  for (int base = 0; base < n; base += 64 * kUnroll) {
    V v[kUnroll];
    // no branches at all (tail lanes re-copy the last element: same value to the same address),
    // so the compiler cannot sink each load into its store's branch — all loads stay in flight
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) v[j] = src[min(base + lane + 64 * j, n - 1)];
    if constexpr (sizeof(V) >= 4) asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) dst[min(base + lane + 64 * j, n - 1)] = v[j];
  }
}

__device__ __forceinline__ void copy_one(const GatherArgs& a, int t, int64_t s, int64_t r, int lane, int piece);

__global__ void __launch_bounds__(kThreads) gather_rows_kernel(GatherArgs a, const int64_t* __restrict__ idx,
                                                               int64_t nrows) {
  const int t = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);  // (row, piece) of tensor t
  const int np = a.pieces[t];
  const int64_t r = item / np;
  const int piece = (int)(item - r * np);
  uint64_t* tr = a.trace ? a.trace + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 2 : nullptr;
  if (tr && threadIdx.x == 0) tr[0] = __builtin_amdgcn_s_memrealtime();
  if (r < nrows) copy_one(a, t, idx[r], r, lane, piece);
  if (tr && threadIdx.x == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
}

// rows[i] = table[cursor' + i] for the next batch, cursor' = meta[0] + n_cur (stored back);
// meta = {cursor, table length}.  One block.
__global__ void __launch_bounds__(256) rows_next_kernel(const int64_t* __restrict__ table, int64_t* meta,
                                                        int64_t* __restrict__ rows, int n_cur, int bs) {
  rows_next_block(table, meta, rows, n_cur, bs);
}

__device__ __forceinline__ void copy_one(const GatherArgs& a, int t, int64_t s, int64_t r, int lane, int piece) {
  s = s < 0 ? s + a.src_rows[t] : s;
  s = s < 0 ? 0 : (s >= a.src_rows[t] ? a.src_rows[t] - 1 : s);
  const int64_t full = a.row_bytes[t];
  const int64_t off = (int64_t)piece * kPiece;
  const int64_t rb = full - off < kPiece || a.pieces[t] == 1 ? full - off : kPiece;  // this piece's bytes
  const char* __restrict__ src = a.src[t] + s * full + off;
  char* __restrict__ dst = a.dst[t] + r * full + off;
  if (((rb | (int64_t)a.src[t] | (int64_t)a.dst[t]) & 15) == 0) {
    copy_row((const u32x4*)src, (u32x4*)dst, (int)(rb >> 4), lane);
  } else if (((rb | (int64_t)a.src[t] | (int64_t)a.dst[t]) & 7) == 0) {
    copy_row((const uint64_t*)src, (uint64_t*)dst, (int)(rb >> 3), lane);
  } else {
    copy_row(src, dst, (int)rb, lane);
  }
}

__global__ void loss_accum_kernel(const float* __restrict__ loss, float* acc, float* ring, int64_t* slot,
                                  int ring_size, float scale, int sync) {
  float v = acc[0] + loss[0] * scale;
  if (sync) {
    int64_t k = slot[0];
    ring[k] = v;
    slot[0] = (k + 1) % ring_size;
    v = 0.f;
  }
  acc[0] = v;
}

}  // namespace

thread_local int g_gather_any_order = 0;
static uint64_t* g_gather_trace = nullptr;
// diagnostics: block start / end stamps of every following gather launch ([blocks][2] u64), or null
RK_API void rk_gather_set_trace(void* tr) { g_gather_trace = (uint64_t*)tr; }

// srcs/dsts: arrays of device pointers (host memory), row_bytes/src_rows per tensor.
static int gather_launch(int ntensors, const void* const* srcs, void* const* dsts, const int64_t* row_bytes,
                         const int64_t* src_rows, const int64_t* idx, int64_t nrows, hipStream_t s) {
  if (ntensors <= 0 || nrows <= 0) return 0;
  if (ntensors > kMaxGather) return (int)hipErrorInvalidValue;
  GatherArgs a{};
  for (int i = 0; i < ntensors; ++i) {
    a.src[i] = (const char*)srcs[i];
    a.dst[i] = (char*)dsts[i];
    a.row_bytes[i] = row_bytes[i];
    a.src_rows[i] = src_rows[i];
    if (row_bytes[i] > ((int64_t)1 << 34) || src_rows[i] <= 0) return (int)hipErrorInvalidValue;
  }
  a.ntensors = ntensors;
  a.trace = g_gather_trace;
  int64_t maxp = 1;
  for (int i = 0; i < ntensors; ++i) {
    // pieces of whole 16-byte vectors only when the row is vector-aligned (else one wave per row)
    const bool vec = ((row_bytes[i] | (int64_t)srcs[i] | (int64_t)dsts[i]) & 15) == 0;
    a.pieces[i] = vec ? (int)((row_bytes[i] + kPiece - 1) / kPiece) : 1;
    maxp = std::max<int64_t>(maxp, a.pieces[i]);
  }
  dim3 grid((unsigned)((nrows * maxp + kRowsPerBlock - 1) / kRowsPerBlock), (unsigned)ntensors);
  if (g_gather_any_order) {
    // AQL barrier bit clear: the gather may start while the previous packet on the stream (the
    // last kernel of the step before) still runs; see rk_gather_rows_any_order
    g_gather_any_order = 0;
    void* args[] = {&a, &idx, &nrows};
    return (int)hipExtLaunchKernel((const void*)gather_rows_kernel, grid, dim3(kThreads), args, 0, s, nullptr, nullptr,
                                   hipExtAnyOrderLaunch);
  }
  gather_rows_kernel<<<grid, kThreads, 0, s>>>(a, idx, nrows);
  return (int)hipGetLastError();
}

RK_API int rk_gather_rows(int ntensors, const void* const* srcs, void* const* dsts, const int64_t* row_bytes,
                          const int64_t* src_rows, const int64_t* idx, int64_t nrows, hipStream_t s) {
  return gather_launch(ntensors, srcs, dsts, row_bytes, src_rows, idx, nrows, s);
}

// Deferred device-loader batches (runtime/data.py PendingRows): advance the epoch cursor past the
// current batch (n_cur rows) and stage the next batch's row indices (up to bs) into `rows`, which
// the next batch's consumer reads.  meta = {cursor, table length} (device).  Graph-capturable.
RK_API int rk_rows_next(const int64_t* table, int64_t* meta, int64_t* rows, int n_cur, int bs, hipStream_t s) {
  if (!table || !meta || !rows || n_cur < 0 || bs < 1) return (int)hipErrorInvalidValue;
  rows_next_kernel<<<1, 256, 0, s>>>(table, meta, rows, n_cur, bs);
  return (int)hipGetLastError();
}

// The NEXT rk_gather_rows on this thread is launched with hipExtAnyOrderLaunch: it does not wait
// for the previous packet on its stream to complete (every packet before that one has completed:
// that packet's own barrier bit waited for them).  Only for a gather whose destination and index
// table no in-flight packet touches — a device loader's ring slot, gathered one batch ahead
// (runtime/data.py DeviceLoader): it then overlaps the previous step's tail kernel instead of
// adding its own dispatch to the step's dependency chain.
RK_API void rk_gather_rows_any_order() { g_gather_any_order = 1; }

RK_API int rk_loss_accum(const float* loss, float* acc, float* ring, int64_t* slot, int ring_size, float scale,
                         int sync, hipStream_t s) {
  loss_accum_kernel<<<1, 1, 0, s>>>(loss, acc, ring, slot, ring_size, scale, sync);
  return (int)hipGetLastError();
}
