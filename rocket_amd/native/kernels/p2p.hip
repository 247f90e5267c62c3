// One-shot peer-to-peer all-reduce over xGMI for small gradient buckets (SURVEY §5
// "MI355X-native communication design": LeNet's 247 KB of fp32 gradients are latency-bound; RCCL's
// small-message path costs tens of µs plus a host hop between two HIP graphs).
//
// Every rank owns, in its own HBM, a double-buffered STAGE area (2 x cap floats) and a FLAGS area
// ([kMaxBlocks][8] u32, uncached).  Both are exported once with hipIpcGetMemHandle and mapped by
// every peer, so a kernel can read a peer's stage and write a peer's flags directly over xGMI.
//
// rk_p2p_allreduce(data, n): region b is the fixed stage range [b*kChunk, (b+1)*kChunk), handled by
// block b % grid (at most kMaxGrid blocks, block-stride):
//   1. copy data[region] into stage[parity][region]                         (local HBM)
//   2. release (L2 write-back, system scope), then store this block's epoch into
//      flags_peer[b][rank] of every peer; poll flags_self[b][peer] >= epoch for every peer
//   3. acquire (system scope), read region from all W stages (W loads in flight per vector),
//      sum in rank order 0..W-1 (bit-identical result on every rank), scale, write data[region].
// The epoch counter of block b lives in device memory (graph-capturable: no host-side step value)
// and selects the stage parity.  Double buffering makes a closing barrier unnecessary: a rank can
// only overwrite stage[p] two launches later, after every peer has signalled the launch in
// between, i.e. after every peer finished reading stage[p].  The block -> region map never
// changes, so the argument holds per block even when n differs between launches (all ranks issue
// the same sequence of launches).
//
// A poll that exceeds the timeout (30 s; a few seconds for the creation self-test) records an error
// in host-mapped memory and gives up instead of hanging the GPU; the timed-out block then skips its
// reduce and leaves its gradients untouched.  So that no rank applies those un-reduced gradients,
// the timed-out block also raises the found flag of up to two device loss-scaling blocks
// (optim_common.h AmpSlot: the optimizer's fault guard, and the fp16 scaler's state): the fused
// optimizer launch that follows in the same stream/graph then skips the whole update, step counter
// included, exactly as for an fp16 overflow.  The host reads the error word (a plain host load) on
// every launch and replay and raises.  The kernel never waits on anything but peer flags.
#include "rk_common.h"
#include "optim_common.h"

#include <cstring>
#include <new>

namespace {
using rk::f32x4;

constexpr int kMaxPeers = 8;
constexpr int kThreads = 256;
constexpr int kVec = 4;                              // floats per 16-byte vector
constexpr int kUnroll = 2;                           // vectors per thread
constexpr int kChunk = kThreads * kVec * kUnroll;    // 2048 floats per block (8 KB)
constexpr int kMaxGrid = 256;                        // blocks per launch (block-stride over regions)
constexpr uint64_t kTicksPerSecond = 100000000ull;   // s_memrealtime runs at 100 MHz

struct P2PArgs {
  float* stage[kMaxPeers];      // every rank's stage base (self included), 2 * cap floats each
  unsigned* flags[kMaxPeers];   // every rank's flags base, [kMaxBlocks][kMaxPeers]
  unsigned* epoch;              // local, [kMaxBlocks]
  unsigned* err;                // host-mapped error word
  float* skip[2];               // AmpSlot found flags raised on a timeout (or null)
  float* data;
  int64_t n, cap;
  uint64_t timeout_ticks;
  float scale;
  int rank, world;
  // loss-ring fold (rk_p2p_set_loss_ring; lring null = none): element lidx of data is the step's
  // loss accumulator (the side channel); its reduced value goes to lring[*lslot] (the slot advances,
  // mod lsize) and the element is cleared -- the Loss capsule's separate bookkeeping launch
  float* lring;
  int64_t* lslot;
  int64_t lidx;
  int lsize;
};

__device__ __forceinline__ void loss_fold(const P2PArgs& a, float v) {
  const int64_t k = a.lslot[0];
  a.lring[k] = v;
  a.lslot[0] = (k + 1) % a.lsize;
  a.data[a.lidx] = 0.f;
}

__device__ __forceinline__ unsigned load_flag(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Write-back of the plain all-reduce: the averaged gradient goes back in place.
struct StoreSum {
  __device__ __forceinline__ void vec(float* data, int64_t j, f32x4 s) const { *(f32x4*)(data + j) = s; }
  __device__ __forceinline__ void one(float* data, int64_t j, float s) const { data[j] = s; }
};

// One region b (kChunk floats): stage, signal, wait, reduce.  False when a peer timed out.
template <int W, class Out = StoreSum>
__device__ __forceinline__ bool p2p_region(const P2PArgs& a, int b, unsigned& s_ep, int& s_timeout,
                                           const Out& out = Out{}) {
  const int t = threadIdx.x;
  if (t == 0) {
    s_ep = a.epoch[b] + 1;
    s_timeout = 0;
  }
  __syncthreads();
  const unsigned ep = s_ep;
  const int64_t par = (int64_t)(ep & 1) * a.cap;
  const int64_t base = (int64_t)b * kChunk;

  // 1. local contribution -> own stage
  float* mine = a.stage[a.rank] + par;
  const bool full = base + kChunk <= a.n;  // block-uniform: no per-vector bounds branches
  if (full) {
    f32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) v[u] = *(const f32x4*)(a.data + base + (int64_t)(u * kThreads + t) * kVec);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) *(f32x4*)(mine + base + (int64_t)(u * kThreads + t) * kVec) = v[u];
  } else {
    for (int64_t j = base + t; j < a.n && j < base + kChunk; j += kThreads) mine[j] = a.data[j];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();

  // 2. signal every peer, then wait for every peer's signal (wave 0, lane p <-> peer p)
  if (t < 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back this XCD's L2
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (t < a.world) {
      __hip_atomic_store(a.flags[t] + b * kMaxPeers + a.rank, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned* f = a.flags[a.rank] + b * kMaxPeers + t;
      if ((int)(load_flag(f) - ep) < 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while ((int)(load_flag(f) - ep) < 0) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
            __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            for (int k = 0; k < 2; ++k)
              if (a.skip[k]) __hip_atomic_store(a.skip[k] + 2, 1.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_timeout = 1;
            break;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // a peer that never signalled: its stage holds stale data -- leave this block's gradients
  // untouched (the raised skip flags make the following optimizer launch a no-op)
  if (s_timeout) return false;
  if (t >= 64) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // this wave's view of the peers' stages
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }

  // 3. reduce: all W contributions of each vector in flight, summed in rank order
  if (full) {
    f32x4 v[kUnroll][W];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
#pragma unroll
      for (int r = 0; r < W; ++r)
        v[u][r] = __builtin_nontemporal_load((const f32x4*)(a.stage[r] + par + base + (int64_t)(u * kThreads + t) * kVec));
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      f32x4 s = v[u][0];
#pragma unroll
      for (int r = 1; r < W; ++r) s += v[u][r];
      const int64_t j = base + (int64_t)(u * kThreads + t) * kVec;
      if (a.lring != nullptr && (uint64_t)(a.lidx - j) < (uint64_t)kVec) {  // the loss slot's vector
        s *= a.scale;
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
          if (j + k == a.lidx) loss_fold(a, s[k]);
          else out.one(a.data, j + k, s[k]);
        }
      } else {
        out.vec(a.data, j, s * a.scale);
      }
    }
  } else {
    for (int64_t j = base + t; j < a.n && j < base + kChunk; j += kThreads) {
      float v[W];
#pragma unroll
      for (int r = 0; r < W; ++r) v[r] = __builtin_nontemporal_load(a.stage[r] + par + j);
      float s = v[0];
#pragma unroll
      for (int r = 1; r < W; ++r) s += v[r];
      if (a.lring != nullptr && j == a.lidx) loss_fold(a, s * a.scale);
      else out.one(a.data, j, s * a.scale);
    }
  }
  if (t == 0) a.epoch[b] = ep;
  __syncthreads();  // s_ep / s_timeout are rewritten by the next region
  return true;
}

// A grid of at most kMaxGrid blocks walks the regions (block-stride): the number of spinning
// blocks is bounded whatever the bucket size, so the kernels of all ranks stay co-resident even
// when several ranks share one device (the single-GPU rehearsal of the multi-GPU paths).
template <int W>
__global__ void __launch_bounds__(kThreads) p2p_allreduce_kernel(P2PArgs a, int nregions) {
  __shared__ unsigned s_ep;
  __shared__ int s_timeout;
  for (int b = blockIdx.x; b < nregions; b += gridDim.x)
    if (!p2p_region<W>(a, b, s_ep, s_timeout)) return;
}

// ---------------------------------------------------------------------------------------------
// All-reduce + AdamW update in one launch (the data-parallel LeNet step at W > 1: backward ->
// THIS -> next step, instead of backward -> all-reduce -> optimizer).  The reduced gradient of a
// parameter element is never stored as such: its block applies the update right away (p, m, v,
// bf16/fp16 shadow, gradient cleared or stored), exactly the arithmetic of the multi-tensor update
// (rk_opt::adam_update).  Elements of the flat buffer that belong to no segment (16-byte padding,
// the loss side channel) get the plain average.  Armed by the host only when that is exact: a
// gradient-sync step, no AMP scaler, an Adam-family optimizer whose every active parameter lies in
// P2P buckets.  A peer timeout: the timed-out block leaves its elements un-updated and raises the
// fault guard's found flag, the host raises on the error word (the step is not usable anyway).
constexpr int kMaxSeg = 32;
struct P2PUpd {
  const int64_t* segs;  // [nseg][10]: rk_opt::TensorRec (8 x int64), flat start, 0
  const rk_opt::AdamHyper* hyper;
  float* step;
  unsigned* counter;
  float* amp;  // AmpSlot block whose found flag skips the update (the fault guard), may be null
  int nseg, ngroups, zero_grads, advance;
};

struct UpdOut {
  const rk_opt::TensorRec* rec;
  const int64_t* start;
  const rk_opt::AdamStep* ks;
  int nseg, zero_grads;
  float gs;
  bool skip;
  __device__ __forceinline__ void one(float* data, int64_t j, float s) const {
    int q = -1;
    for (int i = 0; i < nseg; ++i)
      if (j >= start[i] && j < start[i] + rec[i].n) q = i;
    if (q < 0 || skip) {  // padding / side channel; a skipped step clears (or keeps) the gradient
      data[j] = (q >= 0 && zero_grads) ? 0.f : s;
      return;
    }
    const rk_opt::TensorRec& tr = rec[q];
    const int64_t e = j - start[q];
    rk_opt::epi_apply(tr, ks[tr.group], e, rk_opt::epi_fetch(tr, e), s * gs, zero_grads);
  }
  __device__ __forceinline__ void vec(float* data, int64_t j, f32x4 s) const {
#pragma unroll
    for (int k = 0; k < kVec; ++k) one(data, j + k, s[k]);
  }
};

template <int W>
__global__ void __launch_bounds__(kThreads) p2p_allreduce_upd_kernel(P2PArgs a, int nregions, P2PUpd u) {
  __shared__ unsigned s_ep;
  __shared__ int s_timeout;
  __shared__ rk_opt::TensorRec s_rec[kMaxSeg];
  __shared__ int64_t s_start[kMaxSeg];
  __shared__ rk_opt::AdamStep s_ks[4];
  __shared__ float s_cur, s_gs;
  __shared__ int s_skip;
  const int t = threadIdx.x;
  for (int i = t; i < u.nseg * 10; i += kThreads) {
    const int q = i / 10, f = i % 10;
    if (f < 8) ((int64_t*)&s_rec[q])[f] = u.segs[i];
    else if (f == 8) s_start[q] = u.segs[i];
  }
  if (t == 0) {
    s_cur = u.step[0];
    s_skip = u.amp != nullptr && u.amp[rk_opt::kAmpFound] != 0.f;
    s_gs = u.amp ? u.amp[rk_opt::kAmpInv] : 1.f;
  }
  __syncthreads();
  if (t < u.ngroups) s_ks[t] = rk_opt::adam_step(u.hyper[t], s_cur + 1.f);
  __syncthreads();
  const UpdOut out{s_rec, s_start, s_ks, u.nseg, u.zero_grads, s_gs, s_skip != 0};
  for (int b = blockIdx.x; b < nregions; b += gridDim.x)
    if (!p2p_region<W>(a, b, s_ep, s_timeout, out)) break;
  // every block takes its ticket (a timed-out one too): the last one advances the step counter and
  // consumes the guard's found flag, as the optimizer launch this one replaces would
  if (u.advance) rk_opt::advance_step(u.step, u.counter, s_skip != 0, s_cur, u.amp);
}

struct P2PCtx {
  int rank = 0, world = 0, device = 0;
  double timeout_s = 30.0;
  int64_t cap = 0;
  int max_blocks = 0;
  float* stage = nullptr;
  unsigned* flags = nullptr;
  unsigned* epoch = nullptr;
  unsigned* err_h = nullptr;
  unsigned* err_d = nullptr;
  float* skip[2] = {nullptr, nullptr};
  float* peer_stage[kMaxPeers] = {};
  unsigned* peer_flags[kMaxPeers] = {};
  bool mapped[kMaxPeers] = {};
  // the next launch's loss-ring fold (rk_p2p_set_loss_ring), consumed by it
  float* lf_ring = nullptr;
  int64_t* lf_slot = nullptr;
  int64_t lf_idx = -1;
  int lf_size = 0;
};

constexpr int kHandleBytes = (int)sizeof(hipIpcMemHandle_t);

void release(P2PCtx* c) {
  for (int r = 0; r < kMaxPeers; ++r) {
    if (!c->mapped[r]) continue;
    (void)hipIpcCloseMemHandle(c->peer_stage[r]);
    (void)hipIpcCloseMemHandle(c->peer_flags[r]);
  }
  if (c->stage) (void)hipFree(c->stage);
  if (c->flags) (void)hipFree(c->flags);
  if (c->epoch) (void)hipFree(c->epoch);
  if (c->err_h) (void)hipHostFree(c->err_h);
  delete c;
}

}  // namespace

// bytes of one exported handle set (stage + flags)
RK_API int rk_p2p_handle_bytes() { return 2 * kHandleBytes; }
RK_API int rk_p2p_chunk() { return kChunk; }

// Allocate this rank's stage/flags, export their IPC handles into `handles` (rk_p2p_handle_bytes()).
RK_API int rk_p2p_create(int rank, int world, int64_t cap, void** out, void* handles) {
  if (world < 1 || world > kMaxPeers || rank < 0 || rank >= world || cap <= 0) return (int)hipErrorInvalidValue;
  auto* c = new (std::nothrow) P2PCtx();
  if (!c) return (int)hipErrorOutOfMemory;
  c->rank = rank;
  c->world = world;
  c->cap = (cap + kChunk - 1) / kChunk * kChunk;
  c->max_blocks = (int)(c->cap / kChunk);
  hipError_t e = hipGetDevice(&c->device);
  if (e == hipSuccess) e = hipMalloc((void**)&c->stage, 2 * c->cap * sizeof(float));
  if (e == hipSuccess)
    e = hipExtMallocWithFlags((void**)&c->flags, (size_t)c->max_blocks * kMaxPeers * sizeof(unsigned),
                              hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMalloc((void**)&c->epoch, (size_t)c->max_blocks * sizeof(unsigned));
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->err_h, sizeof(unsigned), hipHostMallocMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c->err_d, c->err_h, 0);
  if (e == hipSuccess) e = hipMemset(c->flags, 0, (size_t)c->max_blocks * kMaxPeers * sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(c->epoch, 0, (size_t)c->max_blocks * sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(c->stage, 0, 2 * c->cap * sizeof(float));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  hipIpcMemHandle_t hs, hf;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&hs, c->stage);
  if (e == hipSuccess) e = hipIpcGetMemHandle(&hf, c->flags);
  if (e != hipSuccess) {
    release(c);
    return (int)e;
  }
  *c->err_h = 0;
  std::memcpy(handles, &hs, kHandleBytes);
  std::memcpy((char*)handles + kHandleBytes, &hf, kHandleBytes);
  *out = c;
  return 0;
}

// Map every peer's stage/flags; `all` = world consecutive handle sets in rank order.
RK_API int rk_p2p_open(void* ctx, const void* all) {
  auto* c = (P2PCtx*)ctx;
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank) {
      c->peer_stage[r] = c->stage;
      c->peer_flags[r] = c->flags;
      continue;
    }
    hipIpcMemHandle_t hs, hf;
    std::memcpy(&hs, (const char*)all + (size_t)r * 2 * kHandleBytes, kHandleBytes);
    std::memcpy(&hf, (const char*)all + (size_t)r * 2 * kHandleBytes + kHandleBytes, kHandleBytes);
    void *ps = nullptr, *pf = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&ps, hs, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    e = hipIpcOpenMemHandle(&pf, hf, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      (void)hipIpcCloseMemHandle(ps);
      return (int)e;
    }
    c->peer_stage[r] = (float*)ps;
    c->peer_flags[r] = (unsigned*)pf;
    c->mapped[r] = true;
  }
  return 0;
}

static int p2p_args(P2PCtx* c, float* data, int64_t n, float scale, P2PArgs& a) {
  if (n > c->cap || ((uintptr_t)data & 15)) return (int)hipErrorInvalidValue;
  for (int r = 0; r < c->world; ++r) {
    if (!c->peer_stage[r]) return (int)hipErrorNotInitialized;
    a.stage[r] = c->peer_stage[r];
    a.flags[r] = c->peer_flags[r];
  }
  for (int r = c->world; r < kMaxPeers; ++r) {  // never dereferenced (r >= world), keep them valid anyway
    a.stage[r] = c->stage;
    a.flags[r] = c->flags;
  }
  a.epoch = c->epoch;
  a.err = c->err_d;
  a.skip[0] = c->skip[0];
  a.skip[1] = c->skip[1];
  a.data = data;
  a.n = n;
  a.cap = c->cap;
  a.scale = scale;
  a.timeout_ticks = (uint64_t)(c->timeout_s * (double)kTicksPerSecond);
  a.rank = c->rank;
  a.world = c->world;
  if (c->lf_ring && c->lf_idx >= 0 && c->lf_idx < n) {
    a.lring = c->lf_ring;
    a.lslot = c->lf_slot;
    a.lidx = c->lf_idx;
    a.lsize = c->lf_size;
  }
  c->lf_ring = nullptr;  // one launch only
  c->lf_idx = -1;
  return 0;
}

// data[0:n] <- scale * sum over ranks (in place, stream-ordered, graph-capturable).  16-byte
// aligned data; n <= cap.
RK_API int rk_p2p_allreduce(void* ctx, float* data, int64_t n, float scale, hipStream_t s) {
  auto* c = (P2PCtx*)ctx;
  if (n <= 0) return 0;
  P2PArgs a{};
  if (int rc = p2p_args(c, data, n, scale, a)) return rc;
  const int regions = (int)((n + kChunk - 1) / kChunk);
  const int blocks = regions < kMaxGrid ? regions : kMaxGrid;
  switch (c->world) {
    case 1: p2p_allreduce_kernel<1><<<blocks, kThreads, 0, s>>>(a, regions); break;
    case 2: p2p_allreduce_kernel<2><<<blocks, kThreads, 0, s>>>(a, regions); break;
    case 3: p2p_allreduce_kernel<3><<<blocks, kThreads, 0, s>>>(a, regions); break;
    case 4: p2p_allreduce_kernel<4><<<blocks, kThreads, 0, s>>>(a, regions); break;
    case 5: p2p_allreduce_kernel<5><<<blocks, kThreads, 0, s>>>(a, regions); break;
    case 6: p2p_allreduce_kernel<6><<<blocks, kThreads, 0, s>>>(a, regions); break;
    case 7: p2p_allreduce_kernel<7><<<blocks, kThreads, 0, s>>>(a, regions); break;
    default: p2p_allreduce_kernel<8><<<blocks, kThreads, 0, s>>>(a, regions); break;
  }
  return (int)hipGetLastError();
}

// The same all-reduce with the Adam/AdamW update applied in its write-back (P2PUpd above).
// segs: device int64 [nseg][10] (TensorRec, flat start into data, 0), nseg <= 32, segments disjoint
// and inside [0, n); hyper: AdamHyper[ngroups] (ngroups <= 4); step / counter: the optimizer's
// device step and ticket counter; amp: its AmpSlot block or null; advance: this launch advances
// the step (the optimizer's last bucket).
RK_API int rk_p2p_allreduce_adam(void* ctx, float* data, int64_t n, float scale, const int64_t* segs, int nseg,
                                 const void* hyper, int ngroups, float* step, unsigned* counter, float* amp,
                                 int zero_grads, int advance, hipStream_t s) {
  auto* c = (P2PCtx*)ctx;
  if (n <= 0) return 0;
  if (nseg < 0 || nseg > kMaxSeg || (nseg && !segs) || ngroups < 1 || ngroups > 4 || !hyper || !step || !counter)
    return (int)hipErrorInvalidValue;
  P2PArgs a{};
  if (int rc = p2p_args(c, data, n, scale, a)) return rc;
  P2PUpd u{segs, (const rk_opt::AdamHyper*)hyper, step, counter, amp, nseg, ngroups, zero_grads, advance};
  const int regions = (int)((n + kChunk - 1) / kChunk);
  const int blocks = regions < kMaxGrid ? regions : kMaxGrid;
  switch (c->world) {
    case 1: p2p_allreduce_upd_kernel<1><<<blocks, kThreads, 0, s>>>(a, regions, u); break;
    case 2: p2p_allreduce_upd_kernel<2><<<blocks, kThreads, 0, s>>>(a, regions, u); break;
    case 3: p2p_allreduce_upd_kernel<3><<<blocks, kThreads, 0, s>>>(a, regions, u); break;
    case 4: p2p_allreduce_upd_kernel<4><<<blocks, kThreads, 0, s>>>(a, regions, u); break;
    case 5: p2p_allreduce_upd_kernel<5><<<blocks, kThreads, 0, s>>>(a, regions, u); break;
    case 6: p2p_allreduce_upd_kernel<6><<<blocks, kThreads, 0, s>>>(a, regions, u); break;
    case 7: p2p_allreduce_upd_kernel<7><<<blocks, kThreads, 0, s>>>(a, regions, u); break;
    default: p2p_allreduce_upd_kernel<8><<<blocks, kThreads, 0, s>>>(a, regions, u); break;
  }
  return (int)hipGetLastError();
}

// The NEXT all-reduce launch on this context also folds the loss bookkeeping in: element idx of
// its buffer (the loss side channel) is averaged as usual, stored to ring[*slot], *slot advances
// mod size, and the element is cleared.  ring / slot: device fp32 [size] / int64 [1].
RK_API int rk_p2p_set_loss_ring(void* ctx, float* ring, int64_t* slot, int size, int64_t idx) {
  if (!ctx || !ring || !slot || size < 1 || idx < 0) return (int)hipErrorInvalidValue;
  auto* c = (P2PCtx*)ctx;
  c->lf_ring = ring;
  c->lf_slot = slot;
  c->lf_size = size;
  c->lf_idx = idx;
  return 0;
}

// Peer-poll timeout of later launches (seconds; default 30).  The creation self-test uses a short one.
RK_API int rk_p2p_set_timeout(void* ctx, double seconds) {
  if (!ctx || !(seconds > 0.0)) return (int)hipErrorInvalidValue;
  ((P2PCtx*)ctx)->timeout_s = seconds;
  return 0;
}

// Device loss-scaling blocks (AmpSlot, >= 3 floats) whose found flag a timed-out launch raises, so
// the optimizer launch after it skips the update; null = none.  Later launches use them.
RK_API int rk_p2p_set_skip(void* ctx, float* a, float* b) {
  if (!ctx) return (int)hipErrorInvalidValue;
  ((P2PCtx*)ctx)->skip[0] = a;
  ((P2PCtx*)ctx)->skip[1] = b;
  return 0;
}

// Host address of the error word (host-mapped memory: Python polls it with a plain load).
RK_API void* rk_p2p_error_ptr(void* ctx) { return ((P2PCtx*)ctx)->err_h; }

// Clear the error word (after the caller has handled a reported timeout).
RK_API int rk_p2p_clear_error(void* ctx) {
  __atomic_store_n(((P2PCtx*)ctx)->err_h, 0u, __ATOMIC_RELEASE);
  return 0;
}

// 0 = healthy; 1 = a peer never signalled within the timeout (results of that launch are invalid)
RK_API int rk_p2p_error(void* ctx) { return (int)__atomic_load_n(((P2PCtx*)ctx)->err_h, __ATOMIC_ACQUIRE); }

RK_API int rk_p2p_destroy(void* ctx) {
  if (!ctx) return 0;
  (void)hipDeviceSynchronize();
  release((P2PCtx*)ctx);
  return 0;
}
