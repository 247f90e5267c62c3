// Native RCCL communicator and bucket reducer.
//
// * Communicator: ncclUniqueId is created on rank 0 and shipped to the other ranks by the
//   Python side over the host (gloo/TCP) group; ncclCommInitRank then builds the RCCL
//   communicator directly — no ProcessGroupNCCL, no watchdog thread, no per-call Python work.
//   Collectives are plain stream-ordered launches on the stream the caller passes, so they are
//   captured by HIP graphs like any kernel.
// * Reducer: gradient buckets are reduced on a dedicated high-priority HIP stream, fenced with
//   events against the compute stream: launch(i) records an event on the compute stream,
//   makes the comm stream wait for it and issues ncclAllReduce(avg) there (so the all-reduce of
//   bucket i overlaps the backward of the earlier layers); join() makes the compute stream
//   wait for every bucket launched since the previous join.  Event record/wait is the
//   fork/join pattern HIP stream capture understands, so a whole DP step can be one graph.
//
// xGMI note: RCCL picks ring/tree per message size; buckets are sized by the Python side
// (>= 1 MiB per peer shard) so that each of the 7 links moves a latency-amortised message.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#define RKR_API extern "C" __attribute__((visibility("default")))

namespace {

thread_local std::string g_err;

int fail_nccl(ncclResult_t r, const char* what) {
  g_err = std::string(what) + ": " + ncclGetErrorString(r);
  return 1000 + (int)r;
}
int fail_hip(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return (int)e;
}

#define NCCL_TRY(call, what)              \
  do {                                    \
    ncclResult_t _r = (call);             \
    if (_r != ncclSuccess) return fail_nccl(_r, what); \
  } while (0)
#define HIP_TRY(call, what)               \
  do {                                    \
    hipError_t _e = (call);               \
    if (_e != hipSuccess) return fail_hip(_e, what); \
  } while (0)

ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt64;
    case 4: return ncclInt32;
    case 5: return ncclUint8;
    default: return ncclFloat32;
  }
}

ncclRedOp_t to_op(int op) {
  switch (op) {
    case 1: return ncclAvg;
    case 2: return ncclMax;
    case 3: return ncclMin;
    default: return ncclSum;
  }
}

struct Comm {
  ncclComm_t nc = nullptr;
  int nranks = 1, rank = 0, device = 0;
};

struct Bucket {
  void* ptr = nullptr;
  int64_t count = 0;
  int dtype = 0;
  hipEvent_t ready = nullptr;  // recorded on the compute stream
  hipEvent_t done = nullptr;   // recorded on the comm stream
  bool pending = false;
};

struct Reducer {
  Comm* comm = nullptr;
  hipStream_t stream = nullptr;
  std::vector<Bucket> buckets;
};

}  // namespace

RKR_API const char* rkr_last_error() { return g_err.c_str(); }

RKR_API int rkr_unique_id_bytes() { return (int)sizeof(ncclUniqueId); }

RKR_API int rkr_unique_id(void* out) {
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

RKR_API int rkr_comm_init(void** out, int nranks, int rank, const void* id_bytes, int device) {
  *out = nullptr;
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  Comm* c = new Comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclResult_t r = ncclCommInitRank(&c->nc, nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail_nccl(r, "ncclCommInitRank");
  }
  *out = c;
  return 0;
}

RKR_API int rkr_comm_destroy(void* comm) {
  Comm* c = (Comm*)comm;
  if (!c) return 0;
  ncclResult_t r = c->nc ? ncclCommDestroy(c->nc) : ncclSuccess;
  delete c;
  return r == ncclSuccess ? 0 : fail_nccl(r, "ncclCommDestroy");
}

RKR_API int rkr_comm_abort(void* comm) {
  Comm* c = (Comm*)comm;
  if (!c) return 0;
  ncclResult_t r = c->nc ? ncclCommAbort(c->nc) : ncclSuccess;
  delete c;
  return r == ncclSuccess ? 0 : fail_nccl(r, "ncclCommAbort");
}

RKR_API int rkr_all_reduce(void* comm, void* buf, int64_t count, int dtype, int op, hipStream_t s) {
  Comm* c = (Comm*)comm;
  NCCL_TRY(ncclAllReduce(buf, buf, (size_t)count, to_nccl(dtype), to_op(op), c->nc, s), "ncclAllReduce");
  return 0;
}

RKR_API int rkr_broadcast(void* comm, void* buf, int64_t count, int dtype, int root, hipStream_t s) {
  Comm* c = (Comm*)comm;
  NCCL_TRY(ncclBroadcast(buf, buf, (size_t)count, to_nccl(dtype), root, c->nc, s), "ncclBroadcast");
  return 0;
}

RKR_API int rkr_all_gather(void* comm, const void* send, void* recv, int64_t count, int dtype, hipStream_t s) {
  Comm* c = (Comm*)comm;
  NCCL_TRY(ncclAllGather(send, recv, (size_t)count, to_nccl(dtype), c->nc, s), "ncclAllGather");
  return 0;
}

RKR_API int rkr_reduce_scatter(void* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                               hipStream_t s) {
  Comm* c = (Comm*)comm;
  NCCL_TRY(ncclReduceScatter(send, recv, (size_t)count, to_nccl(dtype), to_op(op), c->nc, s), "ncclReduceScatter");
  return 0;
}

// ---------------------------------------------------------------------------- reducer
RKR_API int rkr_reducer_create(void** out, void* comm, int nbuckets) {
  *out = nullptr;
  Comm* c = (Comm*)comm;
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  Reducer* r = new Reducer();
  r->comm = c;
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);  // hi = greatest priority
  hipError_t e = hipStreamCreateWithPriority(&r->stream, hipStreamNonBlocking, hi);
  if (e != hipSuccess) {
    delete r;
    return fail_hip(e, "hipStreamCreateWithPriority");
  }
  r->buckets.resize(nbuckets);
  for (auto& b : r->buckets) {
    HIP_TRY(hipEventCreateWithFlags(&b.ready, hipEventDisableTiming), "hipEventCreate");
    HIP_TRY(hipEventCreateWithFlags(&b.done, hipEventDisableTiming), "hipEventCreate");
  }
  *out = r;
  return 0;
}

RKR_API int rkr_reducer_set_bucket(void* red, int i, void* ptr, int64_t count, int dtype) {
  Reducer* r = (Reducer*)red;
  if (i < 0 || i >= (int)r->buckets.size()) return fail_hip(hipErrorInvalidValue, "bucket index");
  r->buckets[i].ptr = ptr;
  r->buckets[i].count = count;
  r->buckets[i].dtype = dtype;
  return 0;
}

// bucket i is complete on `compute`: average it across ranks on the comm stream
RKR_API int rkr_reducer_launch(void* red, int i, hipStream_t compute) {
  Reducer* r = (Reducer*)red;
  Bucket& b = r->buckets[i];
  HIP_TRY(hipEventRecord(b.ready, compute), "hipEventRecord(ready)");
  HIP_TRY(hipStreamWaitEvent(r->stream, b.ready, 0), "hipStreamWaitEvent(comm)");
  NCCL_TRY(ncclAllReduce(b.ptr, b.ptr, (size_t)b.count, to_nccl(b.dtype), ncclAvg, r->comm->nc, r->stream),
           "ncclAllReduce(bucket)");
  HIP_TRY(hipEventRecord(b.done, r->stream), "hipEventRecord(done)");
  b.pending = true;
  return 0;
}

// the compute stream waits for every bucket launched since the last join (no host wait)
RKR_API int rkr_reducer_join(void* red, hipStream_t compute) {
  Reducer* r = (Reducer*)red;
  for (auto& b : r->buckets) {
    if (!b.pending) continue;
    HIP_TRY(hipStreamWaitEvent(compute, b.done, 0), "hipStreamWaitEvent(compute)");
    b.pending = false;
  }
  return 0;
}

RKR_API int rkr_reducer_destroy(void* red) {
  Reducer* r = (Reducer*)red;
  if (!r) return 0;
  hipStreamSynchronize(r->stream);
  for (auto& b : r->buckets) {
    hipEventDestroy(b.ready);
    hipEventDestroy(b.done);
  }
  hipStreamDestroy(r->stream);
  delete r;
  return 0;
}
