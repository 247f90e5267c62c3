// Launch-list replay of a captured HIP graph (the step executor for launch-bound training steps).
//
// Why: on MI355X / ROCm 7 every hipGraphLaunch costs a fixed ~5-8 us of GPU idle time at the
// graph boundary (measured: bench/graph_launch_probe.py, profiles/r1_lenet_graph_steady_kernels.md),
// while back-to-back kernel dispatches on one stream cost ~1-2 us each.  A LeNet step is ~50 us of
// kernels, so the boundary is >10% of it.  The graph is still captured (stream capture records
// every launch with its final arguments — pointers into the capture pool, frozen hyper-parameter
// tables, ...), but instead of instantiating it we walk its nodes once, in topological order,
// and re-issue them with plain stream launches on every replay: one ctypes call, N dispatches.
//
// Supported graphs: chains (single-stream captures).  Supported nodes: kernel (hipLaunchKernel with the node's own argument array, which stays
// valid while the graph is alive) and empty.  Anything else (memset/memcpy/event/host/child-graph
// nodes, module launches with an `extra` buffer) makes create() fail and the caller keeps
// replaying the instantiated graph.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#define RKG_API extern "C" __attribute__((visibility("default")))

namespace {

enum Kind { kKernel = 0 };

struct Op {
  Kind kind;
  const void* func = nullptr;
  dim3 grid, block;
  void** args = nullptr;
  unsigned shmem = 0;
};

struct LaunchList {
  std::vector<Op> ops;
};

thread_local std::string g_err;

int fail(const std::string& m, int code = 1) {
  g_err = m;
  return code;
}

}  // namespace

RKG_API const char* rkg_last_error() { return g_err.c_str(); }

// Builds the launch list of `graph` (a hipGraph_t kept alive by the caller).  *out = handle.
// Returns 0, or non-zero with rkg_last_error() naming the unsupported node.
RKG_API int rkg_create(void** out, void* graph_ptr) {
  *out = nullptr;
  hipGraph_t graph = (hipGraph_t)graph_ptr;
  size_t n = 0;
  if (hipGraphGetNodes(graph, nullptr, &n) != hipSuccess) return fail("hipGraphGetNodes failed");
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(graph, nodes.data(), &n) != hipSuccess) return fail("hipGraphGetNodes failed");
  size_t ne = 0;
  if (hipGraphGetEdges(graph, nullptr, nullptr, &ne) != hipSuccess) return fail("hipGraphGetEdges failed");
  std::vector<hipGraphNode_t> from(ne), to(ne);
  if (ne && hipGraphGetEdges(graph, from.data(), to.data(), &ne) != hipSuccess) return fail("hipGraphGetEdges failed");
  // Kahn topological order; ties keep the node-list (creation) order
  std::map<hipGraphNode_t, size_t> pos;
  for (size_t i = 0; i < n; ++i) pos[nodes[i]] = i;
  std::vector<int> indeg(n, 0);
  std::vector<std::vector<size_t>> succ(n);
  for (size_t e = 0; e < ne; ++e) {
    auto a = pos.find(from[e]), b = pos.find(to[e]);
    if (a == pos.end() || b == pos.end()) return fail("edge to an unknown node");
    succ[a->second].push_back(b->second);
    indeg[b->second]++;
  }
  // a single-stream capture is a chain; parallel branches (multi-stream capture, e.g. an
  // all-reduce forked off backward) would be serialised by a one-stream launch list
  for (size_t i = 0; i < n; ++i)
    if (succ[i].size() > 1 || indeg[i] > 1) return fail("graph has parallel branches");
  std::vector<size_t> order, ready;
  for (size_t i = 0; i < n; ++i)
    if (indeg[i] == 0) ready.push_back(i);
  while (!ready.empty()) {
    size_t best = 0;
    for (size_t k = 1; k < ready.size(); ++k)
      if (ready[k] < ready[best]) best = k;
    size_t i = ready[best];
    ready.erase(ready.begin() + best);
    order.push_back(i);
    for (size_t j : succ[i])
      if (--indeg[j] == 0) ready.push_back(j);
  }
  if (order.size() != n) return fail("graph has a cycle");

  auto* ll = new LaunchList();
  for (size_t i : order) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess) {
      delete ll;
      return fail("hipGraphNodeGetType failed");
    }
    Op op{};
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams p{};
      if (hipGraphKernelNodeGetParams(nodes[i], &p) != hipSuccess || p.func == nullptr) {
        delete ll;
        return fail("kernel node without parameters");
      }
      if (p.extra != nullptr) {
        delete ll;
        return fail("kernel node launched with an extra-argument buffer");
      }
      hipFuncAttributes fa;
      if (hipFuncGetAttributes(&fa, p.func) != hipSuccess) {
        delete ll;
        return fail("kernel node function is not a launchable host stub");
      }
      op.kind = kKernel;
      op.func = p.func;
      op.grid = p.gridDim;
      op.block = p.blockDim;
      op.args = p.kernelParams;
      op.shmem = p.sharedMemBytes;
    } else if (t == hipGraphNodeTypeMemset || t == hipGraphNodeTypeMemcpy) {
      // not replayed natively: hipGraphMemcpyNodeGetParams returns success but an unfilled
      // parameter block for captured 1-D copies (measured on ROCm 7.2), so their arguments cannot
      // be recovered reliably — such graphs keep hipGraphLaunch
      delete ll;
      return fail(std::string(t == hipGraphNodeTypeMemcpy ? "memcpy" : "memset") +
                  " node (only kernel nodes are replayed natively)");
    } else if (t == hipGraphNodeTypeEmpty) {
      continue;
    } else {
      delete ll;
      return fail("unsupported graph node type " + std::to_string((int)t));
    }
    ll->ops.push_back(op);
  }
  *out = ll;
  return 0;
}

// Text description of a graph's structure (tests / diagnostics): one line per node
// "N <index> <type> <kernel name or ->" in node-list order, then one line per edge "E <from> <to>".
// Returns the bytes needed (including the terminating NUL); writes at most `cap` bytes to `buf`.
RKG_API int64_t rkg_describe(void* graph_ptr, char* buf, int64_t cap) {
  hipGraph_t graph = (hipGraph_t)graph_ptr;
  size_t n = 0, ne = 0;
  if (hipGraphGetNodes(graph, nullptr, &n) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(graph, nodes.data(), &n) != hipSuccess) return -1;
  if (hipGraphGetEdges(graph, nullptr, nullptr, &ne) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> from(ne), to(ne);
  if (ne && hipGraphGetEdges(graph, from.data(), to.data(), &ne) != hipSuccess) return -1;
  std::map<hipGraphNode_t, size_t> pos;
  std::string out;
  for (size_t i = 0; i < n; ++i) {
    pos[nodes[i]] = i;
    hipGraphNodeType t;
    (void)hipGraphNodeGetType(nodes[i], &t);
    std::string name = "-";
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams p{};
      if (hipGraphKernelNodeGetParams(nodes[i], &p) == hipSuccess && p.func) {
        const char* nm = hipKernelNameRefByPtr(p.func, nullptr);
        if (nm) name = nm;
      }
    }
    out += "N " + std::to_string(i) + " " + std::to_string((int)t) + " " + name + "\n";
  }
  for (size_t e = 0; e < ne; ++e)
    out += "E " + std::to_string(pos[from[e]]) + " " + std::to_string(pos[to[e]]) + "\n";
  const int64_t need = (int64_t)out.size() + 1;
  if (buf && cap > 0) {
    const int64_t k = std::min<int64_t>(cap - 1, (int64_t)out.size());
    std::memcpy(buf, out.data(), (size_t)k);
    buf[k] = 0;
  }
  return need;
}

RKG_API int rkg_size(void* h) { return h ? (int)((LaunchList*)h)->ops.size() : 0; }

// Kind of op i (0 = kernel) or -1.
RKG_API int rkg_kind(void* h, int i) {
  auto* ll = (LaunchList*)h;
  return (ll && i >= 0 && i < (int)ll->ops.size()) ? (int)ll->ops[i].kind : -1;
}

RKG_API int rkg_launch(void* h, hipStream_t s) {
  auto* ll = (LaunchList*)h;
  if (!ll) return fail("null launch list");
  for (const Op& op : ll->ops) {
    hipError_t e = hipSuccess;
    switch (op.kind) {
      case kKernel:
        e = hipLaunchKernel(op.func, op.grid, op.block, op.args, op.shmem, s);
        break;
    }
    if (e != hipSuccess) return fail(std::string("replay launch failed: ") + hipGetErrorString(e), (int)e);
  }
  return 0;
}

RKG_API int rkg_destroy(void* h) {
  delete (LaunchList*)h;
  return 0;
}
