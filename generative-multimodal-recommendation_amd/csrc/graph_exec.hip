// Native multi-stream executor of a captured HIP graph (round 5; the rec step of a BPR batch, common/trainer.py:
// 144-208 with models/diffmm.py:203-258).
//
// The eager rec step issues ~50 launches per batch from Python on three streams (the contrastive terms and the
// text projection beside the main chain); its host cost per launch (~10 us through ctypes) is as large as the
// GPU time, so the GPU waits on the host (scripts/host_vs_gpu_probe.py).  hipGraphLaunch removes the host cost
// but ran the captured step slower (round 4: 104 vs 96 ms per epoch, the three-stream overlap lost).  This
// executor keeps both: the step is captured once into a hipGraph (torch.cuda.CUDAGraph, keep_graph), its
// nodes are read back (kernel / memset / memcpy / empty nodes and their edges), put in a topological order
// and given streams - a node continues the stream of a predecessor it is the first successor of, else takes
// a new stream (up to 1 + n_side, then the stream whose last node is earliest) - and every edge that crosses
// streams becomes an event record + wait.  Stream 0 is the launch stream itself; streams 1.. are the caller's
// side streams (the ones its eager step uses, so the hardware-queue mapping is the eager step's) or, when none
// are given, the executor's own.  gmr_graph_exec_launch then issues the whole step from C++ in one call: each
// kernel through hipLaunchKernel with the node's own argument block (owned by the graph, which the caller keeps
// alive), the side streams forked from and joined back into the launch stream.  The same kernels with the same
// arguments in a dependency-respecting order: results equal the captured step's bit for bit.
#include <algorithm>
#include <new>
#include <vector>

#include "gmr_common.h"

#define GX_HIP(x)                                             \
  do {                                                        \
    hipError_t e__ = (x);                                     \
    if (e__ != hipSuccess) return gmr::hip_status(__func__, e__); \
  } while (0)

namespace {

int gx_fail(const char* fn, const char* msg) {
  gmr::set_error(fn, msg);
  return GMR_ERR_ARG;
}

enum NodeKind { NK_KERNEL, NK_MEMSET, NK_MEMCPY, NK_EMPTY };

struct ExecNode {
  int kind = NK_EMPTY;
  hipKernelNodeParams kp{};
  hipMemsetParams mp{};
  hipMemcpy3DParms cp{};
  int stream = 0;
  std::vector<int> waits;  // events (node ids) this node's stream waits on first
  bool record = false;     // record this node's event after it (a successor on another stream waits on it)
};

struct GraphExec {
  std::vector<ExecNode> nodes;  // in issue (topological) order; ids below index this vector
  std::vector<hipStream_t> streams;  // [0] unused (the launch stream); [1..] side streams
  bool own_streams = false;
  std::vector<hipEvent_t> events;  // per node id (null where no cross-stream successor)
  hipEvent_t fork = nullptr;
  std::vector<hipEvent_t> joins;  // per stream
  ~GraphExec() {
    for (hipEvent_t e : events)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : joins)
      if (e) (void)hipEventDestroy(e);
    if (fork) (void)hipEventDestroy(fork);
    if (own_streams)
      for (size_t i = 1; i < streams.size(); ++i)
        if (streams[i]) (void)hipStreamDestroy(streams[i]);
  }
};

int issue_memset(const hipMemsetParams& m, hipStream_t st) {
  hipError_t e = hipSuccess;
  if (m.elementSize == 1) {
    e = hipMemset2DAsync(m.dst, m.pitch ? m.pitch : m.width, (int)m.value, m.width, m.height ? m.height : 1, st);
  } else {
    for (size_t r = 0; r < (m.height ? m.height : 1) && e == hipSuccess; ++r) {
      char* row = static_cast<char*>(m.dst) + r * m.pitch;
      e = m.elementSize == 2 ? hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(row), (unsigned short)m.value,
                                                 m.width, st)
                             : hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(row), (int)m.value, m.width, st);
    }
  }
  return e == hipSuccess ? GMR_OK : GMR_ERR_ARG;
}

}  // namespace

extern "C" int gmr_graph_exec_create(void* graph, int32_t n_side, void* const* side_streams, void** exec_out) {
  GMR_ARG(graph && exec_out && n_side >= 0 && n_side <= 15, "graph, exec_out, n_side in [0, 15]");
  const int max_streams = 1 + n_side;
  *exec_out = nullptr;
  hipGraph_t g = static_cast<hipGraph_t>(graph);
  size_t n = 0;
  GX_HIP(hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> hn(n);
  if (n) GX_HIP(hipGraphGetNodes(g, hn.data(), &n));
  auto index_of = [&](hipGraphNode_t x) -> int {
    for (size_t i = 0; i < n; ++i)
      if (hn[i] == x) return (int)i;
    return -1;
  };
  std::vector<std::vector<int>> preds(n), succs(n);
  for (size_t i = 0; i < n; ++i) {
    size_t nd = 0;
    GX_HIP(hipGraphNodeGetDependencies(hn[i], nullptr, &nd));
    std::vector<hipGraphNode_t> d(nd);
    if (nd) GX_HIP(hipGraphNodeGetDependencies(hn[i], d.data(), &nd));
    for (hipGraphNode_t x : d) {
      const int j = index_of(x);
      GMR_ARG(j >= 0, "dependency outside the graph");
      preds[i].push_back(j);
      succs[j].push_back((int)i);
    }
  }
  // Kahn's order, lowest original index first among the ready nodes (capture order)
  std::vector<int> indeg(n), order;
  for (size_t i = 0; i < n; ++i) indeg[i] = (int)preds[i].size();
  std::vector<int> ready;
  for (size_t i = 0; i < n; ++i)
    if (!indeg[i]) ready.push_back((int)i);
  while (!ready.empty()) {
    auto it = std::min_element(ready.begin(), ready.end());
    const int v = *it;
    ready.erase(it);
    order.push_back(v);
    for (int w : succs[v])
      if (--indeg[w] == 0) ready.push_back(w);
  }
  GMR_ARG(order.size() == n, "graph has a cycle");
  GraphExec* ex = new (std::nothrow) GraphExec();
  GMR_ARG(ex, "out of host memory");
  std::vector<int> pos(n), stream_of(n, -1), tail;  // tail[s]: last node id issued on stream s
  std::vector<int> first_succ_taken(n, 0);
  for (size_t k = 0; k < n; ++k) pos[order[k]] = (int)k;
  ex->nodes.resize(n);
  ex->events.assign(n, nullptr);
  for (size_t k = 0; k < n; ++k) {
    const int v = order[k];
    ExecNode& nd = ex->nodes[k];
    hipGraphNodeType t;
    if (hipGraphNodeGetType(hn[v], &t) != hipSuccess) {
      delete ex;
      return gx_fail(__func__, "hipGraphNodeGetType failed");
    }
    hipError_t e = hipSuccess;
    if (t == hipGraphNodeTypeKernel) {
      nd.kind = NK_KERNEL;
      e = hipGraphKernelNodeGetParams(hn[v], &nd.kp);
      if (e == hipSuccess && (!nd.kp.func || !nd.kp.kernelParams)) e = hipErrorInvalidValue;
    } else if (t == hipGraphNodeTypeMemset) {
      nd.kind = NK_MEMSET;
      e = hipGraphMemsetNodeGetParams(hn[v], &nd.mp);
    } else if (t == hipGraphNodeTypeMemcpy) {
      nd.kind = NK_MEMCPY;
      e = hipGraphMemcpyNodeGetParams(hn[v], &nd.cp);
    } else if (t == hipGraphNodeTypeEmpty) {
      nd.kind = NK_EMPTY;
    } else {
      delete ex;
      return gx_fail(__func__, "graph node type not supported by the executor (kernel / memset / "
                                         "memcpy / empty only)");
    }
    if (e != hipSuccess) {
      delete ex;
      return gx_fail(__func__, "reading a graph node's parameters failed");
    }
    // stream: continue a predecessor's stream if it is still that stream's last node and this is the first
    // successor to claim it; else a new stream; else the stream whose last node was issued earliest
    int s = -1;
    for (int u : preds[v])
      if (!first_succ_taken[u] && tail[stream_of[u]] == u) {
        s = stream_of[u];
        first_succ_taken[u] = 1;
        break;
      }
    if (s < 0) {
      if ((int)tail.size() < max_streams) {
        s = (int)tail.size();
        tail.push_back(-1);
      } else {
        s = 0;
        for (int q = 1; q < (int)tail.size(); ++q)
          if (pos[tail[q]] < pos[tail[s]]) s = q;
      }
    }
    stream_of[v] = s;
    nd.stream = s;
    for (int u : preds[v])
      if (stream_of[u] != s) {
        nd.waits.push_back(u);
        ex->nodes[pos[u]].record = true;
      }
    tail[s] = v;
  }
  // ids in the executor are issue positions
  for (auto& nd : ex->nodes)
    for (int& w : nd.waits) w = pos[w];
  bool ok = true;
  ex->streams.assign(tail.size(), nullptr);
  ex->own_streams = side_streams == nullptr;
  for (size_t i = 1; i < ex->streams.size(); ++i) {
    if (side_streams) {
      ex->streams[i] = static_cast<hipStream_t>(side_streams[i - 1]);
      ok = ok && ex->streams[i] != nullptr;
    } else {
      ok = ok && hipStreamCreateWithFlags(&ex->streams[i], hipStreamNonBlocking) == hipSuccess;
    }
  }
  for (size_t k = 0; k < n && ok; ++k)
    if (ex->nodes[k].record) ok = hipEventCreateWithFlags(&ex->events[k], hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&ex->fork, hipEventDisableTiming) == hipSuccess;
  ex->joins.assign(tail.size(), nullptr);
  for (auto& e : ex->joins) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    delete ex;
    return gx_fail(__func__, "creating the executor's streams / events failed");
  }
  *exec_out = ex;
  return GMR_OK;
}

extern "C" int gmr_graph_exec_info(const void* exec, int64_t* nodes, int64_t* kernels, int64_t* streams,
                                   int64_t* cross_edges) {
  GMR_ARG(exec, "null executor");
  const GraphExec* ex = static_cast<const GraphExec*>(exec);
  int64_t k = 0, w = 0;
  for (const auto& nd : ex->nodes) {
    k += nd.kind == NK_KERNEL;
    w += (int64_t)nd.waits.size();
  }
  if (nodes) *nodes = (int64_t)ex->nodes.size();
  if (kernels) *kernels = k;
  if (streams) *streams = (int64_t)ex->streams.size();
  if (cross_edges) *cross_edges = w;
  return GMR_OK;
}

extern "C" int gmr_graph_exec_launch(void* exec, void* stream) {
  GMR_ARG(exec, "null executor");
  GraphExec* ex = static_cast<GraphExec*>(exec);
  const hipStream_t s0 = (hipStream_t)stream;
  if (ex->streams.size() > 1) {
    GX_HIP(hipEventRecord(ex->fork, s0));
    for (size_t q = 1; q < ex->streams.size(); ++q) GX_HIP(hipStreamWaitEvent(ex->streams[q], ex->fork, 0));
  }
  for (size_t k = 0; k < ex->nodes.size(); ++k) {
    const ExecNode& nd = ex->nodes[k];
    const hipStream_t st = nd.stream ? ex->streams[nd.stream] : s0;
    for (int w : nd.waits) GX_HIP(hipStreamWaitEvent(st, ex->events[w], 0));
    if (nd.kind == NK_KERNEL) {
      GX_HIP(hipLaunchKernel(nd.kp.func, nd.kp.gridDim, nd.kp.blockDim, nd.kp.kernelParams, nd.kp.sharedMemBytes, st));
    } else if (nd.kind == NK_MEMSET) {
      const int r = issue_memset(nd.mp, st);
      if (r != GMR_OK) return gx_fail(__func__, "memset node failed");
    } else if (nd.kind == NK_MEMCPY) {
      GX_HIP(hipMemcpy3DAsync(&nd.cp, st));
    }
    if (nd.record) GX_HIP(hipEventRecord(ex->events[k], st));
  }
  for (size_t q = 1; q < ex->streams.size(); ++q) {
    GX_HIP(hipEventRecord(ex->joins[q], ex->streams[q]));
    GX_HIP(hipStreamWaitEvent(s0, ex->joins[q], 0));
  }
  return GMR_OK;
}

extern "C" int gmr_graph_exec_destroy(void* exec) {
  delete static_cast<GraphExec*>(exec);
  return GMR_OK;
}
