// graph.hip — the captured training step replayed as main-stream and side-stream graphs, plus the
// host-side event helpers of the eager step's stream plumbing.
//
// The eager step queues ~290 kernels from Python (5.1 of a 5.9 ms C2 step is host enqueue,
// profiles/r4_host_time.txt).  One captured hipGraph removes the host cost, but the HIP runtime
// executes a graph's nodes in one queue, so the weight-gradient branch captured from the side
// stream (2-3.5 ms of GEMMs that overlap the main stream's recurrences in eager mode) runs serially
// with the main chain (7.0 vs 5.8 ms, profiles/r4_graph_queues.txt).
//
// avc_graph_split takes the single graph PyTorch captured (main stream + the side stream forked
// from it, joined at the end) and rebuilds it:
//   * main nodes = every ancestor of the main stream's capture tail at the join (the main chain
//     never waits for the side stream before the join; a side -> main edge is refused);
//   * post nodes = the main-stream nodes captured after the join (the optimizer step): one more
//     graph, launched on the main stream after it has waited for the side stream;
//   * side nodes = ancestors of the side stream's tail that are not main nodes;
//   * "sources" = the main nodes a side node waits for directly.
// mode 0 (default): the main chain cut into <= max_segments graphs after sources (spread evenly),
//   side segment k = the side nodes whose latest main ancestor lies in main segment k; a replay
//   launches main segment k, records an event, makes the side stream wait for it and launches side
//   segment k.  Each boundary costs 15-100 us of main-stream idle time (C2: 6.1-6.2 ms against 5.8
//   eager, profiles/r5_graph_modes.txt).
// mode 1: ONE main graph with an event-record node after every source; each side segment is
//   launched behind a host-side wait for its source's event.  Correct, but the record nodes complete
//   only near the end of the main graph, so the side branch runs after it (6.14 ms).
// Measured and removed (profiles/r5_graph_modes.txt): ordering the side graph on the device -- tiny
// signal kernels on the main chain with polling wait kernels, or hipStreamWaitValue32, on the side
// -- deadlocks against the decoder's full-chip persistent recurrences (one 8-wave, 250-VGPR
// workgroup per CU: a waiting wave on any CU keeps one of them from starting).
//
// Nodes are re-created from their parameters into fresh graphs (never cloned-and-pruned:
// destroying the unwanted nodes of a hipGraphClone left the surviving graphs reading stale kernel
// arguments, round 3).  Memset nodes are rebuilt as zeroing KERNEL nodes: a captured memset node
// that replays after other work on the stream was not reliably complete before the next kernel
// node (round 4, tools/graph_fwd_probe.py; the cause of round 3's NaN from the second replay).
#include <algorithm>
#include <cstdlib>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "common.h"

// cross-stream events of one device: no system-scope fence on record / wait (the default flushes and
// invalidates the L2s for host visibility; the consumers here are kernels on the same GPU, for which
// the device-scope release is enough).  AVC_EV_SYSFENCE=1 restores the default (A/B).
static unsigned ev_flags() {
  static const unsigned f = (getenv("AVC_EV_SYSFENCE") && getenv("AVC_EV_SYSFENCE")[0] == '1')
                                ? hipEventDisableTiming
                                : hipEventDisableTiming | hipEventDisableSystemFence;
  return f;
}
#define kEvFlags ev_flags()

#define GCHK(x, what)                                                    \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      avc_set_error("%s: %s (%s)", what, hipGetErrorString(e_), #x);      \
      return -1;                                                         \
    }                                                                    \
  } while (0)

namespace {

// a memset node of a capture rebuilt as a kernel: words of 4 bytes (value replicated), or bytes
__global__ void graph_fill_words_kernel(unsigned* p, long long n, unsigned v) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}
__global__ void graph_fill_bytes_kernel(unsigned char* p, long long n, unsigned char v) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}

struct Split {
  std::vector<hipGraph_t> gm, gs;
  std::vector<hipGraphExec_t> em, es;  // es[k] null when segment k has no side nodes
  std::vector<hipEvent_t> ev;
  hipEvent_t join = nullptr;
  hipGraph_t gp = nullptr;  // the main-stream nodes after the join (optimizer step), if any
  hipGraphExec_t ep = nullptr;
  int mode = 0;
  std::vector<int> wait_src;       // mode 1: the source side segment k waits for (-1: none)
  std::vector<hipEvent_t> src_ev;  // mode 1: one event per source, recorded by a node of the main graph
  // census: main nodes before the join, side nodes, main -> side edges, segments, kernel nodes,
  // memset nodes (rebuilt as kernels), memcpy nodes, empty nodes, main nodes after the join,
  // event-record nodes (mode 1)
  int counts[AVC_GRAPH_COUNTS] = {};
};

int preds(hipGraphNode_t n, std::vector<hipGraphNode_t>& out) {
  size_t k = 0;
  GCHK(hipGraphNodeGetDependencies(n, nullptr, &k), "avc_graph_split");
  out.resize(k);
  if (k) GCHK(hipGraphNodeGetDependencies(n, out.data(), &k), "avc_graph_split");
  return 0;
}

int ancestors(hipGraphNode_t const* tails, int n, std::unordered_set<hipGraphNode_t>& seen) {
  std::vector<hipGraphNode_t> stack(tails, tails + n), p;
  while (!stack.empty()) {
    hipGraphNode_t x = stack.back();
    stack.pop_back();
    if (!seen.insert(x).second) continue;
    if (preds(x, p)) return -1;
    stack.insert(stack.end(), p.begin(), p.end());
  }
  return 0;
}

void destroy(Split* s) {
  if (!s) return;
  for (auto e : s->em) if (e) (void)hipGraphExecDestroy(e);
  for (auto e : s->es) if (e) (void)hipGraphExecDestroy(e);
  for (auto g : s->gm) if (g) (void)hipGraphDestroy(g);
  for (auto g : s->gs) if (g) (void)hipGraphDestroy(g);
  for (hipEvent_t e : s->ev) if (e) (void)hipEventDestroy(e);
  if (s->join) (void)hipEventDestroy(s->join);
  if (s->ep) (void)hipGraphExecDestroy(s->ep);
  if (s->gp) (void)hipGraphDestroy(s->gp);
  for (hipEvent_t e : s->src_ev) if (e) (void)hipEventDestroy(e);
  delete s;
}

int fill_node(hipGraph_t dst, const hipMemsetParams& p, const hipGraphNode_t* d, size_t nd, hipGraphNode_t* out) {
  AVC_CHECK_ARG(p.height <= 1 && (p.elementSize == 1 || p.elementSize == 4),
                "avc_graph_split: memset node %zu x %zu, element %u bytes is not rebuilt as a kernel", p.width,
                p.height, p.elementSize);
  hipKernelNodeParams k = {};
  long long n = (long long)p.width;
  void* ptr = p.dst;
  unsigned char vb = (unsigned char)p.value;
  unsigned vw = p.value;
  void* args_w[3] = {&ptr, &n, &vw};
  void* args_b[3] = {&ptr, &n, &vb};
  k.blockDim = dim3(256);
  k.gridDim = dim3((unsigned)std::max<long long>(1, std::min<long long>(1024, (n + 255) / 256)));
  k.sharedMemBytes = 0;
  if (p.elementSize == 4) {
    k.func = reinterpret_cast<void*>(&graph_fill_words_kernel);
    k.kernelParams = args_w;
  } else {
    k.func = reinterpret_cast<void*>(&graph_fill_bytes_kernel);
    k.kernelParams = args_b;
  }
  GCHK(hipGraphAddKernelNode(out, dst, d, nd, &k), "avc_graph_split (memset as kernel)");
  return 0;
}

// Copy of one node into dst (kernel, memset -> kernel, memcpy and empty nodes: what a stream
// capture of the step produces).
int copy_node(hipGraph_t dst, hipGraphNode_t src, const std::vector<hipGraphNode_t>& deps, hipGraphNode_t* out) {
  hipGraphNodeType t;
  GCHK(hipGraphNodeGetType(src, &t), "avc_graph_split");
  const hipGraphNode_t* d = deps.empty() ? nullptr : deps.data();
  switch (t) {
    case hipGraphNodeTypeKernel: {
      hipKernelNodeParams p;
      GCHK(hipGraphKernelNodeGetParams(src, &p), "avc_graph_split");
      GCHK(hipGraphAddKernelNode(out, dst, d, deps.size(), &p), "avc_graph_split");
      return 0;
    }
    case hipGraphNodeTypeMemset: {
      hipMemsetParams p;
      GCHK(hipGraphMemsetNodeGetParams(src, &p), "avc_graph_split");
      return fill_node(dst, p, d, deps.size(), out);
    }
    case hipGraphNodeTypeMemcpy: {
      hipMemcpy3DParms p;
      GCHK(hipGraphMemcpyNodeGetParams(src, &p), "avc_graph_split");
      GCHK(hipGraphAddMemcpyNode(out, dst, d, deps.size(), &p), "avc_graph_split");
      return 0;
    }
    case hipGraphNodeTypeEmpty:
      GCHK(hipGraphAddEmptyNode(out, dst, d, deps.size()), "avc_graph_split");
      return 0;
    default:
      avc_set_error("avc_graph_split: node type %d is not supported", (int)t);
      return -1;
  }
}

// New graph holding copies of the nodes with keep[i] (in topological order `order`, with the edges
// among them), instantiated.
int sub_graph(const std::vector<hipGraphNode_t>& nodes, const std::vector<int>& order,
              const std::vector<std::vector<int>>& pr, const std::vector<char>& keep, hipGraph_t* out,
              hipGraphExec_t* exec) {
  GCHK(hipGraphCreate(out, 0), "avc_graph_split");
  std::vector<hipGraphNode_t> made(nodes.size(), nullptr), deps;
  for (int i : order) {
    if (!keep[i]) continue;
    deps.clear();
    for (int j : pr[i])
      if (keep[j]) deps.push_back(made[j]);
    if (copy_node(*out, nodes[i], deps, &made[i])) return -1;
  }
  GCHK(hipGraphInstantiate(exec, *out, nullptr, nullptr, 0), "avc_graph_split");
  return 0;
}

// ONE graph of every main node (s->gm[0] / em[0]) with an event record node after every source (on the
// chain: the source's successors depend on it); flag_of[main node] = its source index
int main_record_graph(const std::vector<hipGraphNode_t>& nodes, const std::vector<int>& order,
                      const std::vector<std::vector<int>>& pr, const std::vector<int>& pos,
                      const std::vector<int>& flag_of, Split* s) {
  std::vector<hipGraphNode_t> made(nodes.size(), nullptr), deps;
  GCHK(hipGraphCreate(&s->gm[0], 0), "avc_graph_split");
  for (int i : order) {
    if (pos[i] < 0) continue;
    deps.clear();
    for (int j : pr[i]) deps.push_back(made[j]);
    if (copy_node(s->gm[0], nodes[i], deps, &made[i])) return -1;
    if (flag_of[i] >= 0) {
      hipGraphNode_t ev;
      GCHK(hipGraphAddEventRecordNode(&ev, s->gm[0], &made[i], 1, s->src_ev[flag_of[i]]), "avc_graph_split");
      made[i] = ev;
      ++s->counts[9];
    }
  }
  GCHK(hipGraphInstantiate(&s->em[0], s->gm[0], nullptr, nullptr, 0), "avc_graph_split");
  return 0;
}

int build(hipGraph_t g, hipGraphNode_t const* main_tails, int n_main, hipGraphNode_t const* side_tails, int n_side,
          int max_seg, int mode, Split* s) {
  size_t nn = 0;
  GCHK(hipGraphGetNodes(g, nullptr, &nn), "avc_graph_split");
  std::vector<hipGraphNode_t> nodes(nn);
  if (nn) GCHK(hipGraphGetNodes(g, nodes.data(), &nn), "avc_graph_split");
  std::unordered_map<hipGraphNode_t, int> idx;
  for (size_t i = 0; i < nn; ++i) {
    idx[nodes[i]] = (int)i;
    hipGraphNodeType t;
    GCHK(hipGraphNodeGetType(nodes[i], &t), "avc_graph_split");
    if (t == hipGraphNodeTypeKernel) ++s->counts[4];
    else if (t == hipGraphNodeTypeMemset) ++s->counts[5];
    else if (t == hipGraphNodeTypeMemcpy) ++s->counts[6];
    else if (t == hipGraphNodeTypeEmpty) ++s->counts[7];
  }
  // main = ancestors of the main tail at the join; side = ancestors of the side tail that are not
  // main; post = the rest: main-stream nodes captured after the join (the optimizer step)
  std::unordered_set<hipGraphNode_t> mainset, sideset;
  if (ancestors(main_tails, n_main, mainset) || ancestors(side_tails, n_side, sideset)) return -1;
  for (hipGraphNode_t x : mainset) sideset.erase(x);
  AVC_CHECK_ARG(!sideset.empty(), "avc_graph_split: no side-stream nodes");
  std::vector<char> post(nn, 0);
  int npost = 0;
  for (size_t i = 0; i < nn; ++i)
    if (!mainset.count(nodes[i]) && !sideset.count(nodes[i])) post[i] = 1, ++npost;
  // predecessor lists; topological order (Kahn, lowest creation index first: the capture order)
  std::vector<std::vector<int>> pr(nn), succ(nn);
  std::vector<int> indeg(nn, 0);
  std::vector<hipGraphNode_t> p;
  for (size_t i = 0; i < nn; ++i) {
    if (preds(nodes[i], p)) return -1;
    const bool im = mainset.count(nodes[i]) != 0;
    for (hipGraphNode_t y : p) {
      const int j = idx.at(y);
      AVC_CHECK_ARG(!(im && !mainset.count(y)),
                    "avc_graph_split: a main-stream node waits for a side-stream node before the join");
      AVC_CHECK_ARG(post[i] || !post[j], "avc_graph_split: a node before the join waits for a node after it");
      pr[i].push_back(j);
      succ[j].push_back((int)i);
      ++indeg[i];
    }
  }
  std::vector<int> order, heap;
  auto cmp = [](int a, int b) { return a > b; };
  for (size_t i = 0; i < nn; ++i)
    if (!indeg[i]) heap.push_back((int)i);
  std::make_heap(heap.begin(), heap.end(), cmp);
  while (!heap.empty()) {
    std::pop_heap(heap.begin(), heap.end(), cmp);
    const int x = heap.back();
    heap.pop_back();
    order.push_back(x);
    for (int y : succ[x])
      if (!--indeg[y]) {
        heap.push_back(y);
        std::push_heap(heap.begin(), heap.end(), cmp);
      }
  }
  AVC_CHECK_ARG(order.size() == nn, "avc_graph_split: the graph has a cycle");
  // main positions in topological order; need[s] = latest main position a side node depends on
  std::vector<int> pos(nn, -1), need(nn, -1);
  int nm = 0;
  for (int x : order)
    if (mainset.count(nodes[x])) pos[x] = nm++;
  std::vector<int> sources;  // main positions some side node waits for directly
  for (int x : order) {
    if (pos[x] >= 0 || post[x]) continue;
    for (int j : pr[x]) {
      if (pos[j] >= 0) {
        need[x] = std::max(need[x], pos[j]);
        sources.push_back(pos[j]);
        ++s->counts[2];
      } else {
        need[x] = std::max(need[x], need[j]);
      }
    }
  }
  std::sort(sources.begin(), sources.end());
  sources.erase(std::unique(sources.begin(), sources.end()), sources.end());
  s->counts[0] = (int)mainset.size();
  s->counts[1] = (int)sideset.size();
  s->counts[8] = npost;
  // cuts: after every source (at most max_seg - 1 of them, spread evenly; mode 1: all of them); the
  // last segment ends the graph
  std::vector<int> cuts;
  const int ns = (int)sources.size(), K = mode == 1 ? ns : std::min(max_seg - 1, ns);
  for (int k = 1; k <= K; ++k) cuts.push_back(sources[(long long)k * ns / K - 1]);
  cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
  if (cuts.empty() || cuts.back() != nm - 1) cuts.push_back(nm - 1);
  const int S = (int)cuts.size();
  auto seg_of = [&](int mp) { return (int)(std::lower_bound(cuts.begin(), cuts.end(), mp) - cuts.begin()); };
  const int SM = mode == 1 ? 1 : S;  // mode 1: ONE main graph, S side segments
  s->gm.assign(SM, nullptr);
  s->em.assign(SM, nullptr);
  s->gs.assign(S, nullptr);
  s->es.assign(S, nullptr);
  s->ev.assign(S, nullptr);
  if (mode == 1) {
    std::vector<int> src_of(nn, -1);  // main node -> its source index
    for (size_t i = 0; i < nn; ++i)
      if (pos[i] >= 0) {
        auto it = std::lower_bound(sources.begin(), sources.end(), pos[i]);
        if (it != sources.end() && *it == pos[i]) src_of[i] = (int)(it - sources.begin());
      }
    s->src_ev.assign(sources.size(), nullptr);
    for (auto& e : s->src_ev) GCHK(hipEventCreateWithFlags(&e, kEvFlags), "avc_graph_split");
    if (main_record_graph(nodes, order, pr, pos, src_of, s)) return -1;
    s->wait_src.assign(S, -1);
    for (int k = 0; k < S; ++k) {
      auto it = std::lower_bound(sources.begin(), sources.end(), cuts[k]);
      if (it != sources.end() && *it == cuts[k]) s->wait_src[k] = (int)(it - sources.begin());
    }
  }
  for (int k = 0; k < S; ++k) {
    std::vector<char> km(nn, 0), ks(nn, 0);
    bool any_side = false;
    for (size_t i = 0; i < nn; ++i) {
      if (post[i]) continue;
      if (pos[i] >= 0) km[i] = seg_of(pos[i]) == k;
      else if (seg_of(std::max(need[i], 0)) == k) ks[i] = any_side = true;
    }
    if (mode == 0 && sub_graph(nodes, order, pr, km, &s->gm[k], &s->em[k])) return -1;
    if (any_side) {
      if (sub_graph(nodes, order, pr, ks, &s->gs[k], &s->es[k])) return -1;
      GCHK(hipEventCreateWithFlags(&s->ev[k], kEvFlags), "avc_graph_split");
    }
  }
  if (npost && sub_graph(nodes, order, pr, post, &s->gp, &s->ep)) return -1;
  GCHK(hipEventCreateWithFlags(&s->join, kEvFlags), "avc_graph_split");
  s->counts[3] = S;
  return 0;
}

}  // namespace

extern "C" int avc_capture_deps(void* stream, void** out, int max_out) {
  AVC_CHECK_ARG(out && max_out > 0, "avc_capture_deps: bad args");
  hipStreamCaptureStatus st;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  GCHK(hipStreamGetCaptureInfo_v2(as_stream(stream), &st, &id, &g, &deps, &nd), "avc_capture_deps");
  AVC_CHECK_ARG(st == hipStreamCaptureStatusActive, "avc_capture_deps: the stream is not capturing");
  AVC_CHECK_ARG((int)nd <= max_out, "avc_capture_deps: %zu dependencies > %d", nd, max_out);
  for (size_t i = 0; i < nd; ++i) out[i] = deps[i];
  return (int)nd;
}

extern "C" int avc_graph_split(void* graph, void* const* main_tails, int n_main, void* const* side_tails, int n_side,
                               int max_segments, int mode, void** handle, int* counts) {
  AVC_CHECK_ARG(graph && main_tails && side_tails && n_main > 0 && n_side > 0 && handle && max_segments >= 1 &&
                    (mode == 0 || mode == 1),
                "avc_graph_split: bad args");
  Split* s = new Split;
  s->mode = mode;
  if (build(reinterpret_cast<hipGraph_t>(graph), reinterpret_cast<hipGraphNode_t const*>(main_tails), n_main,
            reinterpret_cast<hipGraphNode_t const*>(side_tails), n_side, max_segments, mode, s)) {
    destroy(s);
    return -1;
  }
  if (counts)
    for (int i = 0; i < AVC_GRAPH_COUNTS; ++i) counts[i] = s->counts[i];
  *handle = s;
  return 0;
}

extern "C" int avc_graph_launch2(void* handle, void* main_stream, void* side_stream) {
  Split* s = reinterpret_cast<Split*>(handle);
  AVC_CHECK_ARG(s, "avc_graph_launch2: null handle");
  hipStream_t m = as_stream(main_stream), sd = as_stream(side_stream);
  // the side stream starts after everything queued on the main stream before the replay
  GCHK(hipEventRecord(s->join, m), "avc_graph_launch2");
  GCHK(hipStreamWaitEvent(sd, s->join, 0), "avc_graph_launch2");
  if (s->mode == 1) {
    GCHK(hipGraphLaunch(s->em[0], m), "avc_graph_launch2");
    for (size_t k = 0; k < s->es.size(); ++k) {
      if (!s->es[k]) continue;
      if (s->wait_src[k] >= 0) GCHK(hipStreamWaitEvent(sd, s->src_ev[s->wait_src[k]], 0), "avc_graph_launch2");
      GCHK(hipGraphLaunch(s->es[k], sd), "avc_graph_launch2");
    }
  } else {
    for (size_t k = 0; k < s->em.size(); ++k) {
      GCHK(hipGraphLaunch(s->em[k], m), "avc_graph_launch2");
      if (s->es[k]) {
        GCHK(hipEventRecord(s->ev[k], m), "avc_graph_launch2");
        GCHK(hipStreamWaitEvent(sd, s->ev[k], 0), "avc_graph_launch2");
        GCHK(hipGraphLaunch(s->es[k], sd), "avc_graph_launch2");
      }
    }
  }
  GCHK(hipEventRecord(s->join, sd), "avc_graph_launch2");
  GCHK(hipStreamWaitEvent(m, s->join, 0), "avc_graph_launch2");
  if (s->ep) GCHK(hipGraphLaunch(s->ep, m), "avc_graph_launch2");
  return 0;
}

extern "C" int avc_graph_split_destroy(void* handle) {
  destroy(reinterpret_cast<Split*>(handle));
  return 0;
}

// ---------------------------------------------------------------- host-side event helpers
// Cross-stream ordering of the step (weight-gradient side stream, pack prefetch) with raw HIP
// events on raw stream handles: torch.cuda.Event / current_stream() cost ~10-15 us of Python
// per use, ~1 ms per AutoVC step at ~90 uses.  Events are created once (a ring on the Python
// side) and re-recorded; hipStreamWaitEvent waits for the record current at the time of the call.
extern "C" int avc_event_create(void** out) {
  AVC_CHECK_ARG(out, "avc_event_create: null");
  hipEvent_t e = nullptr;
  GCHK(hipEventCreateWithFlags(&e, kEvFlags), "avc_event_create");
  *out = e;
  return 0;
}

extern "C" int avc_event_record(void* ev, void* stream) {
  AVC_CHECK_ARG(ev, "avc_event_record: null event");
  GCHK(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), as_stream(stream)), "avc_event_record");
  return 0;
}

extern "C" int avc_stream_wait_event(void* stream, void* ev) {
  AVC_CHECK_ARG(ev, "avc_stream_wait_event: null event");
  GCHK(hipStreamWaitEvent(as_stream(stream), reinterpret_cast<hipEvent_t>(ev), 0), "avc_stream_wait_event");
  return 0;
}
