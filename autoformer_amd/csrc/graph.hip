// graph.hip — the training step as TWO hipGraphs that run concurrently on the main and the
// weight-gradient streams.
//
// The eager step queues ~290 kernels from Python; on a host whose Python is slow that queueing
// takes longer than the GPU step (profiles/r3_host_time.txt).  One captured hipGraph removes the
// host cost, but the HIP runtime executes a graph's nodes in one queue, so the weight-gradient
// branch captured from the side stream (2.8 ms of GEMMs that overlap the main stream's
// recurrences in eager mode) would run serially after the main chain's nodes (7.0 vs 5.9 ms).
//
// avc_graph_split takes the single graph that PyTorch captured (main stream + the side stream
// forked from it) and rebuilds it as two graphs:
//   * main nodes = every ancestor of the main stream's capture tail at the join (the main
//     chain never waits for the side stream before the join, so none of them is a side node);
//   * side nodes = ancestors of the side stream's tail that are not main nodes;
//   * the main chain is cut into at most max_segments segments after main nodes that side nodes
//     wait for; side segment k holds the side nodes whose latest main dependency lies in main
//     segment k.  A side -> main edge before the join is refused.
// avc_graph_launch2 launches, per segment, the main graph on the main stream, records an event
// there, makes the side stream wait for it and launches the side graph; finally the main stream
// waits for the side stream.
#include <algorithm>
#include <cstdlib>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "common.h"

namespace {

// One replay = segments k = 0 .. K-1: main graph M_k on the main stream, event E_k, the side
// stream waits E_k, side graph S_k on the side stream; then the main stream waits for the side.
// (Event record / wait NODES inside two separately launched graphs do not order them at node
// granularity on ROCm 7: the side graph's waits resolved only when the whole main graph had
// finished, profiles/r3_graph_split.txt -- so the cross edges are cut between launches.)
struct Split {
  std::vector<hipGraph_t> gm, gs;
  std::vector<hipGraphExec_t> em, es;  // es[k] null when segment k has no side nodes
  std::vector<hipEvent_t> ev;
  hipEvent_t join = nullptr;
  int n_main = 0, n_side = 0, n_cross = 0;
};

#define GCHK(x, what)                                                    \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      avc_set_error("%s: %s (%s)", what, hipGetErrorString(e_), #x);      \
      return -1;                                                         \
    }                                                                    \
  } while (0)

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
  for (hipEvent_t e : s->ev) (void)hipEventDestroy(e);
  if (s->join) (void)hipEventDestroy(s->join);
  delete s;
}

// Copy of one node into dst (kernel, memset, memcpy and empty nodes: what a stream capture of the
// step produces).  Nodes are re-created from their parameters, never cloned-and-pruned: destroying
// the unwanted nodes of a hipGraphClone left the surviving graphs reading stale kernel arguments
// on later launches (NaN after the first replay, profiles/r3_graph_split.txt).
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
      GCHK(hipGraphAddMemsetNode(out, dst, d, deps.size(), &p), "avc_graph_split");
      return 0;
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

int build(hipGraph_t g, hipGraphNode_t const* main_tails, int n_main, hipGraphNode_t const* side_tails, int n_side,
          int max_seg, Split* s) {
  size_t nn = 0;
  GCHK(hipGraphGetNodes(g, nullptr, &nn), "avc_graph_split");
  std::vector<hipGraphNode_t> nodes(nn);
  if (nn) GCHK(hipGraphGetNodes(g, nodes.data(), &nn), "avc_graph_split");
  std::unordered_map<hipGraphNode_t, int> idx;
  for (size_t i = 0; i < nn; ++i) idx[nodes[i]] = (int)i;
  std::unordered_set<hipGraphNode_t> mainset, sideset;
  if (ancestors(main_tails, n_main, mainset) || ancestors(side_tails, n_side, sideset)) return -1;
  for (hipGraphNode_t x : mainset) sideset.erase(x);
  AVC_CHECK_ARG(mainset.size() + sideset.size() == nn,
                "avc_graph_split: %zu of %zu nodes are neither main nor side ancestors of the join",
                nn - mainset.size() - sideset.size(), nn);
  AVC_CHECK_ARG(!sideset.empty(), "avc_graph_split: no side-stream nodes");
  // predecessor lists; topological order (Kahn) of the whole graph
  std::vector<std::vector<int>> pr(nn);
  std::vector<int> indeg(nn, 0);
  std::vector<std::vector<int>> succ(nn);
  std::vector<hipGraphNode_t> p;
  for (size_t i = 0; i < nn; ++i) {
    if (preds(nodes[i], p)) return -1;
    const bool im = mainset.count(nodes[i]) != 0;
    for (hipGraphNode_t y : p) {
      const int j = idx.at(y);
      AVC_CHECK_ARG(!(im && !mainset.count(y)),
                    "avc_graph_split: a main-stream node waits for a side-stream node before the join");
      pr[i].push_back(j);
      succ[j].push_back((int)i);
      ++indeg[i];
    }
  }
  std::vector<int> order, q;
  for (size_t i = 0; i < nn; ++i)
    if (!indeg[i]) q.push_back((int)i);
  while (!q.empty()) {
    const int x = q.back();
    q.pop_back();
    order.push_back(x);
    for (int y : succ[x])
      if (!--indeg[y]) q.push_back(y);
  }
  AVC_CHECK_ARG(order.size() == nn, "avc_graph_split: the graph has a cycle");
  // main positions in topological order; need[s] = latest main position a side node depends on
  std::vector<int> pos(nn, -1), need(nn, -1);
  int nm = 0;
  for (int x : order)
    if (mainset.count(nodes[x])) pos[x] = nm++;
  std::vector<int> sources;  // main positions some side node waits for directly
  for (int x : order) {
    if (pos[x] >= 0) continue;
    for (int j : pr[x]) {
      if (pos[j] >= 0) {
        need[x] = std::max(need[x], pos[j]);
        sources.push_back(pos[j]);
        ++s->n_cross;
      } else {
        need[x] = std::max(need[x], need[j]);
      }
    }
  }
  std::sort(sources.begin(), sources.end());
  sources.erase(std::unique(sources.begin(), sources.end()), sources.end());
  // cuts: after at most max_seg - 1 of the sources, spread evenly; the last segment ends the graph
  std::vector<int> cuts;
  const int ns = (int)sources.size(), K = std::min(max_seg - 1, ns);
  for (int k = 1; k <= K; ++k) cuts.push_back(sources[(long long)k * ns / K - 1]);
  cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
  if (cuts.empty() || cuts.back() != nm - 1) cuts.push_back(nm - 1);
  int S = (int)cuts.size();
  // debug (AVC_GRAPH_RUNS=1): segments = the runs of main / side nodes in creation order
  static const bool runs = getenv("AVC_GRAPH_RUNS") && getenv("AVC_GRAPH_RUNS")[0] == '1';
  std::vector<int> run_of(nn, 0);
  if (runs) {
    int r = 0;
    bool prev_main = true;
    for (size_t i = 0; i < nn; ++i) {
      const bool im = pos[i] >= 0;
      if (im && !prev_main) ++r;  // a main run after a side run opens segment r + 1
      run_of[i] = r;
      prev_main = im;
    }
    S = r + 1;
  }
  // debug: AVC_GRAPH_CLONE_ONLY=1 one copy of the whole graph as "main segment 0", no side graphs;
  // =2 the same single graph with every main node created before every side node
  static const int whole = getenv("AVC_GRAPH_CLONE_ONLY") ? atoi(getenv("AVC_GRAPH_CLONE_ONLY")) : 0;
  if (whole == 2) {
    std::vector<int> mfirst;
    for (int x : order)
      if (pos[x] >= 0) mfirst.push_back(x);
    for (int x : order)
      if (pos[x] < 0) mfirst.push_back(x);
    order.swap(mfirst);
  }
  if (whole) {
    s->gm.assign(1, nullptr);
    s->gs.assign(1, nullptr);
    s->em.assign(1, nullptr);
    s->es.assign(1, nullptr);
    s->ev.assign(1, nullptr);
    std::vector<char> all(nn, 1);
    if (sub_graph(nodes, order, pr, all, &s->gm[0], &s->em[0])) return -1;
    GCHK(hipEventCreateWithFlags(&s->ev[0], hipEventDisableTiming), "avc_graph_split");
    GCHK(hipEventCreateWithFlags(&s->join, hipEventDisableTiming), "avc_graph_split");
    return 0;
  }
  auto seg_of = [&](int mp) { return (int)(std::lower_bound(cuts.begin(), cuts.end(), mp) - cuts.begin()); };
  s->gm.assign(S, nullptr);
  s->gs.assign(S, nullptr);
  s->em.assign(S, nullptr);
  s->es.assign(S, nullptr);
  s->ev.assign(S, nullptr);
  for (int k = 0; k < S; ++k) {
    std::vector<char> km(nn, 0), ks(nn, 0);
    bool any_side = false;
    for (size_t i = 0; i < nn; ++i) {
      if (runs) {
        if (run_of[i] != k) continue;
        if (pos[i] >= 0) km[i] = 1;
        else ks[i] = any_side = true;
        continue;
      }
      if (pos[i] >= 0) km[i] = seg_of(pos[i]) == k;
      else if (seg_of(std::max(need[i], 0)) == k) ks[i] = any_side = true;
    }
    if (sub_graph(nodes, order, pr, km, &s->gm[k], &s->em[k])) return -1;
    if (any_side && sub_graph(nodes, order, pr, ks, &s->gs[k], &s->es[k])) return -1;
    GCHK(hipEventCreateWithFlags(&s->ev[k], hipEventDisableTiming), "avc_graph_split");
  }
  GCHK(hipEventCreateWithFlags(&s->join, hipEventDisableTiming), "avc_graph_split");
  s->n_main = (int)mainset.size();
  s->n_side = (int)sideset.size();
  return 0;
}

}  // namespace

extern "C" int avc_capture_deps(void* stream, void** out, int max_out) {
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
                               int max_segments, void** handle, int* counts) {
  AVC_CHECK_ARG(graph && main_tails && side_tails && n_main > 0 && n_side > 0 && handle && max_segments >= 1,
                "avc_graph_split: bad args");
  Split* s = new Split;
  if (build(reinterpret_cast<hipGraph_t>(graph), reinterpret_cast<hipGraphNode_t const*>(main_tails), n_main,
            reinterpret_cast<hipGraphNode_t const*>(side_tails), n_side, max_segments, s)) {
    destroy(s);
    return -1;
  }
  if (counts) {
    counts[0] = s->n_main;
    counts[1] = s->n_side;
    counts[2] = s->n_cross;
    counts[3] = (int)s->em.size();
  }
  *handle = s;
  return 0;
}

extern "C" int avc_graph_launch2(void* handle, void* main_stream, void* side_stream) {
  Split* s = reinterpret_cast<Split*>(handle);
  AVC_CHECK_ARG(s, "avc_graph_launch2: null handle");
  hipStream_t m = as_stream(main_stream), sd = as_stream(side_stream);
  static const bool serial = getenv("AVC_GRAPH_SERIAL") && getenv("AVC_GRAPH_SERIAL")[0] == '1';  // debug
  if (serial) sd = m;
  static const bool skip_side = getenv("AVC_GRAPH_SKIP_SIDE") && getenv("AVC_GRAPH_SKIP_SIDE")[0] == '1';  // debug
  for (size_t k = 0; k < s->em.size(); ++k) {
    GCHK(hipGraphLaunch(s->em[k], m), "avc_graph_launch2");
    if (s->es[k] && !skip_side) {
      GCHK(hipEventRecord(s->ev[k], m), "avc_graph_launch2");
      GCHK(hipStreamWaitEvent(sd, s->ev[k], 0), "avc_graph_launch2");
      GCHK(hipGraphLaunch(s->es[k], sd), "avc_graph_launch2");
    }
  }
  GCHK(hipEventRecord(s->join, sd), "avc_graph_launch2");
  GCHK(hipStreamWaitEvent(m, s->join, 0), "avc_graph_launch2");
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
  GCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming), "avc_event_create");
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
