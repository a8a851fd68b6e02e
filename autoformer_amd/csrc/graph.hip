// graph.hip — the captured training step replayed as main-stream and side-stream graph segments,
// plus the host-side event helpers of the eager step's stream plumbing.
//
// The eager step queues ~290 kernels from Python (5.1 of a 5.9 ms C2 step is host enqueue,
// profiles/r4_host_time.txt).  One captured hipGraph removes the host cost, but the HIP runtime
// executes a graph's nodes in one queue, so the weight-gradient branch captured from the side
// stream (3.5 ms of GEMMs that overlap the main stream's recurrences in eager mode) runs serially
// with the main chain (7.0 vs 5.8 ms, profiles/r4_graph_queues.txt).  Event record / wait NODES
// inside two separately launched graphs do not order them at node granularity on ROCm 7 (the
// side graph's waits resolved only when the whole main graph had finished, round 3), so the
// cross-stream edges are cut BETWEEN launches:
//
// avc_graph_split takes the single graph PyTorch captured (main stream + the side stream forked
// from it, joined at the end) and rebuilds it as segments:
//   * main nodes = every ancestor of the main stream's capture tail at the join (the main chain
//     never waits for the side stream before the join; a side -> main edge is refused);
//   * post nodes = the main-stream nodes captured after the join (the optimizer step): one more
//     graph, launched on the main stream after it has waited for the side stream;
//   * side nodes = ancestors of the side stream's tail that are not main nodes;
//   * the main chain is cut after every main node a side node waits for ("source"; at most
//     max_segments segments, cuts spread evenly over the sources beyond that); side segment k
//     holds the side nodes whose latest main ancestor lies in main segment k.
// avc_graph_launch2 launches, per segment, main graph k on the main stream, records event k there,
// makes the side stream wait for it and launches side graph k; the main stream finally waits for
// the side stream.  That is mode 0; each boundary cost 15-100 us of main-stream idle time (22
// boundaries: a C2 replay at 6.2 ms against 5.8 eager).  Mode 1 (the default) keeps ONE main graph
// and ONE side graph and orders them on the device instead: a tiny signal kernel after every
// source on the main chain publishes the replay number, a tiny wait kernel on the side chain polls
// for it (build_flags below).
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

// Device-flag form (mode 1): the main chain is ONE graph that publishes its progress, the side
// branch ONE graph that waits for it on the device.  sync[0] / sync[1] = replay counters of the main
// / side graph (each graph's first node increments its own, so they agree within a replay: the main
// stream waits for the side at the end of every replay); sync[2 + f] = the main counter as of the
// last time source f completed.  Every sync word is read and written agent-coherently (sc1: the
// per-XCD L2s are not coherent with each other); a kernel boundary on the producing queue has
// already made the source's outputs visible (end-of-kernel release) before its signal runs.
__device__ __forceinline__ unsigned ld_u32_sc1(const unsigned* p) {
  return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u32_sc1(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void graph_epoch_kernel(unsigned* ctr) {
  if (threadIdx.x == 0) st_u32_sc1(ctr, ld_u32_sc1(ctr) + 1u);
}
__global__ void graph_signal_kernel(const unsigned* main_ctr, unsigned* flag) {
  if (threadIdx.x == 0) st_u32_sc1(flag, ld_u32_sc1(main_ctr));
}
// spins (s_sleep between polls) until the source's flag reaches this replay; bounded: after ~2 s of
// the 100 MHz REALTIME clock it raises fault bit 1 (value 2) and lets the side branch run on, so a
// stalled main chain shows at the next fault check instead of hanging the queue
__global__ void graph_wait_kernel(const unsigned* side_ctr, const unsigned* flag, unsigned* fault) {
  if (threadIdx.x != 0) return;
  const unsigned want = ld_u32_sc1(side_ctr);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_u32_sc1(flag) != want) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
      if (fault) atomicOr(fault, 2u);
      break;
    }
  }
}

struct Split {
  std::vector<hipGraph_t> gm, gs;
  std::vector<hipGraphExec_t> em, es;  // es[k] null when segment k has no side nodes
  std::vector<hipEvent_t> ev;
  hipEvent_t join = nullptr;
  hipGraph_t gp = nullptr;  // the main-stream nodes after the join (optimizer step), if any
  hipGraphExec_t ep = nullptr;
  unsigned* sync = nullptr;  // mode 1: replay counters + source flags (device)
  // census: main nodes before the join, side nodes, main -> side edges, segments, kernel nodes,
  // memset nodes (rebuilt as kernels), memcpy nodes, empty nodes, main nodes after the join,
  // wait nodes and signal nodes (mode 1)
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
  if (s->sync) (void)hipFree(s->sync);
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

int tiny_node(hipGraph_t dst, void* fn, void** args, const std::vector<hipGraphNode_t>& deps, hipGraphNode_t* out) {
  hipKernelNodeParams k = {};
  k.blockDim = dim3(64);
  k.gridDim = dim3(1);
  k.func = fn;
  k.kernelParams = args;
  GCHK(hipGraphAddKernelNode(out, dst, deps.empty() ? nullptr : deps.data(), deps.size(), &k), "avc_graph_split");
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

// Mode 1: one main graph (a replay-counter node first, a signal node after every source on the
// chain) and one side graph (its counter node first, a wait node before the first side node that
// needs each source).  pos / need / sources as in build(); side nodes are a chain (one captured
// stream), so a wait for the latest source a node needs covers every earlier one.
int build_flags(const std::vector<hipGraphNode_t>& nodes, const std::vector<int>& order,
                const std::vector<std::vector<int>>& pr, const std::vector<int>& pos, const std::vector<char>& post,
                const std::vector<int>& sources, unsigned* fault, Split* s) {
  const size_t nn = nodes.size();
  const int ns = (int)sources.size();
  GCHK(hipMalloc(&s->sync, sizeof(unsigned) * (2 + ns)), "avc_graph_split");
  GCHK(hipMemset(s->sync, 0, sizeof(unsigned) * (2 + ns)), "avc_graph_split");
  GCHK(hipDeviceSynchronize(), "avc_graph_split");
  unsigned* main_ctr = s->sync;
  unsigned* side_ctr = s->sync + 1;
  std::vector<int> flag_of(nn, -1);  // main node -> its source flag
  for (size_t i = 0; i < nn; ++i)
    if (pos[i] >= 0) {
      auto it = std::lower_bound(sources.begin(), sources.end(), pos[i]);
      if (it != sources.end() && *it == pos[i]) flag_of[i] = (int)(it - sources.begin());
    }
  s->gm.assign(1, nullptr);
  s->gs.assign(1, nullptr);
  s->em.assign(1, nullptr);
  s->es.assign(1, nullptr);
  s->ev.assign(1, nullptr);
  std::vector<hipGraphNode_t> made(nn, nullptr), deps;
  // main graph
  GCHK(hipGraphCreate(&s->gm[0], 0), "avc_graph_split");
  hipGraphNode_t mroot;
  {
    void* a[1] = {&main_ctr};
    if (tiny_node(s->gm[0], reinterpret_cast<void*>(&graph_epoch_kernel), a, {}, &mroot)) return -1;
  }
  for (int i : order) {
    if (pos[i] < 0) continue;
    deps.clear();
    for (int j : pr[i]) deps.push_back(made[j]);
    if (deps.empty()) deps.push_back(mroot);
    if (copy_node(s->gm[0], nodes[i], deps, &made[i])) return -1;
    if (flag_of[i] >= 0) {
      // the chain continues through the signal: successors of the source depend on it
      unsigned* flag = s->sync + 2 + flag_of[i];
      void* a[2] = {&main_ctr, &flag};
      hipGraphNode_t sig;
      if (tiny_node(s->gm[0], reinterpret_cast<void*>(&graph_signal_kernel), a, {made[i]}, &sig)) return -1;
      made[i] = sig;
      ++s->counts[10];
    }
  }
  GCHK(hipGraphInstantiate(&s->em[0], s->gm[0], nullptr, nullptr, 0), "avc_graph_split");
  // side graph
  GCHK(hipGraphCreate(&s->gs[0], 0), "avc_graph_split");
  hipGraphNode_t sroot;
  {
    void* a[1] = {&side_ctr};
    if (tiny_node(s->gs[0], reinterpret_cast<void*>(&graph_epoch_kernel), a, {}, &sroot)) return -1;
  }
  std::vector<hipGraphNode_t> wait_node(ns, nullptr);
  int waited = -1;  // the latest source waited for so far
  hipGraphNode_t last_wait = nullptr;
  for (int i : order) {
    if (pos[i] >= 0 || post[i]) continue;
    deps.clear();
    int f = -1;
    for (int j : pr[i]) {
      if (pos[j] >= 0) f = std::max(f, flag_of[j]);
      else deps.push_back(made[j]);
    }
    if (f > waited) {
      std::vector<hipGraphNode_t> wd = deps;
      if (wd.empty()) wd.push_back(last_wait ? last_wait : sroot);
      const unsigned* flag = s->sync + 2 + f;
      void* a[3] = {&side_ctr, &flag, &fault};
      if (tiny_node(s->gs[0], reinterpret_cast<void*>(&graph_wait_kernel), a, wd, &wait_node[f])) return -1;
      last_wait = wait_node[f];
      waited = f;
      ++s->counts[9];
    }
    if (f >= 0 || deps.empty()) deps.push_back(last_wait ? last_wait : sroot);
    if (copy_node(s->gs[0], nodes[i], deps, &made[i])) return -1;
  }
  GCHK(hipGraphInstantiate(&s->es[0], s->gs[0], nullptr, nullptr, 0), "avc_graph_split");
  s->counts[3] = 1;
  return 0;
}

int build(hipGraph_t g, hipGraphNode_t const* main_tails, int n_main, hipGraphNode_t const* side_tails, int n_side,
          int max_seg, int mode, unsigned* fault, Split* s) {
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
  if (mode == 1) {
    if (build_flags(nodes, order, pr, pos, post, sources, fault, s)) return -1;
    if (npost && sub_graph(nodes, order, pr, post, &s->gp, &s->ep)) return -1;
    GCHK(hipEventCreateWithFlags(&s->join, hipEventDisableTiming), "avc_graph_split");
    return 0;
  }
  // cuts: after every source (at most max_seg - 1 of them, spread evenly); the last segment ends the graph
  std::vector<int> cuts;
  const int ns = (int)sources.size(), K = std::min(max_seg - 1, ns);
  for (int k = 1; k <= K; ++k) cuts.push_back(sources[(long long)k * ns / K - 1]);
  cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
  if (cuts.empty() || cuts.back() != nm - 1) cuts.push_back(nm - 1);
  const int S = (int)cuts.size();
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
      if (post[i]) continue;
      if (pos[i] >= 0) km[i] = seg_of(pos[i]) == k;
      else if (seg_of(std::max(need[i], 0)) == k) ks[i] = any_side = true;
    }
    if (sub_graph(nodes, order, pr, km, &s->gm[k], &s->em[k])) return -1;
    if (any_side) {
      if (sub_graph(nodes, order, pr, ks, &s->gs[k], &s->es[k])) return -1;
      GCHK(hipEventCreateWithFlags(&s->ev[k], hipEventDisableTiming), "avc_graph_split");
    }
  }
  if (npost && sub_graph(nodes, order, pr, post, &s->gp, &s->ep)) return -1;
  GCHK(hipEventCreateWithFlags(&s->join, hipEventDisableTiming), "avc_graph_split");
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
                               int max_segments, int mode, void* fault_word, void** handle, int* counts) {
  AVC_CHECK_ARG(graph && main_tails && side_tails && n_main > 0 && n_side > 0 && handle && max_segments >= 1 &&
                    (mode == 0 || mode == 1),
                "avc_graph_split: bad args");
  Split* s = new Split;
  if (build(reinterpret_cast<hipGraph_t>(graph), reinterpret_cast<hipGraphNode_t const*>(main_tails), n_main,
            reinterpret_cast<hipGraphNode_t const*>(side_tails), n_side, max_segments, mode,
            static_cast<unsigned*>(fault_word), s)) {
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
  if (s->sync) {
    // mode 1: the side graph's wait nodes order it after the main graph's signals on the device
    GCHK(hipGraphLaunch(s->em[0], m), "avc_graph_launch2");
    // diagnostic (AVC_GRAPH_M1_SERIAL=1): the side graph starts after the whole main graph
    static const bool serial = getenv("AVC_GRAPH_M1_SERIAL") && getenv("AVC_GRAPH_M1_SERIAL")[0] == '1';
    if (serial) {
      GCHK(hipEventRecord(s->join, m), "avc_graph_launch2");
      GCHK(hipStreamWaitEvent(sd, s->join, 0), "avc_graph_launch2");
    }
    GCHK(hipGraphLaunch(s->es[0], sd), "avc_graph_launch2");
  }
  for (size_t k = 0; k < s->em.size() && !s->sync; ++k) {
    GCHK(hipGraphLaunch(s->em[k], m), "avc_graph_launch2");
    if (s->es[k]) {
      GCHK(hipEventRecord(s->ev[k], m), "avc_graph_launch2");
      GCHK(hipStreamWaitEvent(sd, s->ev[k], 0), "avc_graph_launch2");
      GCHK(hipGraphLaunch(s->es[k], sd), "avc_graph_launch2");
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
