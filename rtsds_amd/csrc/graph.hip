// Lane-split replay of a captured multi-stream hipGraph.
//
// A graph captured from several streams (BiSeNet's spatial-path branch beside the context path,
// the DA iteration's concurrent target forward / discriminator phase) is a DAG of per-stream
// chains joined by cross-stream edges.  hipGraphLaunch of such a graph takes the runtime's
// multi-queue path, which enqueues node by node (~12 us of host time per node: 4.8 ms per
// BiSeNet step of ~330 nodes), while a linear graph goes out as one pre-recorded packet batch
// (~0.1 ms).  Here the captured DAG is decomposed into lanes (chains), each lane is cut into
// linear segments at its cross-lane edges, every segment becomes its own executable graph (a
// clone of the captured graph reduced to the segment's nodes), and a launch replays the
// segments on one stream per lane in topological order, with events for the cross-lane edges.
// The same kernels with the same arguments run, in an order the captured edges allow; only
// the submission changes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/rtsds_hip.h"

namespace {

struct Seg {
  int lane = 0;
  int first_topo = 0;
  std::vector<hipGraphNode_t> nodes;  // in lane order (original graph's nodes)
  std::vector<int> waits;             // indices of segments whose completion this one waits for
  hipGraphExec_t exec = nullptr;
  hipEvent_t done = nullptr;
  bool signalled = false;             // some later segment waits on `done`
};

struct SplitGraph {
  int nlanes = 0;
  std::vector<hipStream_t> lanes;  // lanes[0] = the launch stream (set per launch)
  std::vector<Seg> segs;           // launch order
  std::vector<int> lane_last;      // last segment of each lane (joined at the end)
  hipEvent_t start = nullptr;
  int device = 0;
};

void destroy(SplitGraph* s) {
  if (!s) return;
  for (auto& g : s->segs) {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (g.done) (void)hipEventDestroy(g.done);
  }
  for (size_t i = 1; i < s->lanes.size(); ++i)
    if (s->lanes[i]) (void)hipStreamDestroy(s->lanes[i]);
  if (s->start) (void)hipEventDestroy(s->start);
  delete s;
}

}  // namespace

namespace {

// Nodes, edges, a topological order and the lane (chain) of every node of a captured graph.
struct Analysis {
  std::vector<hipGraphNode_t> nodes;
  std::unordered_map<hipGraphNode_t, int> id;
  std::vector<std::vector<int>> preds, succs;
  std::unordered_set<long long> edge_set;
  std::vector<int> topo, pos, lane;
  int nlanes = 1;
};

int analyze(hipGraph_t graph, int max_lanes, Analysis& A) {
  size_t nn = 0, ne = 0;
  if (hipGraphGetNodes(graph, nullptr, &nn) != hipSuccess) return RTSDS_ERR_LAUNCH;
  A.nodes.resize(nn);
  if (nn && hipGraphGetNodes(graph, A.nodes.data(), &nn) != hipSuccess) return RTSDS_ERR_LAUNCH;
  if (hipGraphGetEdges(graph, nullptr, nullptr, &ne) != hipSuccess) return RTSDS_ERR_LAUNCH;
  std::vector<hipGraphNode_t> from(ne), to(ne);
  if (ne && hipGraphGetEdges(graph, from.data(), to.data(), &ne) != hipSuccess) return RTSDS_ERR_LAUNCH;
  for (size_t i = 0; i < nn; ++i) A.id[A.nodes[i]] = (int)i;
  A.preds.assign(nn, {});
  A.succs.assign(nn, {});
  for (size_t e = 0; e < ne; ++e) {
    const int a = A.id.at(from[e]), b = A.id.at(to[e]);
    A.preds[b].push_back(a);
    A.succs[a].push_back(b);
    A.edge_set.insert((long long)a * (long long)nn + b);
  }
  // topological order (Kahn; ready nodes taken in capture order, i.e. the original node index)
  std::vector<int> indeg(nn);
  A.pos.assign(nn, 0);
  for (size_t i = 0; i < nn; ++i) indeg[i] = (int)A.preds[i].size();
  std::vector<int> ready;
  for (size_t i = 0; i < nn; ++i)
    if (!indeg[i]) ready.push_back((int)i);
  while (!ready.empty()) {
    auto it = std::min_element(ready.begin(), ready.end());
    const int v = *it;
    ready.erase(it);
    A.pos[v] = (int)A.topo.size();
    A.topo.push_back(v);
    for (int w : A.succs[v])
      if (--indeg[w] == 0) ready.push_back(w);
  }
  if (A.topo.size() != nn) return RTSDS_ERR_SHAPE;  // not a DAG
  // lanes: each node continues the lane of a predecessor that is still that lane's tail
  // (lowest lane first); otherwise it opens a new lane, or -- past max_lanes -- is appended to
  // the lane of its latest predecessor (an extra, harmless serialisation).
  A.lane.assign(nn, -1);
  std::vector<int> tail;
  for (int v : A.topo) {
    int best = -1;
    for (int p : A.preds[v])
      if (tail[A.lane[p]] == p && (best < 0 || A.lane[p] < best)) best = A.lane[p];
    if (best < 0) {
      if ((int)tail.size() < max_lanes) {
        best = (int)tail.size();
        tail.push_back(-1);
      } else {
        int lp = -1;
        for (int p : A.preds[v])
          if (lp < 0 || A.pos[p] > A.pos[lp]) lp = p;
        best = lp >= 0 ? A.lane[lp] : 0;
      }
    }
    A.lane[v] = best;
    tail[best] = v;
  }
  A.nlanes = std::max<int>(1, (int)tail.size());
  return RTSDS_OK;
}

}  // namespace

extern "C" int rtsds_abi_version(void) { return RTSDS_ABI_VERSION; }

// Nodes captured so far into the graph a capturing stream records into (negative status if the
// stream is not capturing): GraphedStep ends a segment at a collective only when it has nodes.
extern "C" int rtsds_capture_nodes(void* stream) {
  hipStreamCaptureStatus st;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  if (hipStreamGetCaptureInfo_v2((hipStream_t)stream, &st, &id, &g, &deps, &nd) != hipSuccess) return -RTSDS_ERR_LAUNCH;
  if (st != hipStreamCaptureStatusActive || !g) return -RTSDS_ERR_UNSUPPORTED;
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -RTSDS_ERR_LAUNCH;
  return (int)n;
}

// Node count of a captured graph (0: an empty capture, e.g. between two back-to-back collectives).
extern "C" int rtsds_graph_nodes(void* graph) {
  if (!graph) return -RTSDS_ERR_SHAPE;
  size_t n = 0;
  if (hipGraphGetNodes((hipGraph_t)graph, nullptr, &n) != hipSuccess) return -RTSDS_ERR_LAUNCH;
  return (int)n;
}

extern "C" int rtsds_graph_lanes(void* graph, int max_lanes) {
  if (!graph || max_lanes < 1) return -RTSDS_ERR_SHAPE;
  Analysis A;
  const int rc = analyze((hipGraph_t)graph, max_lanes, A);
  return rc == RTSDS_OK ? A.nlanes : -rc;
}

extern "C" int rtsds_graph_split(void* graph_v, int max_lanes, void** handle, int* n_segments, int* n_lanes) {
  if (!graph_v || !handle || max_lanes < 1) return RTSDS_ERR_SHAPE;
  *handle = nullptr;
  hipGraph_t graph = (hipGraph_t)graph_v;
  Analysis A;
  {
    const int rc = analyze(graph, max_lanes, A);
    if (rc != RTSDS_OK) return rc;
  }
  const size_t nn = A.nodes.size();
  const auto& nodes = A.nodes;
  const auto& id = A.id;
  const auto& preds = A.preds;
  const auto& edge_set = A.edge_set;
  const auto& topo = A.topo;
  const auto& pos = A.pos;
  const auto& lane = A.lane;
  for (size_t i = 0; i < nn; ++i) {  // only node types whose clone replays as captured
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess) return RTSDS_ERR_LAUNCH;
    if (t != hipGraphNodeTypeKernel && t != hipGraphNodeTypeMemcpy && t != hipGraphNodeTypeMemset &&
        t != hipGraphNodeTypeEmpty)
      return RTSDS_ERR_UNSUPPORTED;
  }
  const int L = A.nlanes;

  // segments: cut a lane before a node with a cross-lane predecessor and after that predecessor
  std::vector<char> cut_before(nn, 0), cut_after(nn, 0);
  for (size_t v = 0; v < nn; ++v)
    for (int p : preds[v])
      if (lane[p] != lane[v]) {
        cut_before[v] = 1;
        cut_after[p] = 1;
      }
  std::vector<std::vector<int>> lane_nodes(L);
  for (int v : topo) lane_nodes[lane[v]].push_back(v);
  SplitGraph* s = new SplitGraph();
  s->nlanes = L;
  (void)hipGetDevice(&s->device);
  std::vector<int> seg_of(nn, -1);
  std::vector<Seg> segs;
  for (int l = 0; l < L; ++l) {
    int cur = -1, prev = -1;
    for (int v : lane_nodes[l]) {
      if (cur < 0 || cut_before[v] || (prev >= 0 && cut_after[prev])) {
        segs.emplace_back();
        cur = (int)segs.size() - 1;
        segs[cur].lane = l;
        segs[cur].first_topo = pos[v];
      }
      segs[cur].nodes.push_back(nodes[v]);
      seg_of[v] = cur;
      prev = v;
    }
  }
  // launch order: by the topological position of the first node (a segment's cross-lane
  // predecessors all precede its first node, so the segments they end are launched earlier)
  std::vector<int> order(segs.size());
  for (size_t i = 0; i < segs.size(); ++i) order[i] = (int)i;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return segs[a].first_topo < segs[b].first_topo; });
  std::vector<int> rank(segs.size());
  for (size_t i = 0; i < order.size(); ++i) rank[order[i]] = (int)i;
  for (size_t v = 0; v < nn; ++v)
    for (int p : preds[v])
      if (lane[p] != lane[v]) {
        auto& w = segs[seg_of[v]].waits;
        const int src = rank[seg_of[p]];
        if (std::find(w.begin(), w.end(), src) == w.end()) w.push_back(src);
      }
  for (int i : order) s->segs.push_back(std::move(segs[i]));
  for (auto& g : s->segs)
    for (int w : g.waits) s->segs[w].signalled = true;

  int rc = RTSDS_OK;
  // per segment: a clone of the captured graph reduced to the segment's nodes, chained linearly
  for (auto& g : s->segs) {
    hipGraph_t c = nullptr;
    if (hipGraphClone(&c, graph) != hipSuccess) { rc = RTSDS_ERR_LAUNCH; break; }
    std::unordered_set<hipGraphNode_t> keep(g.nodes.begin(), g.nodes.end());
    std::vector<hipGraphNode_t> cl(g.nodes.size());
    for (size_t i = 0; i < g.nodes.size() && rc == RTSDS_OK; ++i)
      if (hipGraphNodeFindInClone(&cl[i], g.nodes[i], c) != hipSuccess) rc = RTSDS_ERR_LAUNCH;
    for (size_t i = 0; i < nn && rc == RTSDS_OK; ++i) {
      if (keep.count(nodes[i])) continue;
      hipGraphNode_t x;
      if (hipGraphNodeFindInClone(&x, nodes[i], c) != hipSuccess || hipGraphDestroyNode(x) != hipSuccess)
        rc = RTSDS_ERR_LAUNCH;
    }
    for (size_t i = 1; i < g.nodes.size() && rc == RTSDS_OK; ++i) {
      const int a = id.at(g.nodes[i - 1]), b = id.at(g.nodes[i]);
      if (!edge_set.count((long long)a * (long long)nn + b) &&
          hipGraphAddDependencies(c, &cl[i - 1], &cl[i], 1) != hipSuccess)
        rc = RTSDS_ERR_LAUNCH;
    }
    if (rc == RTSDS_OK && hipGraphInstantiate(&g.exec, c, nullptr, nullptr, 0) != hipSuccess) rc = RTSDS_ERR_LAUNCH;
    (void)hipGraphDestroy(c);
    if (rc != RTSDS_OK) break;
    if (g.signalled && hipEventCreateWithFlags(&g.done, hipEventDisableTiming) != hipSuccess) {
      rc = RTSDS_ERR_LAUNCH;
      break;
    }
  }
  s->lanes.assign(L, nullptr);
  for (int l = 1; l < L && rc == RTSDS_OK; ++l)
    if (hipStreamCreateWithFlags(&s->lanes[l], hipStreamNonBlocking) != hipSuccess) rc = RTSDS_ERR_LAUNCH;
  if (rc == RTSDS_OK && hipEventCreateWithFlags(&s->start, hipEventDisableTiming) != hipSuccess) rc = RTSDS_ERR_LAUNCH;
  s->lane_last.assign(L, -1);
  for (size_t i = 0; i < s->segs.size(); ++i) s->lane_last[s->segs[i].lane] = (int)i;
  for (int l = 1; l < L && rc == RTSDS_OK; ++l) {
    const int i = s->lane_last[l];
    if (i >= 0 && !s->segs[i].done) {
      s->segs[i].signalled = true;
      if (hipEventCreateWithFlags(&s->segs[i].done, hipEventDisableTiming) != hipSuccess) rc = RTSDS_ERR_LAUNCH;
    }
  }
  if (rc != RTSDS_OK) {
    destroy(s);
    return rc;
  }
  *handle = s;
  if (n_segments) *n_segments = (int)s->segs.size();
  if (n_lanes) *n_lanes = L;
  return RTSDS_OK;
}

extern "C" int rtsds_graph_split_launch(void* handle, void* stream) {
  SplitGraph* s = (SplitGraph*)handle;
  if (!s) return RTSDS_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  s->lanes[0] = st;
  if (s->nlanes > 1) {  // every lane starts after the work already queued on the launch stream
    if (hipEventRecord(s->start, st) != hipSuccess) return RTSDS_ERR_LAUNCH;
    for (int l = 1; l < s->nlanes; ++l)
      if (hipStreamWaitEvent(s->lanes[l], s->start, 0) != hipSuccess) return RTSDS_ERR_LAUNCH;
  }
  for (auto& g : s->segs) {
    hipStream_t ls = s->lanes[g.lane];
    for (int w : g.waits)
      if (hipStreamWaitEvent(ls, s->segs[w].done, 0) != hipSuccess) return RTSDS_ERR_LAUNCH;
    if (hipGraphLaunch(g.exec, ls) != hipSuccess) return RTSDS_ERR_LAUNCH;
    if (g.signalled && hipEventRecord(g.done, ls) != hipSuccess) return RTSDS_ERR_LAUNCH;
  }
  for (int l = 1; l < s->nlanes; ++l) {  // the launch stream joins every lane
    const int i = s->lane_last[l];
    if (i >= 0 && hipStreamWaitEvent(st, s->segs[i].done, 0) != hipSuccess) return RTSDS_ERR_LAUNCH;
  }
  return RTSDS_OK;
}

extern "C" int rtsds_graph_split_destroy(void* handle) {
  destroy((SplitGraph*)handle);
  return RTSDS_OK;
}
