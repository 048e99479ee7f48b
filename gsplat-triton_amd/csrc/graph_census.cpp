// Node census of a captured HIP graph: the training step replayed as a graph
// (gsplat_hip/graph_step.py) must hold kernel nodes only -- see DESIGN §3.12
// for the memset nodes whose replays faulted.  The host side checks the census
// after every capture, so a stray torch.zeros / hipMemsetAsync inside the
// captured region fails loudly at capture time instead of at replay.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace gs {
void set_error(const char *fmt, ...);
}

// counts[t] += number of nodes of hipGraphNodeType t (t < 16; larger types
// land in counts[15]); for the first max_memsets memset nodes, memsets[4 k ..
// 4 k + 3] = (destination address, bytes per row, rows, element size).
// Returns 0, or 2 when a HIP graph query fails.
extern "C" int gsplat_hip_graph_node_census(void *graph, int64_t *counts, int64_t *memsets,
                                            int max_memsets) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
  size_t n = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &n);
  if (e != hipSuccess) {
    gs::set_error("graph_node_census: hipGraphGetNodes: %s", hipGetErrorString(e));
    return 2;
  }
  std::vector<hipGraphNode_t> nodes(n);
  if (n) {
    e = hipGraphGetNodes(g, nodes.data(), &n);
    if (e != hipSuccess) {
      gs::set_error("graph_node_census: hipGraphGetNodes: %s", hipGetErrorString(e));
      return 2;
    }
  }
  int k = 0;
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    e = hipGraphNodeGetType(nodes[i], &t);
    if (e != hipSuccess) {
      gs::set_error("graph_node_census: hipGraphNodeGetType: %s", hipGetErrorString(e));
      return 2;
    }
    const int ti = (int)t;
    counts[(ti >= 0 && ti < 16) ? ti : 15] += 1;
    if (t == hipGraphNodeTypeMemset && memsets && k < max_memsets) {
      hipMemsetParams p{};
      if (hipGraphMemsetNodeGetParams(nodes[i], &p) == hipSuccess) {
        memsets[4 * k] = (int64_t)reinterpret_cast<uintptr_t>(p.dst);
        memsets[4 * k + 1] = (int64_t)p.width * (int64_t)p.elementSize;
        memsets[4 * k + 2] = (int64_t)p.height;
        memsets[4 * k + 3] = (int64_t)p.elementSize;
      }
      ++k;
    }
  }
  return 0;
}

// The memcpy nodes of a captured graph (ABI 31): for the first max_nodes,
// out[4 k .. 4 k + 3] = (destination, source, bytes, hipMemcpyKind), -1 where
// the node's parameters cannot be read.  RCCL's one-rank exchange inside a
// captured Gaussian-sharded step is such a node (a device-to-device copy of
// the rank's own block); graph_step allows device-to-device copies there.
// Returns 0, or 2 when a HIP graph query fails.
extern "C" int gsplat_hip_graph_memcpy_census(void *graph, int64_t *out, int max_nodes,
                                              int *n_out) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
  size_t n = 0;
  *n_out = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) {
    gs::set_error("graph_memcpy_census: hipGraphGetNodes failed");
    return 2;
  }
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) {
    gs::set_error("graph_memcpy_census: hipGraphGetNodes failed");
    return 2;
  }
  int k = 0;
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess) {
      gs::set_error("graph_memcpy_census: hipGraphNodeGetType failed");
      return 2;
    }
    if (t != hipGraphNodeTypeMemcpy) continue;
    if (k < max_nodes) {
      hipMemcpy3DParms p{};
      int64_t *o = out + 4 * k;
      o[0] = o[1] = o[2] = o[3] = -1;
      const hipError_t qe = hipGraphMemcpyNodeGetParams(nodes[i], &p);
      if (qe == hipSuccess) {
        o[0] = (int64_t)reinterpret_cast<uintptr_t>(p.dstPtr.ptr);
        o[1] = (int64_t)reinterpret_cast<uintptr_t>(p.srcPtr.ptr);
        o[2] = (int64_t)p.extent.width * (int64_t)p.extent.height * (int64_t)p.extent.depth;
        o[3] = (int64_t)p.kind;
      } else {
        o[3] = -1000 - (int64_t)qe;  // unreadable: -1000 - the HIP error code
      }
    }
    ++k;
  }
  *n_out = k;
  return 0;
}
