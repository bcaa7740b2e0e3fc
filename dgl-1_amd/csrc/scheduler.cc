// Degree-bucketing schedule behind runtime.degree_bucketing._CAPI_* (the
// reference's src/scheduler/scheduler.cc:13-93 and scheduler_apis.cc:16-60).
//
// The reference groups messages with unordered_maps, so its bucket and node
// order is whatever the hash tables yield. This build fixes one order: buckets
// by ascending degree, nodes ascending inside a bucket, each node's messages
// in message order, zero-degree receivers last (ascending) as a degree-0
// bucket with no message section — the same five arrays, deterministic.
#include <algorithm>
#include <numeric>

#include "graph_index.h"

namespace dglhip {
namespace gi {

using rt::Args;
using rt::NDArray;
using rt::RetValue;

std::vector<NDArray> degree_bucketing(Ids msg_ids, Ids vids, Ids recv_ids) {
  const int64_t m = msg_ids.n;
  DGLHIP_CHECK(vids.n == m, "message ids and destinations differ in length ("
                                << m << " vs " << vids.n << ")");
  // Messages grouped by destination, message order kept inside a group.
  id_vec order(m);
  std::iota(order.begin(), order.end(), int64_t(0));
  std::stable_sort(order.begin(), order.end(),
                   [&](int64_t a, int64_t b) { return vids[a] < vids[b]; });
  struct Node {
    int64_t deg, vid, first;  // first: offset of its messages in `order`
  };
  std::vector<Node> nodes;
  for (int64_t i = 0; i < m;) {
    int64_t j = i;
    while (j < m && vids[order[j]] == vids[order[i]]) ++j;
    nodes.push_back({j - i, vids[order[i]], i});
    i = j;
  }
  std::stable_sort(nodes.begin(), nodes.end(),
                   [](const Node& a, const Node& b) { return a.deg < b.deg; });
  // Receivers without messages (scheduler.cc:33-39).
  id_vec zero;
  {
    id_vec present;
    for (const Node& n : nodes) present.push_back(n.vid);
    std::sort(present.begin(), present.end());
    for (int64_t i = 0; i < recv_ids.n; ++i)
      if (!std::binary_search(present.begin(), present.end(), recv_ids[i]))
        zero.push_back(recv_ids[i]);
    std::sort(zero.begin(), zero.end());
    zero.erase(std::unique(zero.begin(), zero.end()), zero.end());
  }
  id_vec degs, nid_section, mid_section, nids, mids;
  nids.reserve(nodes.size() + zero.size());
  mids.reserve(m);
  for (size_t i = 0; i < nodes.size();) {
    size_t j = i;
    while (j < nodes.size() && nodes[j].deg == nodes[i].deg) ++j;
    degs.push_back(nodes[i].deg);
    nid_section.push_back(static_cast<int64_t>(j - i));
    mid_section.push_back(nodes[i].deg * static_cast<int64_t>(j - i));
    for (size_t k = i; k < j; ++k) {
      nids.push_back(nodes[k].vid);
      for (int64_t t = 0; t < nodes[k].deg; ++t) mids.push_back(msg_ids[order[nodes[k].first + t]]);
    }
    i = j;
  }
  if (!zero.empty()) {
    degs.push_back(0);
    nid_section.push_back(static_cast<int64_t>(zero.size()));
    nids.insert(nids.end(), zero.begin(), zero.end());
  }
  return {NDArray::FromVector(degs), NDArray::FromVector(nids), NDArray::FromVector(nid_section),
          NDArray::FromVector(mids), NDArray::FromVector(mid_section)};
}

}  // namespace gi

void register_scheduler_functions() {
  using namespace gi;
  using rt::register_global;
  const std::string ns = "runtime.degree_bucketing._CAPI_";
  register_global(ns + "DGLDegreeBucketing", [](const Args& a, RetValue* rv) {
    // (msg_ids, vids, recv_ids)
    rv->set_func(rt::ndarray_vector_func(degree_bucketing(id_arg(a, 0), id_arg(a, 1),
                                                          id_arg(a, 2))));
  });
  register_global(ns + "DGLDegreeBucketingForEdges", [](const Args& a, RetValue* rv) {
    // (vids): message i goes to vids[i]; receivers are the destinations.
    Ids v = id_arg(a, 0);
    id_vec mid(v.n);
    std::iota(mid.begin(), mid.end(), int64_t(0));
    rv->set_func(rt::ndarray_vector_func(degree_bucketing(Ids{mid.data(), v.n}, v, v)));
  });
  register_global(ns + "DGLDegreeBucketingForRecvNodes", [](const Args& a, RetValue* rv) {
    // (graph, vids): the in-edges of vids are the messages.
    Graph* g = graph_arg(a, 0);
    Ids v = id_arg(a, 1);
    EdgeArrays e = g->in_edges(v);
    const int64_t m = static_cast<int64_t>(e.id.size());
    rv->set_func(rt::ndarray_vector_func(
        degree_bucketing(Ids{e.id.data(), m}, Ids{e.dst.data(), m}, v)));
  });
  register_global(ns + "DGLDegreeBucketingForFullGraph", [](const Args& a, RetValue* rv) {
    // (graph): every edge is a message; every node receives.
    Graph* g = graph_arg(a, 0);
    EdgeArrays e = g->edges("");
    id_vec nodes(g->num_vertices());
    std::iota(nodes.begin(), nodes.end(), int64_t(0));
    const int64_t m = static_cast<int64_t>(e.id.size());
    rv->set_func(rt::ndarray_vector_func(degree_bucketing(
        Ids{e.id.data(), m}, Ids{e.dst.data(), m}, Ids{nodes.data(), g->num_vertices()})));
  });
}

}  // namespace dglhip
