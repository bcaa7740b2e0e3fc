// Native graph index and the 45 graph_index._CAPI_* functions of the
// reference (src/graph/graph_apis.cc:98-482), on the flat-array structures of
// graph_index.h. Argument lists, return conventions and results follow the
// reference function by function; each implementation cites what it restates.
#include "graph_index.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <numeric>
#include <random>
#include <set>
#include <unordered_map>
#include <unordered_set>

namespace dglhip {
namespace gi {

using rt::Args;
using rt::Body;
using rt::NDArray;
using rt::RetValue;

namespace {

int num_threads() { return default_num_threads(); }

NDArray to_nd(const id_vec& v) { return NDArray::FromVector(v); }
NDArray to_nd(const edge_vec& v) { return NDArray::FromIds(v.data(), static_cast<int64_t>(v.size())); }

Body edge_array_func(const EdgeArrays& ea) {
  // ConvertEdgeArrayToPackedFunc (graph_apis.cc:21-36): 0 src, 1 dst, 2 id.
  return rt::ndarray_vector_func({to_nd(ea.src), to_nd(ea.dst), to_nd(ea.id)});
}

Body subgraph_func(const Subgraph& sg) {
  // ConvertSubgraphToPackedFunc (graph_apis.cc:52-69): 0 graph handle (a new
  // graph object owned by the caller), 1 induced vertices, 2 induced edges.
  auto graph = sg.graph;
  NDArray nv = to_nd(sg.induced_vertices), ne = to_nd(sg.induced_edges);
  return [graph, nv, ne](const Args& a, RetValue* rv) {
    const int64_t which = a.i64(0);
    if (which == 0) {
      rv->set_handle(graph->clone().release());
    } else if (which == 1) {
      rv->set_array(nv);
    } else if (which == 2) {
      rv->set_array(ne);
    } else {
      DGLHIP_CHECK(false, "invalid choice " << which);
    }
  };
}

[[noreturn]] void unsupported(const char* what, const char* kind) {
  throw Error(std::string(what) + " isn't supported in " + kind);
}

// Positions p[0..k) of k distinct items drawn uniformly from [0, n), ascending
// (Floyd's algorithm; the reference's RandomSample + sort draws from the same
// distribution, immutable_graph.cc:663-741).
void sample_positions(int64_t n, int64_t k, std::mt19937_64* rng, id_vec* out) {
  std::unordered_set<int64_t> chosen;
  chosen.reserve(static_cast<size_t>(k) * 2);
  for (int64_t j = n - k; j < n; ++j) {
    std::uniform_int_distribution<int64_t> d(0, j);
    const int64_t t = d(*rng);
    if (!chosen.insert(t).second) chosen.insert(j);
  }
  out->assign(chosen.begin(), chosen.end());
  std::sort(out->begin(), out->end());
}

}  // namespace

// ------------------------------------------------------------------ CSR
// First entry i in [0, n) with !ok(i), or -1 (parallel scan; the reported
// entry is the lowest failing one, so the message does not depend on threads).
template <typename Ok>
static int64_t first_invalid(int64_t n, Ok&& ok) {
  std::atomic<int64_t> bad{n};
  parallel_for(n, num_threads(), [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e && i < bad.load(std::memory_order_relaxed); ++i)
      if (!ok(i)) {
        int64_t cur = bad.load();
        while (i < cur && !bad.compare_exchange_weak(cur, i)) {}
        break;
      }
  }, int64_t(1) << 16);
  return bad.load() == n ? -1 : bad.load();
}

// Stable scatter of input entries into the CSR, parallel and O(n) reads in
// total. The rows are split into `parts` nnz-balanced ranges and the input
// into `parts` contiguous chunks. Pass 1: every chunk counts its entries per
// range; pass 2: every chunk writes its entries' input positions into a
// staging array grouped by (range, chunk) (offsets from a prefix sum in that
// order); pass 3: every range places its staged entries, which are in input
// order, row by row. So a row's slots keep input order whatever the thread
// count, and each pass reads the input once (the earlier version had every
// thread scan all n entries: n x threads reads).
template <typename Pos>
static void place_stable(int64_t n, const int64_t* row, const int64_t* col, const int64_t* id,
                         const std::vector<int64_t>& bounds, CSR& c) {
  const int parts = static_cast<int>(bounds.size()) - 1;
  // range of each row: binary search over the (few) bounds
  auto range_of = [&](int64_t r) {
    return static_cast<int>(std::upper_bound(bounds.begin() + 1, bounds.end() - 1, r) -
                            (bounds.begin() + 1));
  };
  std::vector<int64_t> cnt(static_cast<size_t>(parts) * parts, 0);  // [chunk][range]
  auto chunk_beg = [&](int t) { return n * t / parts; };
  parallel_for(parts, parts, [&](int64_t b, int64_t e, int) {
    for (int64_t t = b; t < e; ++t) {
      int64_t* ct = cnt.data() + t * parts;
      for (int64_t i = chunk_beg(static_cast<int>(t)); i < chunk_beg(static_cast<int>(t) + 1); ++i)
        ++ct[range_of(row[i])];
    }
  }, 2);
  std::vector<int64_t> off(static_cast<size_t>(parts) * parts);  // (range, chunk) order
  std::vector<int64_t> range_start(static_cast<size_t>(parts) + 1, n);
  int64_t acc = 0;
  for (int p = 0; p < parts; ++p) {
    range_start[p] = acc;
    for (int t = 0; t < parts; ++t) {
      off[static_cast<size_t>(t) * parts + p] = acc;
      acc += cnt[static_cast<size_t>(t) * parts + p];
    }
  }
  std::vector<Pos> stage(static_cast<size_t>(n));
  parallel_for(parts, parts, [&](int64_t b, int64_t e, int) {
    for (int64_t t = b; t < e; ++t) {
      int64_t* ot = off.data() + t * parts;
      for (int64_t i = chunk_beg(static_cast<int>(t)); i < chunk_beg(static_cast<int>(t) + 1); ++i)
        stage[ot[range_of(row[i])]++] = static_cast<Pos>(i);
    }
  }, 2);
  parallel_for(parts, parts, [&](int64_t b, int64_t e, int) {
    for (int64_t p = b; p < e; ++p) {
      const int64_t r0 = bounds[p], r1 = bounds[p + 1];
      if (r0 >= r1) continue;
      id_vec pos(c.indptr.begin() + r0, c.indptr.begin() + r1);
      for (int64_t s = range_start[p]; s < range_start[p + 1]; ++s) {
        const int64_t i = static_cast<int64_t>(stage[s]);
        const int64_t k = pos[row[i] - r0]++;
        c.indices[k] = col[i];
        c.eid[k] = id ? id[i] : i;
      }
    }
  }, 2);
}

CSR build_csr(int64_t nrows, int64_t ncols, const int64_t* row, const int64_t* col,
              const int64_t* id, int64_t n, bool sort_cols) {
  // Stable counting sort by row. Degrees are counted with relaxed atomic adds;
  // placement (place_stable) splits the rows into nnz-balanced ranges, so a
  // row's slots keep input order whatever the thread count.
  CSR c;
  const int64_t bad = first_invalid(n, [&](int64_t i) {
    return row[i] >= 0 && row[i] < nrows && col[i] >= 0 && col[i] < ncols;
  });
  DGLHIP_CHECK(bad < 0, "Invalid vertices: " << row[bad] << ", " << col[bad]);
  c.indptr.assign(static_cast<size_t>(nrows) + 1, 0);
  int64_t* cnt = c.indptr.data() + 1;
  const int nt = num_threads();
  parallel_for(n, nt, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) __atomic_fetch_add(&cnt[row[i]], 1, __ATOMIC_RELAXED);
  }, int64_t(1) << 16);
  for (int64_t r = 0; r < nrows; ++r) c.indptr[r + 1] += c.indptr[r];
  c.indices.resize(n);
  c.eid.resize(n);
  const int parts = (n >= (int64_t(1) << 20)) ? nt : 1;
  std::vector<int64_t> bounds(parts + 1, nrows);
  bounds[0] = 0;
  for (int t = 1; t < parts; ++t) {
    bounds[t] = std::upper_bound(c.indptr.begin(), c.indptr.end(), n * t / parts) -
                c.indptr.begin() - 1;
    bounds[t] = std::max(bounds[t], bounds[t - 1]);
  }
  if (parts == 1) {
    id_vec pos(c.indptr.begin(), c.indptr.end() - 1);
    for (int64_t i = 0; i < n; ++i) {
      const int64_t k = pos[row[i]]++;
      c.indices[k] = col[i];
      c.eid[k] = id ? id[i] : i;
    }
  } else if (n <= int64_t(0xffffffff)) {
    place_stable<uint32_t>(n, row, col, id, bounds, c);
  } else {
    place_stable<int64_t>(n, row, col, id, bounds, c);
  }
  if (sort_cols) {
    parallel_for(nrows, num_threads(), [&](int64_t b, int64_t e, int) {
      std::vector<std::pair<int64_t, int64_t>> tmp;
      for (int64_t r = b; r < e; ++r) {
        const int64_t s = c.indptr[r], t = c.indptr[r + 1];
        if (std::is_sorted(c.indices.begin() + s, c.indices.begin() + t)) continue;
        tmp.clear();
        for (int64_t k = s; k < t; ++k) tmp.emplace_back(c.indices[k], c.eid[k]);
        std::stable_sort(tmp.begin(), tmp.end(),
                         [](const auto& x, const auto& y) { return x.first < y.first; });
        for (int64_t k = s; k < t; ++k) {
          c.indices[k] = tmp[k - s].first;
          c.eid[k] = tmp[k - s].second;
        }
      }
    });
  }
  return c;
}

// Transposed CSR: entry (r, indices[k]) becomes (indices[k], r). Rows of the
// source are scanned in ascending order, so each new row comes out sorted by
// neighbour with parallel edges in their old slot order
// (ImmutableGraph::CSR::Transpose, immutable_graph.cc:254-258).
static CSRPtr transpose(const CSR& c) {
  const int64_t n = c.rows();
  id_vec row(c.nnz());
  for (int64_t r = 0; r < n; ++r)
    std::fill(row.begin() + c.indptr[r], row.begin() + c.indptr[r + 1], r);
  return std::make_shared<CSR>(
      build_csr(n, n, c.indices.data(), row.data(), c.eid.data(), c.nnz(), false));
}

// ------------------------------------------------------------------ Graph
void Graph::check_vertex(int64_t v) const {
  DGLHIP_CHECK(has_vertex(v), "invalid vertex: " << v);
}

void Graph::add_vertices(int64_t) { unsupported("AddVertices", "ImmutableGraph"); }
void Graph::add_edge(int64_t, int64_t) { unsupported("AddEdge", "ImmutableGraph"); }
void Graph::add_edges(Ids, Ids) { unsupported("AddEdges", "ImmutableGraph"); }
void Graph::clear() { unsupported("Clear", "ImmutableGraph"); }
EdgeArrays Graph::find_edges(Ids) const { unsupported("FindEdges", "ImmutableGraph"); }
Subgraph Graph::edge_subgraph(Ids) const { unsupported("EdgeSubgraph", "ImmutableGraph"); }

EdgeArrays Graph::edge_ids(Ids u, Ids v) const {
  // graph.cc:205-249 / immutable_graph.cc:414-456: one-many, many-one or
  // pairwise; every edge between each pair, pairs in order.
  DGLHIP_CHECK(u.n == v.n || u.n == 1 || v.n == 1, "Invalid src and dst id array.");
  const int64_t us = (u.n == 1 && v.n != 1) ? 0 : 1;
  const int64_t vs = (v.n == 1 && u.n != 1) ? 0 : 1;
  EdgeArrays out;
  for (int64_t i = 0, j = 0; i < u.n && j < v.n; i += us, j += vs) {
    const int64_t a = u[i], b = v[j];
    DGLHIP_CHECK(has_vertex(a) && has_vertex(b), "invalid edge: " << a << " -> " << b);
    for (int64_t e : edge_id(a, b)) {
      out.src.push_back(a);
      out.dst.push_back(b);
      out.id.push_back(e);
    }
  }
  return out;
}

id_vec Graph::has_edges_between(Ids u, Ids v) const {
  // graph.cc:117-145
  id_vec out;
  if (u.n == 1) {
    for (int64_t i = 0; i < v.n; ++i) out.push_back(has_edge_between(u[0], v[i]) ? 1 : 0);
  } else if (v.n == 1) {
    for (int64_t i = 0; i < u.n; ++i) out.push_back(has_edge_between(u[i], v[0]) ? 1 : 0);
  } else {
    DGLHIP_CHECK(u.n == v.n, "Invalid src and dst id array.");
    for (int64_t i = 0; i < u.n; ++i) out.push_back(has_edge_between(u[i], v[i]) ? 1 : 0);
  }
  return out;
}

static id_vec degrees_of(const Graph& g, const CSR& c, Ids v) {
  const int64_t bad = first_invalid(v.n, [&](int64_t i) { return g.has_vertex(v[i]); });
  DGLHIP_CHECK(bad < 0, "Invalid vertex: " << v[bad]);
  id_vec out(v.n);
  parallel_for(v.n, num_threads(), [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) out[i] = c.degree(v[i]);
  }, int64_t(1) << 16);
  return out;
}

id_vec Graph::in_degrees(Ids v) const { return degrees_of(*this, *in_csr(), v); }

id_vec Graph::out_degrees(Ids v) const { return degrees_of(*this, *out_csr(), v); }

// ------------------------------------------------------------------ MutableGraph
MutableGraph::MutableGraph(Ids src, Ids dst, Ids eid, int64_t num_nodes, bool multigraph)
    : Graph(multigraph) {
  // Graph::Graph(src_ids, dst_ids, edge_ids, ...) (graph.cc:16-45).
  DGLHIP_CHECK(src.n == dst.n && src.n == eid.n, "vectors in COO must have the same length");
  DGLHIP_CHECK(num_nodes >= 0, "invalid number of nodes " << num_nodes);
  n_ = num_nodes;
  const int64_t bad = first_invalid(src.n, [&](int64_t i) {
    return has_vertex(src[i]) && has_vertex(dst[i]);
  });
  DGLHIP_CHECK(bad < 0, "Invalid vertices: src=" << src[bad] << " dst=" << dst[bad]);
  src_.assign(src.p, src.p + src.n);
  dst_.assign(dst.p, dst.p + dst.n);
  eid_.assign(eid.p, eid.p + eid.n);
}

MutableGraph::MutableGraph(const MutableGraph& o)
    : Graph(o.multigraph_), n_(o.n_), src_(o.src_), dst_(o.dst_), eid_(o.eid_) {
  std::lock_guard<std::mutex> lk(o.mu_);
  in_ = o.in_;
  out_ = o.out_;
}

std::unique_ptr<Graph> MutableGraph::clone() const {
  return std::unique_ptr<Graph>(new MutableGraph(*this));
}

void MutableGraph::invalidate() {
  std::lock_guard<std::mutex> lk(mu_);
  in_.reset();
  out_.reset();
  in_deg_.reset();
  out_deg_.reset();
}

std::shared_ptr<const id_vec> MutableGraph::degree_table(bool in) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto& slot = in ? in_deg_ : out_deg_;
  if (!slot) {
    auto deg = std::make_shared<id_vec>(static_cast<size_t>(n_), 0);
    const edge_vec& end = in ? dst_ : src_;
    int64_t* d = deg->data();
    parallel_for(num_edges(), num_threads(), [&](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; ++i) __atomic_fetch_add(&d[end[i]], 1, __ATOMIC_RELAXED);
    }, int64_t(1) << 16);
    slot = deg;
  }
  return slot;
}

static id_vec lookup_degrees(const Graph& g, const id_vec& deg, Ids v) {
  const int64_t bad = first_invalid(v.n, [&](int64_t i) { return g.has_vertex(v[i]); });
  DGLHIP_CHECK(bad < 0, "Invalid vertex: " << v[bad]);
  id_vec out(v.n);
  parallel_for(v.n, num_threads(), [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) out[i] = deg[v[i]];
  }, int64_t(1) << 16);
  return out;
}

id_vec MutableGraph::in_degrees(Ids v) const { return lookup_degrees(*this, *degree_table(true), v); }

id_vec MutableGraph::out_degrees(Ids v) const {
  return lookup_degrees(*this, *degree_table(false), v);
}

CSRPtr MutableGraph::in_csr() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (!in_)
    in_ = std::make_shared<CSR>(
        build_csr(n_, n_, dst_.data(), src_.data(), eid_.data(), num_edges(), false));
  return in_;
}

CSRPtr MutableGraph::out_csr() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (!out_)
    out_ = std::make_shared<CSR>(
        build_csr(n_, n_, src_.data(), dst_.data(), eid_.data(), num_edges(), false));
  return out_;
}

void MutableGraph::add_vertices(int64_t n) {
  DGLHIP_CHECK(n >= 0, "invalid number of vertices " << n);
  n_ += n;
  invalidate();
}

void MutableGraph::add_edge(int64_t u, int64_t v) {
  // graph.cc:53-67: the new edge's id is the current edge count.
  DGLHIP_CHECK(has_vertex(u) && has_vertex(v), "Invalid vertices: src=" << u << " dst=" << v);
  eid_.push_back(num_edges());
  src_.push_back(u);
  dst_.push_back(v);
  invalidate();
}

void MutableGraph::add_edges(Ids u, Ids v) {
  // graph.cc:69-94 (one-many, many-one, many-many). All ids are validated
  // before any edge is added.
  int64_t m;
  if (u.n == 1) {
    m = v.n;
  } else if (v.n == 1) {
    m = u.n;
  } else {
    DGLHIP_CHECK(u.n == v.n, "Invalid src and dst id array.");
    m = u.n;
  }
  const int64_t us = u.n == 1 ? 0 : 1, vs = (v.n == 1 && u.n != 1) ? 0 : 1;
  const int64_t bad = first_invalid(m, [&](int64_t i) {
    return has_vertex(u[i * us]) && has_vertex(v[i * vs]);
  });
  DGLHIP_CHECK(bad < 0, "Invalid vertices: src=" << u[bad * us] << " dst=" << v[bad * vs]);
  const int64_t e0 = num_edges();
  // geometric growth even for one bulk append (a graph of 10^9 edges is built
  // by one call; growing to the exact size would make repeated small appends
  // quadratic)
  const size_t need = static_cast<size_t>(e0 + m);
  if (src_.capacity() < need) {
    const size_t cap = std::max(need, 2 * src_.capacity());
    src_.reserve(cap);
    dst_.reserve(cap);
    eid_.reserve(cap);
  }
  src_.resize(need);
  dst_.resize(need);
  eid_.resize(need);
  parallel_for(m, num_threads(), [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) {
      src_[e0 + i] = u[i * us];
      dst_[e0 + i] = v[i * vs];
      eid_[e0 + i] = e0 + i;
    }
  }, int64_t(1) << 16);
  invalidate();
}

void MutableGraph::clear() {
  n_ = 0;
  src_.clear();
  dst_.clear();
  eid_.clear();
  invalidate();
}

bool MutableGraph::has_edge_between(int64_t u, int64_t v) const {
  if (!has_vertex(u) || !has_vertex(v)) return false;
  auto c = out_csr();
  const auto b = c->indices.begin();
  return std::find(b + c->indptr[u], b + c->indptr[u + 1], v) != b + c->indptr[u + 1];
}

id_vec MutableGraph::predecessors(int64_t v) const {
  // graph.cc:148-162: distinct predecessors, ascending.
  check_vertex(v);
  auto c = in_csr();
  std::set<int64_t> s(c->indices.begin() + c->indptr[v], c->indices.begin() + c->indptr[v + 1]);
  return id_vec(s.begin(), s.end());
}

id_vec MutableGraph::successors(int64_t v) const {
  check_vertex(v);
  auto c = out_csr();
  std::set<int64_t> s(c->indices.begin() + c->indptr[v], c->indices.begin() + c->indptr[v + 1]);
  return id_vec(s.begin(), s.end());
}

id_vec MutableGraph::edge_id(int64_t u, int64_t v) const {
  // graph.cc:182-202: u's out-edges to v in insertion order.
  DGLHIP_CHECK(has_vertex(u) && has_vertex(v), "invalid edge: " << u << " -> " << v);
  auto c = out_csr();
  id_vec out;
  for (int64_t k = c->indptr[u]; k < c->indptr[u + 1]; ++k)
    if (c->indices[k] == v) out.push_back(c->eid[k]);
  return out;
}

EdgeArrays MutableGraph::find_edges(Ids e) const {
  // graph.cc:251-273
  EdgeArrays out;
  out.src.resize(e.n);
  out.dst.resize(e.n);
  out.id.resize(e.n);
  for (int64_t i = 0; i < e.n; ++i) {
    DGLHIP_CHECK(e[i] >= 0 && e[i] < num_edges(), "invalid edge id:" << e[i]);
    out.src[i] = src_[e[i]];
    out.dst[i] = dst_[e[i]];
    out.id[i] = e[i];
  }
  return out;
}

EdgeArrays MutableGraph::in_edges(Ids v) const {
  // graph.cc:276-319
  auto c = in_csr();
  EdgeArrays out;
  for (int64_t i = 0; i < v.n; ++i) DGLHIP_CHECK(has_vertex(v[i]), "Invalid vertex: " << v[i]);
  for (int64_t i = 0; i < v.n; ++i)
    for (int64_t k = c->indptr[v[i]]; k < c->indptr[v[i] + 1]; ++k) {
      out.src.push_back(c->indices[k]);
      out.dst.push_back(v[i]);
      out.id.push_back(c->eid[k]);
    }
  return out;
}

EdgeArrays MutableGraph::out_edges(Ids v) const {
  // graph.cc:322-365
  auto c = out_csr();
  EdgeArrays out;
  for (int64_t i = 0; i < v.n; ++i) DGLHIP_CHECK(has_vertex(v[i]), "Invalid vertex: " << v[i]);
  for (int64_t i = 0; i < v.n; ++i)
    for (int64_t k = c->indptr[v[i]]; k < c->indptr[v[i] + 1]; ++k) {
      out.src.push_back(v[i]);
      out.dst.push_back(c->indices[k]);
      out.id.push_back(c->eid[k]);
    }
  return out;
}

EdgeArrays MutableGraph::edges(const std::string& order) const {
  // graph.cc:368-409: "srcdst" sorts by (src, dst) (parallel edges keep id
  // order); anything else is edge-id order.
  const int64_t m = num_edges();
  id_vec perm(m);
  std::iota(perm.begin(), perm.end(), 0);
  if (order == "srcdst") {
    std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) {
      return src_[a] < src_[b] || (src_[a] == src_[b] && dst_[a] < dst_[b]);
    });
  }
  EdgeArrays out;
  out.src.resize(m);
  out.dst.resize(m);
  out.id = perm;
  for (int64_t i = 0; i < m; ++i) {
    out.src[i] = src_[perm[i]];
    out.dst[i] = dst_[perm[i]];
  }
  return out;
}

int64_t MutableGraph::in_degree(int64_t v) const {
  check_vertex(v);
  return (*degree_table(true))[v];
}

int64_t MutableGraph::out_degree(int64_t v) const {
  check_vertex(v);
  return (*degree_table(false))[v];
}

Subgraph MutableGraph::vertex_subgraph(Ids v) const {
  // graph.cc:441-469: vertex i of the subgraph is v[i]; edges are the
  // out-edges of v[0], v[1], ... (insertion order) that land inside the set.
  std::unordered_map<int64_t, int64_t> newid;
  newid.reserve(static_cast<size_t>(v.n) * 2);
  for (int64_t i = 0; i < v.n; ++i) {
    DGLHIP_CHECK(has_vertex(v[i]), "Invalid vertex: " << v[i]);
    newid[v[i]] = i;
  }
  auto c = out_csr();
  auto g = std::make_shared<MutableGraph>(multigraph_);
  g->n_ = v.n;
  Subgraph sg;
  for (int64_t i = 0; i < v.n; ++i)
    for (int64_t k = c->indptr[v[i]]; k < c->indptr[v[i] + 1]; ++k) {
      auto it = newid.find(c->indices[k]);
      if (it == newid.end()) continue;
      sg.induced_edges.push_back(c->eid[k]);
      g->eid_.push_back(g->num_edges());
      g->src_.push_back(i);
      g->dst_.push_back(it->second);
    }
  sg.induced_vertices.assign(v.p, v.p + v.n);
  sg.graph = g;
  return sg;
}

Subgraph MutableGraph::edge_subgraph(Ids e) const {
  // graph.cc:471-504: vertices numbered in first-appearance order over
  // (src, dst) of the listed edges; edge i of the subgraph is e[i].
  std::unordered_map<int64_t, int64_t> newid;
  Subgraph sg;
  for (int64_t i = 0; i < e.n; ++i) {
    DGLHIP_CHECK(e[i] >= 0 && e[i] < num_edges(), "invalid edge id:" << e[i]);
    for (int64_t x : {src_[e[i]], dst_[e[i]]})
      if (newid.emplace(x, static_cast<int64_t>(newid.size())).second)
        sg.induced_vertices.push_back(x);
  }
  auto g = std::make_shared<MutableGraph>(multigraph_);
  g->n_ = static_cast<int64_t>(sg.induced_vertices.size());
  for (int64_t i = 0; i < e.n; ++i) {
    g->src_.push_back(newid[src_[e[i]]]);
    g->dst_.push_back(newid[dst_[e[i]]]);
    g->eid_.push_back(i);
  }
  sg.induced_edges.assign(e.p, e.p + e.n);
  sg.graph = g;
  return sg;
}

std::vector<NDArray> MutableGraph::get_adj(bool transpose, const std::string& fmt) const {
  // graph.cc:506-554
  const int64_t m = num_edges();
  if (fmt == "coo") {
    NDArray idx = NDArray::Ids(2 * m), eid = NDArray::Ids(m);
    int64_t* p = idx.data<int64_t>();
    const edge_vec& first = transpose ? src_ : dst_;
    const edge_vec& second = transpose ? dst_ : src_;
    std::copy(first.begin(), first.end(), p);
    std::copy(second.begin(), second.end(), p + m);
    std::iota(eid.data<int64_t>(), eid.data<int64_t>() + m, int64_t(0));
    return {idx, eid};
  }
  DGLHIP_CHECK(fmt == "csr", "unsupported format " << fmt);
  auto c = transpose ? out_csr() : in_csr();
  return {to_nd(c->indptr), to_nd(c->indices), to_nd(c->eid)};
}

MutableGraph MutableGraph::line_graph(bool backtracking) const {
  // GraphOp::LineGraph (graph_op.cc:17-31): edge i = (u, v) links to every
  // out-edge of v (except those back to u unless backtracking).
  MutableGraph lg(false);
  lg.n_ = num_edges();
  auto c = out_csr();
  for (int64_t i = 0; i < num_edges(); ++i) {
    const int64_t u = src_[i], v = dst_[i];
    for (int64_t k = c->indptr[v]; k < c->indptr[v + 1]; ++k) {
      if (!backtracking && c->indices[k] == u) continue;
      lg.eid_.push_back(lg.num_edges());
      lg.src_.push_back(i);
      lg.dst_.push_back(c->eid[k]);
    }
  }
  return lg;
}

MutableGraph MutableGraph::disjoint_union(const std::vector<const MutableGraph*>& graphs) {
  // GraphOp::DisjointUnion (graph_op.cc:33-45): vertices and edges of each
  // graph follow those of the previous ones.
  MutableGraph g(false);
  for (const MutableGraph* x : graphs) {
    const int64_t off = g.n_;
    g.n_ += x->n_;
    for (int64_t i = 0; i < x->num_edges(); ++i) {
      g.eid_.push_back(g.num_edges());
      g.src_.push_back(x->src_[i] + off);
      g.dst_.push_back(x->dst_[i] + off);
    }
  }
  return g;
}

std::vector<MutableGraph> MutableGraph::partition_by_sizes(const id_vec& sizes) const {
  // GraphOp::DisjointPartitionBySizes (graph_op.cc:57-114): part i takes the
  // next sizes[i] vertices and the next (their out-degree sum) edges. The
  // edges of a part must stay inside it, as in a disjoint union.
  int64_t total = 0;
  for (int64_t s : sizes) {
    DGLHIP_CHECK(s >= 0, "negative partition size " << s);
    total += s;
  }
  DGLHIP_CHECK(total == n_, "Sum of the given sizes must equal to the number of nodes.");
  auto c = out_csr();
  std::vector<MutableGraph> parts;
  int64_t voff = 0, eoff = 0;
  for (int64_t s : sizes) {
    MutableGraph p(multigraph_);
    p.n_ = s;
    const int64_t ne = c->indptr[voff + s] - c->indptr[voff];
    for (int64_t e = eoff; e < eoff + ne; ++e) {
      const int64_t u = src_[e] - voff, v = dst_[e] - voff;
      DGLHIP_CHECK(u >= 0 && u < s && v >= 0 && v < s,
                   "edge " << e << " crosses partitions: the graph is not a disjoint union "
                           "of parts of these sizes");
      p.src_.push_back(u);
      p.dst_.push_back(v);
      p.eid_.push_back(eid_[e] - eoff);
    }
    parts.push_back(std::move(p));
    voff += s;
    eoff += ne;
  }
  return parts;
}

// ------------------------------------------------------------------ ImmutableGraph
ImmutableGraph::ImmutableGraph(CSRPtr in_csr, CSRPtr out_csr, bool multigraph)
    : Graph(multigraph), in_(std::move(in_csr)), out_(std::move(out_csr)) {
  DGLHIP_CHECK(in_ || out_, "one of the CSRs must exist");
}

ImmutableGraph::ImmutableGraph(Ids src, Ids dst, Ids eid, int64_t num_nodes, bool multigraph)
    : Graph(multigraph) {
  // immutable_graph.cc:260-281: in-CSR sorted by (dst, src), out-CSR by (src, dst).
  DGLHIP_CHECK(src.n == dst.n && src.n == eid.n, "vectors in COO must have the same length");
  in_ = std::make_shared<CSR>(build_csr(num_nodes, num_nodes, dst.p, src.p, eid.p, src.n, true));
  out_ = std::make_shared<CSR>(build_csr(num_nodes, num_nodes, src.p, dst.p, eid.p, src.n, true));
}

ImmutableGraph::ImmutableGraph(const ImmutableGraph& o) : Graph(o.multigraph_) {
  std::lock_guard<std::mutex> lk(o.mu_);
  in_ = o.in_;
  out_ = o.out_;
}

std::unique_ptr<Graph> ImmutableGraph::clone() const {
  return std::unique_ptr<Graph>(new ImmutableGraph(*this));
}

CSRPtr ImmutableGraph::in_csr() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (!in_) in_ = transpose(*out_);
  return in_;
}

CSRPtr ImmutableGraph::out_csr() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (!out_) out_ = transpose(*in_);
  return out_;
}

int64_t ImmutableGraph::num_vertices() const {
  std::lock_guard<std::mutex> lk(mu_);
  return in_ ? in_->rows() : out_->rows();
}

int64_t ImmutableGraph::num_edges() const {
  std::lock_guard<std::mutex> lk(mu_);
  return in_ ? in_->nnz() : out_->nnz();
}

bool ImmutableGraph::has_edge_between(int64_t u, int64_t v) const {
  // immutable_graph.cc:296-306: binary search in v's sorted predecessors.
  if (!has_vertex(u) || !has_vertex(v)) return false;
  auto c = in_csr();
  const auto b = c->indices.begin();
  return std::binary_search(b + c->indptr[v], b + c->indptr[v + 1], u);
}

id_vec ImmutableGraph::predecessors(int64_t v) const {
  // immutable_graph.cc:338-349: the in-CSR row as stored.
  check_vertex(v);
  auto c = in_csr();
  return id_vec(c->indices.begin() + c->indptr[v], c->indices.begin() + c->indptr[v + 1]);
}

id_vec ImmutableGraph::successors(int64_t v) const {
  check_vertex(v);
  auto c = out_csr();
  return id_vec(c->indices.begin() + c->indptr[v], c->indices.begin() + c->indptr[v + 1]);
}

id_vec ImmutableGraph::edge_id(int64_t u, int64_t v) const {
  // GetInEdgeIdRef (immutable_graph.cc:364-380): the run of u in v's sorted row.
  DGLHIP_CHECK(has_vertex(u) && has_vertex(v), "invalid edge: " << u << " -> " << v);
  auto c = in_csr();
  const auto b = c->indices.begin() + c->indptr[v], e = c->indices.begin() + c->indptr[v + 1];
  auto lo = std::lower_bound(b, e, u);
  id_vec out;
  for (auto it = lo; it != e && *it == u; ++it) out.push_back(c->eid[it - c->indices.begin()]);
  return out;
}

EdgeArrays ImmutableGraph::in_edges(Ids v) const {
  // CSR::GetEdges (immutable_graph.cc:47-76)
  auto c = in_csr();
  EdgeArrays out;
  for (int64_t i = 0; i < v.n; ++i) DGLHIP_CHECK(has_vertex(v[i]), "Invalid vertex: " << v[i]);
  for (int64_t i = 0; i < v.n; ++i)
    for (int64_t k = c->indptr[v[i]]; k < c->indptr[v[i] + 1]; ++k) {
      out.src.push_back(c->indices[k]);
      out.dst.push_back(v[i]);
      out.id.push_back(c->eid[k]);
    }
  return out;
}

EdgeArrays ImmutableGraph::out_edges(Ids v) const {
  // immutable_graph.h:299-313: GetEdges on the out-CSR with the ends swapped.
  auto c = out_csr();
  EdgeArrays out;
  for (int64_t i = 0; i < v.n; ++i) DGLHIP_CHECK(has_vertex(v[i]), "Invalid vertex: " << v[i]);
  for (int64_t i = 0; i < v.n; ++i)
    for (int64_t k = c->indptr[v[i]]; k < c->indptr[v[i] + 1]; ++k) {
      out.src.push_back(v[i]);
      out.dst.push_back(c->indices[k]);
      out.id.push_back(c->eid[k]);
    }
  return out;
}

EdgeArrays ImmutableGraph::edges(const std::string& order) const {
  // immutable_graph.cc:458-493: "" / "srcdst" walks the out-CSR; "eid" sorts
  // by edge id.
  DGLHIP_CHECK(order.empty() || order == "srcdst" || order == "eid",
               "unsupported order " << order);
  auto c = out_csr();
  EdgeArrays out;
  const int64_t m = c->nnz();
  out.src.resize(m);
  out.dst.assign(c->indices.begin(), c->indices.end());
  out.id.assign(c->eid.begin(), c->eid.end());
  for (int64_t r = 0; r < c->rows(); ++r)
    std::fill(out.src.begin() + c->indptr[r], out.src.begin() + c->indptr[r + 1], r);
  if (order == "eid") {
    id_vec perm(m);
    std::iota(perm.begin(), perm.end(), 0);
    std::stable_sort(perm.begin(), perm.end(),
                     [&](int64_t a, int64_t b) { return c->eid[a] < c->eid[b]; });
    EdgeArrays s;
    for (int64_t i : perm) {
      s.src.push_back(out.src[i]);
      s.dst.push_back(out.dst[i]);
      s.id.push_back(out.id[i]);
    }
    return s;
  }
  return out;
}

int64_t ImmutableGraph::in_degree(int64_t v) const {
  check_vertex(v);
  return in_csr()->degree(v);
}

int64_t ImmutableGraph::out_degree(int64_t v) const {
  check_vertex(v);
  return out_csr()->degree(v);
}

Subgraph ImmutableGraph::vertex_subgraph(Ids v) const {
  // immutable_graph.cc:167-204,495-512: sorted vertex list; the subgraph keeps
  // the CSR the parent has (out-CSR preferred), entries whose neighbour is in
  // the set, renumbered; new edge ids are slot positions.
  DGLHIP_CHECK(std::is_sorted(v.p, v.p + v.n), "The input vertex list has to be sorted");
  std::unordered_map<int64_t, int64_t> newid;
  newid.reserve(static_cast<size_t>(v.n) * 2);
  for (int64_t i = 0; i < v.n; ++i) {
    DGLHIP_CHECK(has_vertex(v[i]), "Vertex Id " << v[i] << " isn't in a graph of "
                                                 << num_vertices() << " vertices");
    newid[v[i]] = i;
  }
  bool use_out;
  CSRPtr c;
  {
    std::lock_guard<std::mutex> lk(mu_);
    use_out = out_ != nullptr;
    c = use_out ? out_ : in_;
  }
  auto sub = std::make_shared<CSR>();
  sub->indptr.assign(static_cast<size_t>(v.n) + 1, 0);
  Subgraph sg;
  for (int64_t i = 0; i < v.n; ++i) {
    for (int64_t k = c->indptr[v[i]]; k < c->indptr[v[i] + 1]; ++k) {
      auto it = newid.find(c->indices[k]);
      if (it == newid.end()) continue;
      sub->indices.push_back(it->second);
      sg.induced_edges.push_back(c->eid[k]);
    }
    sub->indptr[i + 1] = sub->nnz();
  }
  sub->eid.resize(sub->nnz());
  std::iota(sub->eid.begin(), sub->eid.end(), int64_t(0));
  sg.graph = use_out ? std::make_shared<ImmutableGraph>(nullptr, sub, multigraph_)
                     : std::make_shared<ImmutableGraph>(sub, nullptr, multigraph_);
  sg.induced_vertices.assign(v.p, v.p + v.n);
  return sg;
}

std::vector<NDArray> ImmutableGraph::get_adj(bool transpose, const std::string& fmt) const {
  // immutable_graph.cc:553-575
  auto c = transpose ? out_csr() : in_csr();
  if (fmt == "csr") return {to_nd(c->indptr), to_nd(c->indices), to_nd(c->eid)};
  DGLHIP_CHECK(fmt == "coo", "unsupported adjacency matrix format " << fmt);
  const int64_t m = c->nnz();
  NDArray idx = NDArray::Ids(2 * m);
  int64_t* p = idx.data<int64_t>();
  for (int64_t r = 0; r < c->rows(); ++r)
    std::fill(p + c->indptr[r], p + c->indptr[r + 1], r);
  std::copy(c->indices.begin(), c->indices.end(), p + m);
  return {idx, to_nd(c->eid)};
}

// ------------------------------------------------------------------ sampling
namespace {

struct Sampled {
  std::shared_ptr<Graph> graph;
  id_vec vertices, edges, layers;
  std::vector<float> prob;
};

std::atomic<uint64_t> g_sample_calls{0};

uint64_t sample_seed(int64_t i) {
  // Fresh per call and per seed set (the reference seeds rand_r with
  // time(nullptr), immutable_graph.cc:797).
  const uint64_t t = static_cast<uint64_t>(
      std::chrono::high_resolution_clock::now().time_since_epoch().count());
  return t ^ (g_sample_calls.fetch_add(1) * 0x9E3779B97F4A7C15ull) ^ (uint64_t(i) << 32);
}

// ImmutableGraph::SampleSubgraph + CompactSubgraph (immutable_graph.cc:
// 792-1011), uniform case: breadth-first from the seeds; each vertex above the
// last hop keeps min(deg, k) of its neighbours (all of them, or k drawn
// uniformly without replacement, in row order); the subgraph's vertices are
// the visited ids ascending, with their hop as layer id.
Sampled sample_neighbors(const ImmutableGraph& g, Ids seeds, bool in_dir, int num_hops,
                         int64_t k, uint64_t seed) {
  DGLHIP_CHECK(k >= 0 && num_hops >= 0, "invalid sampling parameters");
  auto csr = in_dir ? g.in_csr() : g.out_csr();
  std::mt19937_64 rng(seed);
  std::unordered_set<int64_t> seen;
  std::vector<std::pair<int64_t, int>> queue;
  for (int64_t i = 0; i < seeds.n; ++i) {
    g.check_vertex(seeds[i]);
    if (seen.insert(seeds[i]).second) queue.emplace_back(seeds[i], 0);
  }
  // Sampled neighbour lists per expanded vertex: (vertex, [ (nbr, eid)... ]).
  std::vector<std::pair<int64_t, std::pair<id_vec, id_vec>>> lists;
  id_vec pos;
  for (size_t q = 0; q < queue.size(); ++q) {
    const int64_t v = queue[q].first;
    const int level = queue[q].second;
    if (level >= num_hops) continue;
    const int64_t s = csr->indptr[v], deg = csr->degree(v);
    id_vec nbr, eid;
    if (deg <= k) {
      nbr.assign(csr->indices.begin() + s, csr->indices.begin() + s + deg);
      eid.assign(csr->eid.begin() + s, csr->eid.begin() + s + deg);
    } else {
      sample_positions(deg, k, &rng, &pos);
      for (int64_t p : pos) {
        nbr.push_back(csr->indices[s + p]);
        eid.push_back(csr->eid[s + p]);
      }
    }
    for (int64_t x : nbr)
      if (seen.insert(x).second) queue.emplace_back(x, level + 1);
    lists.emplace_back(v, std::make_pair(std::move(nbr), std::move(eid)));
  }
  std::sort(queue.begin(), queue.end(),
            [](const auto& a, const auto& b) { return a.first < b.first; });
  std::sort(lists.begin(), lists.end(),
            [](const auto& a, const auto& b) { return a.first < b.first; });
  Sampled out;
  const int64_t nv = static_cast<int64_t>(queue.size());
  std::unordered_map<int64_t, int64_t> newid;
  newid.reserve(static_cast<size_t>(nv) * 2);
  for (int64_t i = 0; i < nv; ++i) {
    out.vertices.push_back(queue[i].first);
    out.layers.push_back(queue[i].second);
    newid[queue[i].first] = i;
  }
  out.prob.assign(nv, 0.0f);
  auto sub = std::make_shared<CSR>();
  sub->indptr.assign(static_cast<size_t>(nv) + 1, 0);
  size_t li = 0;
  for (int64_t i = 0; i < nv; ++i) {
    if (li < lists.size() && lists[li].first == out.vertices[i]) {
      for (int64_t x : lists[li].second.first) sub->indices.push_back(newid.at(x));
      for (int64_t e : lists[li].second.second) out.edges.push_back(e);
      ++li;
    }
    sub->indptr[i + 1] = sub->nnz();
  }
  sub->eid.resize(sub->nnz());
  std::iota(sub->eid.begin(), sub->eid.end(), int64_t(0));
  out.graph = in_dir ? std::make_shared<ImmutableGraph>(sub, nullptr, g.multigraph())
                     : std::make_shared<ImmutableGraph>(nullptr, sub, g.multigraph());
  return out;
}

Body sampled_func(std::vector<Sampled> sg) {
  // ConvertSubgraphToPackedFunc(vector<SampledSubgraph>) (graph_apis.cc:72-95):
  // [graphs..., vertices..., edges..., layer ids..., sample probs...].
  auto holder = std::make_shared<std::vector<Sampled>>(std::move(sg));
  return [holder](const Args& a, RetValue* rv) {
    const int64_t n = static_cast<int64_t>(holder->size());
    const int64_t which = a.i64(0);
    DGLHIP_CHECK(which >= 0 && which < 5 * n, "invalid choice " << which);
    const Sampled& s = (*holder)[which % n];
    switch (which / n) {
      case 0:
        rv->set_handle(s.graph->clone().release());
        break;
      case 1:
        rv->set_array(to_nd(s.vertices));
        break;
      case 2:
        rv->set_array(to_nd(s.edges));
        break;
      case 3:
        rv->set_array(to_nd(s.layers));
        break;
      default: {
        NDArray p = NDArray::Empty({static_cast<int64_t>(s.prob.size())}, 2, 32);
        if (!s.prob.empty()) std::memcpy(p.data<float>(), s.prob.data(), s.prob.size() * 4);
        rv->set_array(p);
      }
    }
  };
}

void neighbor_uniform_sample(int num_seeds, const Args& a, RetValue* rv) {
  // CAPI_NeighborUniformSample<num_seeds> (graph_apis.cc:431-455): handle,
  // num_seeds seed arrays, neighbour type, hops, fan-out, valid seed arrays.
  Graph* g = graph_arg(a, 0);
  auto* ig = dynamic_cast<ImmutableGraph*>(g);
  DGLHIP_CHECK(ig, "sampling isn't implemented in mutable graph");
  std::vector<Ids> seeds;
  for (int i = 0; i < num_seeds; ++i) seeds.push_back(id_arg(a, i + 1));
  const std::string neigh_type = a.str(num_seeds + 1);
  const int num_hops = static_cast<int>(a.i64(num_seeds + 2));
  const int64_t num_neighbors = a.i64(num_seeds + 3);
  const int num_valid = static_cast<int>(a.i64(num_seeds + 4));
  DGLHIP_CHECK(num_valid >= 0 && num_valid <= num_seeds, "invalid number of seed arrays");
  DGLHIP_CHECK(neigh_type == "in" || neigh_type == "out",
               "neighbor type must be 'in' or 'out', got " << neigh_type);
  std::vector<Sampled> out(num_seeds);
  id_vec base_seeds(num_seeds);
  for (int i = 0; i < num_seeds; ++i) base_seeds[i] = static_cast<int64_t>(sample_seed(i));
  parallel_for(num_valid, num_threads(), [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i)
      out[i] = sample_neighbors(*ig, seeds[i], neigh_type == "in", num_hops, num_neighbors,
                                static_cast<uint64_t>(base_seeds[i]));
  }, 2);
  for (int i = num_valid; i < num_seeds; ++i) {  // padding slots: empty subgraphs
    out[i].graph = std::make_shared<ImmutableGraph>(std::make_shared<CSR>(), nullptr,
                                                    ig->multigraph());
  }
  rv->set_func(sampled_func(std::move(out)));
}

template <int N>
void sample_capi(const Args& a, RetValue* rv) {
  neighbor_uniform_sample(N, a, rv);
}

}  // namespace

// ------------------------------------------------------------------ arguments
Ids id_arg(const Args& a, int i) {
  const DGLHipTensor* t = a.tensor(i);
  DGLHIP_CHECK(t->device_type == rt::kDLCPU && t->ndim == 1 && t->dtype_code == 0 &&
                   t->dtype_bits == 64 && t->dtype_lanes == 1,
               "Invalid id array (argument " << i << "): expected a 1-D int64 CPU array");
  Ids ids;
  ids.n = t->shape[0];
  ids.p = rt::data_as<int64_t>(t, 0, 64, "id array");
  return ids;
}

Graph* graph_arg(const Args& a, int i) {
  auto* g = static_cast<Graph*>(a.handle(i));
  DGLHIP_CHECK(g, "null graph handle");
  return g;
}

static MutableGraph* mutable_arg(const Args& a, int i, const char* api) {
  auto* g = dynamic_cast<MutableGraph*>(graph_arg(a, i));
  DGLHIP_CHECK(g, api << " isn't implemented in immutable graph");
  return g;
}

// IdArray of handles of new graphs (graph_apis.cc:382-420).
static NDArray handle_array(std::vector<MutableGraph>&& parts) {
  NDArray arr = NDArray::Ids(static_cast<int64_t>(parts.size()));
  for (size_t i = 0; i < parts.size(); ++i)
    arr.data<int64_t>()[i] =
        reinterpret_cast<intptr_t>(static_cast<Graph*>(new MutableGraph(std::move(parts[i]))));
  return arr;
}

// GraphOp::MapParentIdToSubgraphId (graph_op.cc:116-157): position of each
// query id in parent_vids, -1 when absent.
static NDArray map_subgraph_nid(Ids parent, Ids query) {
  NDArray out = NDArray::Ids(query.n);
  int64_t* r = out.data<int64_t>();
  if (std::is_sorted(parent.p, parent.p + parent.n)) {
    for (int64_t i = 0; i < query.n; ++i) {
      const int64_t* it = std::lower_bound(parent.p, parent.p + parent.n, query[i]);
      r[i] = (it != parent.p + parent.n && *it == query[i]) ? it - parent.p : -1;
    }
  } else {
    std::unordered_map<int64_t, int64_t> m;
    for (int64_t i = 0; i < parent.n; ++i) m[parent[i]] = i;
    for (int64_t i = 0; i < query.n; ++i) {
      auto it = m.find(query[i]);
      r[i] = it == m.end() ? -1 : it->second;
    }
  }
  return out;
}

}  // namespace gi

void register_graph_index_functions() {
  using namespace gi;
  using rt::register_global;
  const std::string ns = "graph_index._CAPI_";

  register_global(ns + "DGLGraphCreateMutable", [](const Args& a, RetValue* rv) {
    rv->set_handle(static_cast<Graph*>(new MutableGraph(a.b(0))));
  });
  register_global(ns + "DGLGraphCreate", [](const Args& a, RetValue* rv) {
    // (src_ids, dst_ids, edge_ids, multigraph, num_nodes, readonly)
    Ids src = id_arg(a, 0), dst = id_arg(a, 1), eid = id_arg(a, 2);
    const bool multigraph = a.b(3), readonly = a.b(5);
    const int64_t n = a.i64(4);
    Graph* g = readonly ? static_cast<Graph*>(new ImmutableGraph(src, dst, eid, n, multigraph))
                        : static_cast<Graph*>(new MutableGraph(src, dst, eid, n, multigraph));
    rv->set_handle(g);
  });
  register_global(ns + "DGLGraphFree", [](const Args& a, RetValue*) {
    delete static_cast<Graph*>(a.handle(0));
  });
  register_global(ns + "DGLGraphAddVertices", [](const Args& a, RetValue*) {
    graph_arg(a, 0)->add_vertices(a.i64(1));
  });
  register_global(ns + "DGLGraphAddEdge", [](const Args& a, RetValue*) {
    graph_arg(a, 0)->add_edge(a.i64(1), a.i64(2));
  });
  register_global(ns + "DGLGraphAddEdges", [](const Args& a, RetValue*) {
    graph_arg(a, 0)->add_edges(id_arg(a, 1), id_arg(a, 2));
  });
  register_global(ns + "DGLGraphClear", [](const Args& a, RetValue*) {
    graph_arg(a, 0)->clear();
  });
  register_global(ns + "DGLGraphIsMultigraph", [](const Args& a, RetValue* rv) {
    rv->set_bool(graph_arg(a, 0)->multigraph());
  });
  register_global(ns + "DGLGraphIsReadonly", [](const Args& a, RetValue* rv) {
    rv->set_bool(graph_arg(a, 0)->readonly());
  });
  register_global(ns + "DGLGraphNumVertices", [](const Args& a, RetValue* rv) {
    rv->set_int(graph_arg(a, 0)->num_vertices());
  });
  register_global(ns + "DGLGraphNumEdges", [](const Args& a, RetValue* rv) {
    rv->set_int(graph_arg(a, 0)->num_edges());
  });
  register_global(ns + "DGLGraphHasVertex", [](const Args& a, RetValue* rv) {
    rv->set_bool(graph_arg(a, 0)->has_vertex(a.i64(1)));
  });
  register_global(ns + "DGLGraphHasVertices", [](const Args& a, RetValue* rv) {
    Graph* g = graph_arg(a, 0);
    Ids v = id_arg(a, 1);
    id_vec out(v.n);
    for (int64_t i = 0; i < v.n; ++i) out[i] = g->has_vertex(v[i]) ? 1 : 0;
    rv->set_array(to_nd(out));
  });
  register_global(ns + "DGLMapSubgraphNID", [](const Args& a, RetValue* rv) {
    rv->set_array(map_subgraph_nid(id_arg(a, 0), id_arg(a, 1)));
  });
  register_global(ns + "DGLGraphHasEdgeBetween", [](const Args& a, RetValue* rv) {
    rv->set_bool(graph_arg(a, 0)->has_edge_between(a.i64(1), a.i64(2)));
  });
  register_global(ns + "DGLGraphHasEdgesBetween", [](const Args& a, RetValue* rv) {
    rv->set_array(to_nd(graph_arg(a, 0)->has_edges_between(id_arg(a, 1), id_arg(a, 2))));
  });
  register_global(ns + "DGLGraphPredecessors", [](const Args& a, RetValue* rv) {
    DGLHIP_CHECK(a.i64(2) >= 1, "invalid radius: " << a.i64(2));
    rv->set_array(to_nd(graph_arg(a, 0)->predecessors(a.i64(1))));
  });
  register_global(ns + "DGLGraphSuccessors", [](const Args& a, RetValue* rv) {
    DGLHIP_CHECK(a.i64(2) >= 1, "invalid radius: " << a.i64(2));
    rv->set_array(to_nd(graph_arg(a, 0)->successors(a.i64(1))));
  });
  register_global(ns + "DGLGraphEdgeId", [](const Args& a, RetValue* rv) {
    rv->set_array(to_nd(graph_arg(a, 0)->edge_id(a.i64(1), a.i64(2))));
  });
  register_global(ns + "DGLGraphEdgeIds", [](const Args& a, RetValue* rv) {
    rv->set_func(edge_array_func(graph_arg(a, 0)->edge_ids(id_arg(a, 1), id_arg(a, 2))));
  });
  register_global(ns + "DGLGraphFindEdges", [](const Args& a, RetValue* rv) {
    rv->set_func(edge_array_func(graph_arg(a, 0)->find_edges(id_arg(a, 1))));
  });
  register_global(ns + "DGLGraphInEdges_1", [](const Args& a, RetValue* rv) {
    const int64_t v = a.i64(1);
    Graph* g = graph_arg(a, 0);
    g->check_vertex(v);
    rv->set_func(edge_array_func(g->in_edges(Ids{&v, 1})));
  });
  register_global(ns + "DGLGraphInEdges_2", [](const Args& a, RetValue* rv) {
    rv->set_func(edge_array_func(graph_arg(a, 0)->in_edges(id_arg(a, 1))));
  });
  register_global(ns + "DGLGraphOutEdges_1", [](const Args& a, RetValue* rv) {
    const int64_t v = a.i64(1);
    Graph* g = graph_arg(a, 0);
    g->check_vertex(v);
    rv->set_func(edge_array_func(g->out_edges(Ids{&v, 1})));
  });
  register_global(ns + "DGLGraphOutEdges_2", [](const Args& a, RetValue* rv) {
    rv->set_func(edge_array_func(graph_arg(a, 0)->out_edges(id_arg(a, 1))));
  });
  register_global(ns + "DGLGraphEdges", [](const Args& a, RetValue* rv) {
    Graph* g = graph_arg(a, 0);
    const std::string order = a.str(1);
    auto* mg = dynamic_cast<MutableGraph*>(g);
    if (mg && order != "srcdst") {
      // id order is the storage order: one copy per array straight into the
      // returned NDArrays (no permutation, no intermediate vectors), which is
      // what the engine reads to build its device CSRs of 10^9-edge graphs
      rv->set_func(rt::ndarray_vector_func(
          {to_nd(mg->src()), to_nd(mg->dst()), to_nd(mg->eid())}));
      return;
    }
    rv->set_func(edge_array_func(g->edges(order)));
  });
  register_global(ns + "DGLGraphInDegree", [](const Args& a, RetValue* rv) {
    rv->set_int(graph_arg(a, 0)->in_degree(a.i64(1)));
  });
  register_global(ns + "DGLGraphInDegrees", [](const Args& a, RetValue* rv) {
    rv->set_array(to_nd(graph_arg(a, 0)->in_degrees(id_arg(a, 1))));
  });
  register_global(ns + "DGLGraphOutDegree", [](const Args& a, RetValue* rv) {
    rv->set_int(graph_arg(a, 0)->out_degree(a.i64(1)));
  });
  register_global(ns + "DGLGraphOutDegrees", [](const Args& a, RetValue* rv) {
    rv->set_array(to_nd(graph_arg(a, 0)->out_degrees(id_arg(a, 1))));
  });
  register_global(ns + "DGLGraphVertexSubgraph", [](const Args& a, RetValue* rv) {
    rv->set_func(subgraph_func(graph_arg(a, 0)->vertex_subgraph(id_arg(a, 1))));
  });
  register_global(ns + "DGLGraphEdgeSubgraph", [](const Args& a, RetValue* rv) {
    rv->set_func(subgraph_func(graph_arg(a, 0)->edge_subgraph(id_arg(a, 1))));
  });
  register_global(ns + "DGLDisjointUnion", [](const Args& a, RetValue* rv) {
    // (pointer to an array of graph handles, count)
    auto** handles = static_cast<void**>(a.handle(0));
    const int64_t n = a.i64(1);
    DGLHIP_CHECK(n == 0 || handles, "null graph list");
    std::vector<const MutableGraph*> graphs;
    for (int64_t i = 0; i < n; ++i) {
      auto* g = dynamic_cast<const MutableGraph*>(static_cast<Graph*>(handles[i]));
      DGLHIP_CHECK(g, "_CAPI_DGLDisjointUnion isn't implemented in immutable graph");
      graphs.push_back(g);
    }
    rv->set_handle(static_cast<Graph*>(new MutableGraph(MutableGraph::disjoint_union(graphs))));
  });
  register_global(ns + "DGLDisjointPartitionByNum", [](const Args& a, RetValue* rv) {
    MutableGraph* g = mutable_arg(a, 0, "_CAPI_DGLDisjointPartitionByNum");
    const int64_t num = a.i64(1);
    DGLHIP_CHECK(num > 0 && g->num_vertices() % num == 0,
                 "Number of partitions must evenly divide the number of nodes.");
    rv->set_array(handle_array(g->partition_by_sizes(id_vec(num, g->num_vertices() / num))));
  });
  register_global(ns + "DGLDisjointPartitionBySizes", [](const Args& a, RetValue* rv) {
    MutableGraph* g = mutable_arg(a, 0, "_CAPI_DGLDisjointPartitionBySizes");
    Ids sizes = id_arg(a, 1);
    rv->set_array(handle_array(g->partition_by_sizes(id_vec(sizes.p, sizes.p + sizes.n))));
  });
  register_global(ns + "DGLGraphLineGraph", [](const Args& a, RetValue* rv) {
    MutableGraph* g = mutable_arg(a, 0, "_CAPI_DGLGraphLineGraph");
    rv->set_handle(static_cast<Graph*>(new MutableGraph(g->line_graph(a.b(1)))));
  });
  register_global(ns + "DGLGraphUniformSampling", sample_capi<1>);
  register_global(ns + "DGLGraphUniformSampling2", sample_capi<2>);
  register_global(ns + "DGLGraphUniformSampling4", sample_capi<4>);
  register_global(ns + "DGLGraphUniformSampling8", sample_capi<8>);
  register_global(ns + "DGLGraphUniformSampling16", sample_capi<16>);
  register_global(ns + "DGLGraphUniformSampling32", sample_capi<32>);
  register_global(ns + "DGLGraphUniformSampling64", sample_capi<64>);
  register_global(ns + "DGLGraphUniformSampling128", sample_capi<128>);
  register_global(ns + "DGLGraphGetAdj", [](const Args& a, RetValue* rv) {
    // (handle, transpose, format) -> indexable [arrays] (graph_apis.cc:474-482)
    rv->set_func(rt::ndarray_vector_func(graph_arg(a, 0)->get_adj(a.b(1), a.str(2))));
  });
}

}  // namespace dglhip
