// Native graph index of libdgl_hip: the structure behind the reference's 45
// graph_index._CAPI_* functions (src/graph/graph_apis.cc), re-designed around
// flat arrays.
//
// The reference keeps a mutable graph as per-vertex adjacency vectors
// (include/dgl/graph.h: adjlist_, reverse_adjlist_, all_edges_*) and an
// immutable one as two CSRs (include/dgl/immutable_graph.h). Here:
//   * MutableGraph stores the edge list in edge-id order (src_, dst_, eid_) —
//     append-only, one contiguous array per field — and derives its in- and
//     out-adjacency as CSRs built on demand by a stable counting sort, cached
//     until the next mutation. A CSR row lists its slots in edge-insertion
//     order, which is exactly the order of the reference's adjacency vectors,
//     so every query returns the same sequence.
//   * ImmutableGraph holds the in-CSR (rows = dst) and/or out-CSR (rows = src)
//     with each row sorted by neighbour id (immutable_graph.cc:206-237; ties
//     between parallel edges keep input order, which the reference leaves to
//     std::sort); the missing one is derived by a transpose on first use.
#pragma once

#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "runtime.h"

namespace dglhip {
namespace gi {

using id_vec = std::vector<int64_t>;

// Allocator whose resize() leaves new elements uninitialised: the edge arrays
// of a 10^9-edge graph are filled in parallel right after they grow, so a
// serial zero-fill (and its page faults) would double the cost of AddEdges.
template <typename T>
struct uninit_allocator : std::allocator<T> {
  template <typename U> struct rebind { using other = uninit_allocator<U>; };
  uninit_allocator() = default;
  template <typename U> uninit_allocator(const uninit_allocator<U>&) noexcept {}
  template <typename U> void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
  template <typename U, typename... A> void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
using edge_vec = std::vector<int64_t, uninit_allocator<int64_t>>;

// Compressed adjacency: row r owns slots [indptr[r], indptr[r+1]); indices[k]
// is the neighbour and eid[k] the edge id of slot k.
struct CSR {
  id_vec indptr{0};
  edge_vec indices;
  edge_vec eid;
  int64_t rows() const { return static_cast<int64_t>(indptr.size()) - 1; }
  int64_t nnz() const { return static_cast<int64_t>(indices.size()); }
  int64_t degree(int64_t r) const { return indptr[r + 1] - indptr[r]; }
};
using CSRPtr = std::shared_ptr<const CSR>;

// Rows of a CSR built from entries (row[i], col[i], id[i]); a row's slots keep
// the entries' input order (stable counting sort), or, with sort_cols, are
// ordered by (col, input position).
CSR build_csr(int64_t nrows, int64_t ncols, const int64_t* row, const int64_t* col,
              const int64_t* id, int64_t n, bool sort_cols);

struct EdgeArrays {
  id_vec src, dst, id;
};

class Graph;

struct Subgraph {
  std::shared_ptr<Graph> graph;
  id_vec induced_vertices;
  id_vec induced_edges;
};

// Id array view: host, 1-D, int64 (IsValidIdArray, src/c_api_common.h:35-38).
struct Ids {
  const int64_t* p = nullptr;
  int64_t n = 0;
  int64_t operator[](int64_t i) const { return p[i]; }
};

class Graph {
 public:
  explicit Graph(bool multigraph) : multigraph_(multigraph) {}
  virtual ~Graph() = default;
  virtual std::unique_ptr<Graph> clone() const = 0;

  virtual bool readonly() const = 0;
  bool multigraph() const { return multigraph_; }
  virtual int64_t num_vertices() const = 0;
  virtual int64_t num_edges() const = 0;
  bool has_vertex(int64_t v) const { return v >= 0 && v < num_vertices(); }
  void check_vertex(int64_t v) const;

  // Mutation (MutableGraph only).
  virtual void add_vertices(int64_t n);
  virtual void add_edge(int64_t u, int64_t v);
  virtual void add_edges(Ids u, Ids v);
  virtual void clear();

  virtual bool has_edge_between(int64_t u, int64_t v) const = 0;
  virtual id_vec predecessors(int64_t v) const = 0;
  virtual id_vec successors(int64_t v) const = 0;
  // Ids of the edges u -> v (graph_interface.h:151).
  virtual id_vec edge_id(int64_t u, int64_t v) const = 0;
  // All edges between the (broadcast) pairs, in pair order (graph.cc:205-249).
  EdgeArrays edge_ids(Ids u, Ids v) const;
  id_vec has_edges_between(Ids u, Ids v) const;
  virtual EdgeArrays find_edges(Ids e) const;
  virtual EdgeArrays in_edges(Ids v) const = 0;
  virtual EdgeArrays out_edges(Ids v) const = 0;
  virtual EdgeArrays edges(const std::string& order) const = 0;
  virtual int64_t in_degree(int64_t v) const = 0;
  virtual int64_t out_degree(int64_t v) const = 0;
  // in-adjacency (rows = dst) and out-adjacency (rows = src), built on demand
  virtual CSRPtr in_csr() const = 0;
  virtual CSRPtr out_csr() const = 0;
  virtual id_vec in_degrees(Ids v) const;
  virtual id_vec out_degrees(Ids v) const;
  virtual Subgraph vertex_subgraph(Ids v) const = 0;
  virtual Subgraph edge_subgraph(Ids e) const;
  // [idx(2E), eid(E)] for "coo", [indptr, indices, eid] for "csr"
  // (graph.cc:506-554, immutable_graph.cc:553-575).
  virtual std::vector<rt::NDArray> get_adj(bool transpose, const std::string& fmt) const = 0;

 protected:
  bool multigraph_;
};

class MutableGraph : public Graph {
 public:
  explicit MutableGraph(bool multigraph = false) : Graph(multigraph) {}
  MutableGraph(Ids src, Ids dst, Ids eid, int64_t num_nodes, bool multigraph);
  MutableGraph(const MutableGraph& o);
  std::unique_ptr<Graph> clone() const override;

  bool readonly() const override { return false; }
  int64_t num_vertices() const override { return n_; }
  int64_t num_edges() const override { return static_cast<int64_t>(src_.size()); }

  void add_vertices(int64_t n) override;
  void add_edge(int64_t u, int64_t v) override;
  void add_edges(Ids u, Ids v) override;
  void clear() override;

  bool has_edge_between(int64_t u, int64_t v) const override;
  id_vec predecessors(int64_t v) const override;
  id_vec successors(int64_t v) const override;
  id_vec edge_id(int64_t u, int64_t v) const override;
  EdgeArrays find_edges(Ids e) const override;
  EdgeArrays in_edges(Ids v) const override;
  EdgeArrays out_edges(Ids v) const override;
  EdgeArrays edges(const std::string& order) const override;
  int64_t in_degree(int64_t v) const override;
  int64_t out_degree(int64_t v) const override;
  id_vec in_degrees(Ids v) const override;
  id_vec out_degrees(Ids v) const override;
  Subgraph vertex_subgraph(Ids v) const override;
  Subgraph edge_subgraph(Ids e) const override;
  std::vector<rt::NDArray> get_adj(bool transpose, const std::string& fmt) const override;

  // graph_op.cc
  MutableGraph line_graph(bool backtracking) const;
  static MutableGraph disjoint_union(const std::vector<const MutableGraph*>& graphs);
  std::vector<MutableGraph> partition_by_sizes(const id_vec& sizes) const;

  const edge_vec& src() const { return src_; }
  const edge_vec& dst() const { return dst_; }
  const edge_vec& eid() const { return eid_; }
  CSRPtr in_csr() const override;   // rows = dst, slots in edge-insertion order
  CSRPtr out_csr() const override;  // rows = src

 private:
  void invalidate();
  // per-vertex in/out degree, counted from the edge arrays on demand (no CSR
  // needed: the reference's adjacency vectors know their sizes)
  std::shared_ptr<const id_vec> degree_table(bool in) const;
  int64_t n_ = 0;
  edge_vec src_, dst_, eid_;  // per edge position; eid_ = id kept in the adjacency
  mutable std::mutex mu_;
  mutable CSRPtr in_, out_;
  mutable std::shared_ptr<const id_vec> in_deg_, out_deg_;
};

class ImmutableGraph : public Graph {
 public:
  ImmutableGraph(CSRPtr in_csr, CSRPtr out_csr, bool multigraph);
  ImmutableGraph(Ids src, Ids dst, Ids eid, int64_t num_nodes, bool multigraph);
  ImmutableGraph(const ImmutableGraph& o);
  std::unique_ptr<Graph> clone() const override;

  bool readonly() const override { return true; }
  int64_t num_vertices() const override;
  int64_t num_edges() const override;

  bool has_edge_between(int64_t u, int64_t v) const override;
  id_vec predecessors(int64_t v) const override;
  id_vec successors(int64_t v) const override;
  id_vec edge_id(int64_t u, int64_t v) const override;
  EdgeArrays in_edges(Ids v) const override;
  EdgeArrays out_edges(Ids v) const override;
  EdgeArrays edges(const std::string& order) const override;
  int64_t in_degree(int64_t v) const override;
  int64_t out_degree(int64_t v) const override;
  Subgraph vertex_subgraph(Ids v) const override;
  std::vector<rt::NDArray> get_adj(bool transpose, const std::string& fmt) const override;

  CSRPtr in_csr() const override;   // rows = dst, indices = src, sorted per row
  CSRPtr out_csr() const override;  // rows = src, indices = dst, sorted per row

 private:
  mutable std::mutex mu_;
  mutable CSRPtr in_, out_;
};

// Degree-bucketing schedule (sched::DegreeBucketing, src/scheduler/scheduler.cc:
// 13-93): [degs, nids, nid_section, mids, mid_section].
std::vector<rt::NDArray> degree_bucketing(Ids msg_ids, Ids vids, Ids recv_ids);

Ids id_arg(const rt::Args& a, int i);
Graph* graph_arg(const rt::Args& a, int i);

}  // namespace gi
}  // namespace dglhip
