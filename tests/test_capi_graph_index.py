"""The reference's C-ABI boundary on libdgl_hip.so.

Every graph_index._CAPI_* function of src/graph/graph_apis.cc and every
runtime.degree_bucketing._CAPI_* of src/scheduler/scheduler_apis.cc is called
through the PackedFunc runtime exactly as the reference's Python layer calls
it (python/dgl/graph_index.py, runtime/degree_bucketing.py), using the
test-side client in capi_client.py. Expected values are the known answers of
the reference's own tests (tests/graph_index/test_graph_index.py,
tests/graph_index/test_subgraph.py, tests/compute/test_graph_index.py,
tests/compute/test_sampler.py, tests/compute/test_transform.py), restated, and
differential checks against this engine's own graph index and CSR builder.
No GPU is used here.
"""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp
import torch

import capi_client as C
from capi_client import DB, GI, edge_triple, ids

import dgl
from dgl import kernel

GRAPH_API = [
    "DGLGraphCreateMutable", "DGLGraphCreate", "DGLGraphFree", "DGLGraphAddVertices",
    "DGLGraphAddEdge", "DGLGraphAddEdges", "DGLGraphClear", "DGLGraphIsMultigraph",
    "DGLGraphIsReadonly", "DGLGraphNumVertices", "DGLGraphNumEdges", "DGLGraphHasVertex",
    "DGLGraphHasVertices", "DGLMapSubgraphNID", "DGLGraphHasEdgeBetween",
    "DGLGraphHasEdgesBetween", "DGLGraphPredecessors", "DGLGraphSuccessors", "DGLGraphEdgeId",
    "DGLGraphEdgeIds", "DGLGraphFindEdges", "DGLGraphInEdges_1", "DGLGraphInEdges_2",
    "DGLGraphOutEdges_1", "DGLGraphOutEdges_2", "DGLGraphEdges", "DGLGraphInDegree",
    "DGLGraphInDegrees", "DGLGraphOutDegree", "DGLGraphOutDegrees", "DGLGraphVertexSubgraph",
    "DGLGraphEdgeSubgraph", "DGLDisjointUnion", "DGLDisjointPartitionByNum",
    "DGLDisjointPartitionBySizes", "DGLGraphLineGraph", "DGLGraphUniformSampling",
    "DGLGraphUniformSampling2", "DGLGraphUniformSampling4", "DGLGraphUniformSampling8",
    "DGLGraphUniformSampling16", "DGLGraphUniformSampling32", "DGLGraphUniformSampling64",
    "DGLGraphUniformSampling128", "DGLGraphGetAdj",
]
SCHED_API = ["DGLDegreeBucketing", "DGLDegreeBucketingForEdges",
             "DGLDegreeBucketingForRecvNodes", "DGLDegreeBucketingForFullGraph"]


class G(object):
    """Minimal restatement of the reference GraphIndex's CAPI use
    (python/dgl/graph_index.py:20-600), enough to drive the tests."""

    def __init__(self, handle=None, multigraph=False):
        self.h = handle if handle is not None else GI._CAPI_DGLGraphCreateMutable(multigraph)

    @classmethod
    def create(cls, src, dst, n, multigraph=False, readonly=False, eid=None):
        src = np.asarray(src, dtype=np.int64)
        eid = np.arange(len(src)) if eid is None else eid
        return cls(GI._CAPI_DGLGraphCreate(ids(src), ids(dst), ids(eid), multigraph, n,
                                           readonly))

    def __del__(self):
        if self.h:
            GI._CAPI_DGLGraphFree(self.h)

    def __getattr__(self, name):
        f = getattr(GI, "_CAPI_DGLGraph" + name)
        return lambda *a: f(self.h, *a)


def _mutable(n, edges, multigraph=True):
    g = G(multigraph=multigraph)
    g.AddVertices(n)
    for u, v in edges:
        g.AddEdge(u, v)
    return g


def test_all_reference_names_registered():
    names = set(C.global_names())
    missing = ["graph_index._CAPI_" + n for n in GRAPH_API
               if "graph_index._CAPI_" + n not in names]
    missing += ["runtime.degree_bucketing._CAPI_" + n for n in SCHED_API
                if "runtime.degree_bucketing._CAPI_" + n not in names]
    assert len(GRAPH_API) == 45 and not missing, missing


def test_edge_id_known_answers():
    # tests/graph_index/test_graph_index.py:6-70
    g = G(multigraph=True)
    assert g.IsMultigraph() == 1 and g.IsReadonly() == 0
    g.AddVertices(4)
    g.AddEdge(0, 1)
    assert g.EdgeId(0, 1).numpy().tolist() == [0]
    g.AddEdge(0, 1)
    assert g.EdgeId(0, 1).numpy().tolist() == [0, 1]
    g.AddEdges(ids([0, 1, 1, 2]), ids([2, 2, 2, 3]))
    _, _, eid = edge_triple(g.EdgeIds(ids([0, 0, 2, 1]), ids([2, 1, 3, 2])))
    assert eid.tolist() == [2, 0, 1, 5, 3, 4]
    src, dst, eid = edge_triple(g.FindEdges(ids([1, 3, 5])))
    assert src.tolist() == [0, 1, 2] and dst.tolist() == [1, 2, 3] and eid.tolist() == [1, 3, 5]
    _, _, eid = edge_triple(g.EdgeIds(ids([0]), ids([1, 2])))  # source broadcasting
    assert eid.tolist() == [0, 1, 2]
    _, _, eid = edge_triple(g.EdgeIds(ids([1, 0]), ids([2])))  # destination broadcasting
    assert eid.tolist() == [3, 4, 2]
    g.Clear()
    with pytest.raises(C.CAPIError):
        g.EdgeId(0, 1)
    g.AddVertices(4)
    g.AddEdge(0, 1)
    assert g.EdgeId(0, 1).numpy().tolist() == [0]
    assert g.NumVertices() == 4 and g.NumEdges() == 1


def test_predecessors_successors_known_answer():
    # tests/graph_index/test_graph_index.py:124-146: distinct, ascending
    g = _mutable(4, [(0, 1), (0, 1), (0, 2), (2, 0), (3, 0), (0, 0), (0, 0)])
    assert g.Predecessors(0, 1).numpy().tolist() == [0, 2, 3]
    assert g.Successors(0, 1).numpy().tolist() == [0, 1, 2]
    with pytest.raises(C.CAPIError):
        g.Predecessors(0, 0)  # radius must be >= 1


def test_create_from_edge_list_ids():
    # tests/graph_index/test_graph_index.py:148-152
    elist = [(2, 1), (1, 0), (2, 0), (3, 0), (0, 2)]
    src, dst = zip(*elist)
    for ro in (False, True):
        g = G.create(src, dst, 4, readonly=ro)
        assert g.IsReadonly() == int(ro)
        for i, (u, v) in enumerate(elist):
            assert g.EdgeId(u, v).numpy().tolist() == [i]


def _rand_graph(n, density, seed, shuffle=True):
    """Random simple graph; edges in (src, dst) order like the reference's
    scipy COO input, or shuffled."""
    rng = np.random.default_rng(seed)
    m = sp.random(n, n, density=density, format="coo", random_state=seed) != 0
    m = m.tocoo()
    perm = rng.permutation(m.nnz) if shuffle else np.lexsort((m.col, m.row))
    return m.row[perm].astype(np.int64), m.col[perm].astype(np.int64)


def _sort_by_eid(t):
    o = np.argsort(t[2], kind="stable")
    return tuple(x[o] for x in t)


def check_basics(g, ig, rng):
    # tests/compute/test_graph_index.py:40-106 (mutable vs immutable)
    n = g.NumVertices()
    assert n == ig.NumVertices() and g.NumEdges() == ig.NumEdges()
    for order in ("srcdst", "eid"):
        a, b = edge_triple(g.Edges(order)), edge_triple(ig.Edges(order))
        for x, y in zip(a, b):
            assert np.array_equal(x, y), order
    for i in range(n):
        assert g.HasVertex(i) == ig.HasVertex(i)
        assert np.array_equal(g.Predecessors(i, 1).numpy(), ig.Predecessors(i, 1).numpy())
        assert np.array_equal(g.Successors(i, 1).numpy(), ig.Successors(i, 1).numpy())
    v = rng.integers(0, n, 10)
    for fn in ("InEdges_2", "OutEdges_2"):
        a = _sort_by_eid(edge_triple(getattr(g, fn)(ids(v))))
        b = _sort_by_eid(edge_triple(getattr(ig, fn)(ids(v))))
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    assert np.array_equal(g.InDegrees(ids(v)).numpy(), ig.InDegrees(ids(v)).numpy())
    assert np.array_equal(g.OutDegrees(ids(v)).numpy(), ig.OutDegrees(ids(v)).numpy())
    for u in v:
        assert g.InDegree(int(u)) == ig.InDegree(int(u))
        assert g.OutDegree(int(u)) == ig.OutDegree(int(u))
        for w in v:
            if len(g.EdgeId(int(u), int(w)).numpy()) == 1:
                assert np.array_equal(g.EdgeId(int(u), int(w)).numpy(),
                                      ig.EdgeId(int(u), int(w)).numpy())
            assert g.HasEdgeBetween(int(u), int(w)) == ig.HasEdgeBetween(int(u), int(w))
    assert np.array_equal(edge_triple(g.EdgeIds(ids(v), ids(v)))[2],
                          edge_triple(ig.EdgeIds(ids(v), ids(v)))[2])
    assert np.array_equal(g.HasEdgesBetween(ids(v), ids(v)).numpy(),
                          ig.HasEdgesBetween(ids(v), ids(v)).numpy())


def _adj_dense(g):
    f = g.GetAdj(False, "coo")
    idx = f(0).numpy().reshape(2, -1)
    n = g.NumVertices()
    d = np.zeros((n, n), dtype=np.int64)
    np.add.at(d, (idx[0], idx[1]), 1)
    return d


@pytest.mark.parametrize("source", ["elist", "nx", "rand"])
def test_mutable_vs_immutable_basics(source):
    rng = np.random.default_rng(3)
    if source == "elist":
        src, dst, n = [2, 2, 3, 6, 10, 10], [3, 5, 0, 10, 3, 15], 16
    elif source == "nx":
        src, dst, n = [2, 2, 3, 1, 4, 4], [3, 5, 0, 0, 3, 5], 6
    else:
        n = 100
        src, dst = _rand_graph(n, 0.1, 7)
    g = G.create(src, dst, n)
    ig = G.create(src, dst, n, readonly=True)
    assert np.array_equal(_adj_dense(g), _adj_dense(ig))
    check_basics(g, ig, rng)


def test_node_subgraph_mutable_vs_immutable():
    # tests/compute/test_graph_index.py:112-135, tests/graph_index/test_subgraph.py
    n = 100
    # edge ids in (src, dst) order, as from the reference's scipy input: the
    # mutable subgraph numbers its edges in insertion order, the immutable one
    # in sorted-row order, and the two agree only then
    src, dst = _rand_graph(n, 0.1, 11, shuffle=False)
    g = G.create(src, dst, n)
    ig = G.create(src, dst, n, readonly=True)
    rng = np.random.default_rng(5)
    v1 = rng.integers(0, n, 20)
    v = np.unique(v1)
    sg, sig = g.VertexSubgraph(ids(v)), ig.VertexSubgraph(ids(v))
    subg, subig = G(sg(0)), G(sig(0))
    assert subg.IsReadonly() == 0 and subig.IsReadonly() == 1
    assert np.array_equal(sg(1).numpy(), v) and np.array_equal(sig(1).numpy(), v)
    check_basics(subg, subig, rng)
    assert np.array_equal(_adj_dense(subg), _adj_dense(subig))
    # every subgraph edge maps to a parent edge between the mapped endpoints
    s, d, e = edge_triple(subg.Edges(""))
    ind = sg(2).numpy()
    for a, b, x in zip(s, d, e):
        assert ind[x] in g.EdgeId(int(v[a]), int(v[b])).numpy()
    m1 = GI._CAPI_DGLMapSubgraphNID(sg(1), ids(v1[:10])).numpy()
    m2 = GI._CAPI_DGLMapSubgraphNID(sig(1), ids(v1[:10])).numpy()
    assert np.array_equal(m1, m2) and np.array_equal(v[m1], v1[:10])
    # unsorted parent ids take the hash-map path; absent ids map to -1
    par = ids([7, 3, 9])
    assert GI._CAPI_DGLMapSubgraphNID(par, ids([9, 4, 7])).numpy().tolist() == [2, -1, 0]


def test_edge_subgraph_known_answer():
    # tests/graph_index/test_subgraph.py:21-34
    g = _mutable(4, [(0, 1), (0, 1), (0, 2), (2, 3)], multigraph=False)
    sg = g.EdgeSubgraph(ids([3, 2]))
    subg = G(sg(0))
    nodes, edges = sg(1).numpy(), sg(2).numpy()
    assert nodes.tolist() == [2, 3, 0] and edges.tolist() == [3, 2]
    for s, d, e in zip(*edge_triple(subg.Edges(""))):
        assert edges[e] in g.EdgeId(int(nodes[s]), int(nodes[d])).numpy()
    ig = G.create([0], [1], 2, readonly=True)
    with pytest.raises(C.CAPIError, match="EdgeSubgraph"):
        ig.EdgeSubgraph(ids([0]))


def test_against_engine_graph_index():
    """The engine's DGLGraph index (dgl.graph_index.GraphIndex, a handle on
    the native index since r02) answers what a second native index built
    through the raw C-ABI client answers, on a random multigraph; and the
    engine's own CSR builder (the g-SpMM path) reproduces the index's CSR."""
    rng = np.random.default_rng(0)
    n, m = 300, 4000
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    gi = dgl.graph_index.GraphIndex(multigraph=True)
    gi.add_nodes(n)
    gi.add_edges(src, dst)
    g = G(multigraph=True)
    g.AddVertices(n)
    g.AddEdges(ids(src[:1000]), ids(dst[:1000]))
    g.AddEdges(ids(src[1000:]), ids(dst[1000:]))
    v = rng.integers(0, n, 50)
    for mine, ref in ((g.InEdges_2(ids(v)), gi.in_edges(v)),
                      (g.OutEdges_2(ids(v)), gi.out_edges(v))):
        for x, y in zip(edge_triple(mine), ref):
            assert np.array_equal(x, y.numpy())
    for x, y in zip(edge_triple(g.Edges("srcdst")), gi.edges("srcdst")):
        assert np.array_equal(x, y.numpy())
    assert np.array_equal(g.InDegrees(ids(np.arange(n))).numpy(), gi.in_degrees().numpy())
    assert np.array_equal(g.OutDegrees(ids(np.arange(n))).numpy(), gi.out_degrees().numpy())
    pu, pv = src[:40], dst[:40]
    mine = edge_triple(g.EdgeIds(ids(pu), ids(pv)))
    for x, y in zip(mine, gi.edge_ids(pu, pv)):
        assert np.array_equal(x, y.numpy())
    # GetAdj: the COO the reference's sparse product consumes, and the CSR
    # the engine's kernels use (same rows, same slot order)
    coo = g.GetAdj(False, "coo")
    idx = coo(0).numpy().reshape(2, -1)
    assert np.array_equal(idx[0], dst) and np.array_equal(idx[1], src)
    assert np.array_equal(coo(1).numpy(), np.arange(m))
    coo_t = g.GetAdj(True, "coo")(0).numpy().reshape(2, -1)
    assert np.array_equal(coo_t[0], src) and np.array_equal(coo_t[1], dst)
    csr = g.GetAdj(False, "csr")
    eng = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                           kernel.ORDER_EID, "cpu", schedule=False)
    assert np.array_equal(csr(0).numpy(), eng.indptr.numpy())
    assert np.array_equal(csr(1).numpy(), eng.indices.long().numpy())
    assert np.array_equal(csr(2).numpy(), eng.eid.numpy())
    # immutable: rows sorted by (dst, src), parallel edges in id order
    ig = G.create(src, dst, n, readonly=True, multigraph=True)
    icsr = ig.GetAdj(False, "csr")
    eng = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                           kernel.ORDER_COL, "cpu", schedule=False)
    assert np.array_equal(icsr(0).numpy(), eng.indptr.numpy())
    assert np.array_equal(icsr(1).numpy(), eng.indices.long().numpy())
    assert np.array_equal(icsr(2).numpy(), eng.eid.numpy())
    icoo = ig.GetAdj(False, "coo")(0).numpy().reshape(2, -1)
    assert np.array_equal(np.repeat(np.arange(n), np.diff(eng.indptr.numpy())), icoo[0])


def test_immutable_transposed_views():
    src, dst = _rand_graph(60, 0.08, 2)
    ig = G.create(src, dst, 60, readonly=True)
    out_csr = ig.GetAdj(True, "csr")
    indptr, indices = out_csr(0).numpy(), out_csr(1).numpy()
    rows = np.repeat(np.arange(60), np.diff(indptr))
    got = sorted(zip(rows.tolist(), indices.tolist()))
    assert got == sorted(zip(src.tolist(), dst.tolist()))
    for r in range(60):
        assert np.all(np.diff(indices[indptr[r]:indptr[r + 1]]) >= 0)


def test_mutation_errors_and_readonly():
    ig = G.create([0, 1], [1, 2], 3, readonly=True)
    for call in (lambda: ig.AddVertices(1), lambda: ig.AddEdge(0, 1),
                 lambda: ig.AddEdges(ids([0]), ids([1])), lambda: ig.Clear(),
                 lambda: ig.FindEdges(ids([0]))):
        with pytest.raises(C.CAPIError, match="isn't supported in ImmutableGraph"):
            call()
    g = _mutable(3, [(0, 1)])
    with pytest.raises(C.CAPIError, match="Invalid vertices"):
        g.AddEdge(0, 3)
    with pytest.raises(C.CAPIError, match="Invalid vertices"):
        g.AddEdges(ids([0, 1]), ids([2, 5]))
    assert g.NumEdges() == 1  # a rejected batch adds nothing
    with pytest.raises(C.CAPIError, match="invalid edge id"):
        g.FindEdges(ids([1]))
    with pytest.raises(C.CAPIError, match="Invalid id array"):
        g.InEdges_2(C.array(np.array([0], dtype=np.int32)))
    assert g.HasVertices(ids([0, 2, 3, -1])).numpy().tolist() == [1, 1, 0, 0]
    assert g.HasEdgesBetween(ids([0]), ids([1, 2])).numpy().tolist() == [1, 0]
    assert g.HasEdgeBetween(0, 7) == 0


def test_line_graph_known_answers():
    # tests/compute/test_transform.py:10-41 on nx.star_graph(5) (both directions)
    import networkx as nx
    star = nx.star_graph(5).to_directed()
    elist = sorted(star.edges())
    g = _mutable(6, elist, multigraph=False)
    lg = G(GI._CAPI_DGLGraphLineGraph(g.h, True))
    assert lg.NumVertices() == 10
    # brute force: edge i=(u,v) -> edge j=(v,w)
    exp = [(i, j) for i, (u, v) in enumerate(elist) for j, (x, w) in enumerate(elist) if x == v]
    s, d, _ = edge_triple(lg.Edges(""))
    assert list(zip(s.tolist(), d.tolist())) == exp
    nb = G(GI._CAPI_DGLGraphLineGraph(g.h, False))
    for i in range(1, 6):
        e1 = int(g.EdgeId(0, i).numpy()[0])
        e2 = int(g.EdgeId(i, 0).numpy()[0])
        assert nb.HasEdgeBetween(e1, e2) == 0 and nb.HasEdgeBetween(e2, e1) == 0
    assert nb.NumEdges() == len([1 for i, (u, v) in enumerate(elist)
                                 for j, (x, w) in enumerate(elist) if x == v and w != u])


def test_disjoint_union_and_partition():
    # python/dgl/graph_index.py:895-947 (batch / unbatch)
    g1 = _mutable(3, [(0, 1), (1, 2), (2, 0)])
    g2 = _mutable(2, [(1, 0)])
    g3 = _mutable(4, [(0, 3), (3, 3), (2, 1)])
    arr = (ctypes.c_void_p * 3)(g1.h.value, g2.h.value, g3.h.value)
    u = G(GI._CAPI_DGLDisjointUnion(ctypes.c_void_p(ctypes.addressof(arr)), 3))
    assert u.NumVertices() == 9 and u.NumEdges() == 7
    s, d, e = edge_triple(u.Edges(""))
    assert s.tolist() == [0, 1, 2, 4, 5, 8, 7] and d.tolist() == [1, 2, 0, 3, 8, 8, 6]
    parts = GI._CAPI_DGLDisjointPartitionBySizes(u.h, ids([3, 2, 4])).numpy()
    for h, ref in zip(parts, (g1, g2, g3)):
        p = G(ctypes.c_void_p(int(h)))
        for x, y in zip(edge_triple(p.Edges("")), edge_triple(ref.Edges(""))):
            assert np.array_equal(x, y)
    even = _mutable(4, [(0, 1), (3, 2)])
    halves = GI._CAPI_DGLDisjointPartitionByNum(even.h, 2).numpy()
    assert [G(ctypes.c_void_p(int(h))).NumEdges() for h in halves] == [1, 1]
    with pytest.raises(C.CAPIError, match="evenly divide"):
        GI._CAPI_DGLDisjointPartitionByNum(even.h, 3)
    cross = _mutable(4, [(0, 3)])
    with pytest.raises(C.CAPIError, match="crosses partitions"):
        GI._CAPI_DGLDisjointPartitionBySizes(cross.h, ids([2, 2]))
    ig = G.create([0], [1], 2, readonly=True)
    arr = (ctypes.c_void_p * 1)(ig.h.value)
    with pytest.raises(C.CAPIError, match="immutable"):
        GI._CAPI_DGLDisjointUnion(ctypes.c_void_p(ctypes.addressof(arr)), 1)


def _verify_sampled(ig, sub_h, verts, seed, fanout):
    # tests/compute/test_sampler.py:31-45
    sub = G(sub_h)
    child = int(np.searchsorted(verts, seed))
    assert verts[child] == seed
    cs, _, ce = edge_triple(sub.InEdges_2(ids([child])))
    assert len(np.unique(cs)) == len(cs) and np.all(np.diff(cs) > 0)
    ps, _, _ = edge_triple(ig.InEdges_2(ids([seed])))
    assert len(cs) == min(fanout, len(ps))
    assert set(verts[cs].tolist()) <= set(ps.tolist())


@pytest.mark.parametrize("fanout", [5, 100])
def test_neighbor_uniform_sampling(fanout):
    n = 100
    src, dst = _rand_graph(n, 0.1, 4)
    ig = G.create(src, dst, n, readonly=True)
    for seed in (0, 17, 63):
        f = GI._CAPI_DGLGraphUniformSampling(ig.h, ids([seed]), "in", 1, fanout, 1)
        verts, edges, layers = f(1).numpy(), f(2).numpy(), f(3).numpy()
        assert np.all(np.diff(verts) > 0) and seed in verts
        assert layers[np.searchsorted(verts, seed)] == 0
        assert len(edges) <= fanout and len(verts) <= fanout + 1
        _verify_sampled(ig, f(0), verts, seed, fanout)
        assert f(4).numpy().dtype == np.float32
    # several seed sets at once, padded to the API width (graph_index.py:1017-1027)
    seeds = [ids([3]), ids([5, 9]), ids(np.zeros(0, dtype=np.int64)),
             ids(np.zeros(0, dtype=np.int64))]
    f = GI._CAPI_DGLGraphUniformSampling4(ig.h, *seeds, "in", 2, fanout, 2)
    for i, sset in enumerate(([3], [5, 9])):
        verts = f(4 + i).numpy()
        for s in sset:
            assert s in verts
        layers = f(12 + i).numpy()
        assert layers.max() <= 2
        assert len(f(8 + i).numpy()) == G(f(i)).NumEdges()
    assert G(f(3)).NumVertices() == 0
    with pytest.raises(C.CAPIError, match="mutable"):
        g = G.create(src, dst, n)
        GI._CAPI_DGLGraphUniformSampling(g.h, ids([0]), "in", 1, 5, 1)


def test_full_fanout_sampling_is_the_neighbourhood():
    # tests/compute/test_sampler.py:8-29 (fan-out 100 on a 100-node graph)
    src, dst = _rand_graph(100, 0.1, 9)
    ig = G.create(src, dst, 100, readonly=True)
    for seed in range(0, 100, 7):
        f = GI._CAPI_DGLGraphUniformSampling(ig.h, ids([seed]), "in", 1, 100, 1)
        verts = f(1).numpy()
        ps, _, pe = edge_triple(ig.InEdges_2(ids([seed])))
        assert len(verts) == len(np.unique(np.append(ps, seed)))
        assert sorted(f(2).numpy().tolist()) == sorted(pe.tolist())


def _bucketing_reference(msg_ids, vids, recv):
    """Brute-force restatement of sched::DegreeBucketing's grouping
    (src/scheduler/scheduler.cc:13-93) in this build's canonical order."""
    by_node = {}
    for m, v in zip(msg_ids, vids):
        by_node.setdefault(int(v), []).append(int(m))
    degs, nids, nsec, mids, msec = [], [], [], [], []
    for d in sorted(set(len(x) for x in by_node.values())):
        nodes = sorted(v for v, x in by_node.items() if len(x) == d)
        degs.append(d)
        nsec.append(len(nodes))
        msec.append(d * len(nodes))
        nids.extend(nodes)
        for v in nodes:
            mids.extend(by_node[v])
    zero = sorted(set(int(r) for r in recv) - set(by_node))
    if zero:
        degs.append(0)
        nsec.append(len(zero))
        nids.extend(zero)
    return degs, nids, nsec, mids, msec


def test_degree_bucketing_capis():
    rng = np.random.default_rng(1)
    n, m = 40, 300
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n - 5, m)  # nodes n-5.. receive nothing
    g = G.create(src, dst, n, multigraph=True)
    recv = np.arange(n)

    def got(f):
        return [f(i).numpy().tolist() for i in range(5)]

    mids = rng.permutation(m)
    assert got(DB._CAPI_DGLDegreeBucketing(ids(mids), ids(dst), ids(recv))) == \
        list(_bucketing_reference(mids, dst, recv))
    assert got(DB._CAPI_DGLDegreeBucketingForEdges(ids(dst))) == \
        list(_bucketing_reference(np.arange(m), dst, dst))
    assert got(DB._CAPI_DGLDegreeBucketingForFullGraph(g.h)) == \
        list(_bucketing_reference(np.arange(m), dst, recv))
    v = np.array([3, 1, 38, 7])
    ins, ind, ine = edge_triple(g.InEdges_2(ids(v)))
    assert got(DB._CAPI_DGLDegreeBucketingForRecvNodes(g.h, ids(v))) == \
        list(_bucketing_reference(ine, ind, v))
    # the same schedule the engine's scheduler builds natively for UDF reduces
    degs, nids, nsec, _, _ = got(DB._CAPI_DGLDegreeBucketingForFullGraph(g.h))
    assert sum(nsec) == n and sorted(nids) == list(range(n))
