"""The engine's DGLGraph runs on the native graph index (csrc/graph_index.cc).

Since r02 dgl.graph_index.GraphIndex holds a handle on the library's graph
object and answers every structural query with a graph_index._CAPI_* call, as
the reference's python/dgl/graph_index.py does against libdgl.so. These tests
pin that relationship: the handle DGLGraph holds is the one a raw C-ABI client
(the reference's calling convention, tests/capi_client.py) can query, the
reference's query semantics now reach the DGLGraph surface (distinct sorted
predecessors, graph.cc:148-178; immutable out-CSR edge order,
immutable_graph.cc:458-493), and the g-SpMM path still reads the same edges.
No GPU is used here.
"""
import ctypes
import pickle

import numpy as np
import pytest
import torch

from capi_client import GI, edge_triple, ids

import dgl
import dgl.function as fn
from dgl.base import DGLError
from oracle import oracle as O


def _graph(readonly=False, seed=0, n=200, m=3000):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    return dgl.DGLGraph((torch.from_numpy(src), torch.from_numpy(dst)), multigraph=True,
                        readonly=readonly), src, dst


@pytest.mark.parametrize("readonly", [False, True])
def test_dglgraph_handle_is_the_native_index(readonly):
    g, src, dst = _graph(readonly)
    h = g._graph._handle
    assert isinstance(h, int) and h
    hc = ctypes.c_void_p(h)
    # the raw client reads the very object DGLGraph mutates and queries
    assert GI._CAPI_DGLGraphNumVertices(hc) == g.number_of_nodes()
    assert GI._CAPI_DGLGraphNumEdges(hc) == len(src)
    assert bool(GI._CAPI_DGLGraphIsReadonly(hc)) == readonly
    v = np.arange(0, 200, 7)
    mine = g.in_edges(torch.from_numpy(v), form="all")
    raw = edge_triple(GI._CAPI_DGLGraphInEdges_2(hc, ids(v)))
    for x, y in zip(mine, raw):
        assert np.array_equal(x.numpy(), y)


def test_mutation_reaches_the_native_index():
    g = dgl.DGLGraph()
    g.add_nodes(5)
    g.add_edges([0, 1, 2], [1, 2, 3])
    g.add_edge(3, 4)
    h = ctypes.c_void_p(g._graph._handle)
    assert GI._CAPI_DGLGraphNumEdges(h) == 4
    s, d, e = edge_triple(GI._CAPI_DGLGraphEdges(h, "eid"))
    assert s.tolist() == [0, 1, 2, 3] and d.tolist() == [1, 2, 3, 4] and e.tolist() == [0, 1, 2, 3]
    # the engine's cached id-order arrays are dropped and refetched on mutation
    assert g._graph.src().tolist() == [0, 1, 2, 3]
    g.add_edge(4, 0)
    assert g._graph.src().tolist() == [0, 1, 2, 3, 4]
    g.clear()
    assert GI._CAPI_DGLGraphNumVertices(h) == 0 and g.number_of_edges() == 0


def test_reference_query_semantics_reach_dglgraph():
    # graph.cc:148-178: predecessors / successors are distinct and ascending
    g = dgl.DGLGraph(multigraph=True)
    g.add_nodes(4)
    g.add_edges([3, 1, 3, 0, 1], [2, 2, 2, 2, 0])
    assert g.predecessors(2).tolist() == [0, 1, 3]
    assert g.successors(1).tolist() == [0, 2]
    # in_edges keep insertion order (adjacency vectors, graph.cc:276-319)
    u, v, e = g.in_edges(2, form="all")
    assert u.tolist() == [3, 1, 3, 0] and e.tolist() == [0, 1, 2, 3]
    # all parallel edges of a pair, in id order
    assert g.edge_ids(3, 2)[2].tolist() == [0, 2]
    with pytest.raises(DGLError):
        g.edge_ids(2, 3)
    assert g.has_edges_between([3, 2], [2, 3]).tolist() == [1, 0]


def test_readonly_index_orders():
    # immutable_graph.cc:206-237: rows sorted by neighbour; edges() walks the
    # out-CSR; the engine's adjacency uses the in-CSR slot order
    g, src, dst = _graph(readonly=True, seed=3, n=50, m=400)
    u, v, e = g.all_edges(form="all")
    key = u.numpy() * 50 + v.numpy()
    assert np.all(np.diff(key) >= 0)
    assert np.array_equal(src[e.numpy()], u.numpy()) and np.array_equal(dst[e.numpy()], v.numpy())
    iu, iv, ie = g.in_edges(7, form="all")
    assert np.all(np.diff(iu.numpy()) >= 0)
    with pytest.raises(DGLError):
        g.add_nodes(1)
    # update_all on the readonly graph: the chain per row in (src, eid) order
    H = np.random.default_rng(1).standard_normal((50, 8)).astype(np.float32)
    g.ndata["h"] = torch.from_numpy(H)
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    order = np.lexsort((np.arange(len(src)), src, dst))
    ref = O.spmm_coo(50, dst[order], src[order], H)
    assert np.array_equal(g.ndata["o"].numpy(), ref)


def test_adjacency_matrix_is_the_index_coo():
    g, src, dst = _graph(seed=5, n=60, m=500)
    A = g.adjacency_matrix()
    idx = A._indices().numpy()
    assert np.array_equal(idx[0], dst) and np.array_equal(idx[1], src)
    At = g.adjacency_matrix(transpose=True)._indices().numpy()
    assert np.array_equal(At[0], src) and np.array_equal(At[1], dst)


@pytest.mark.parametrize("readonly", [False, True])
def test_pickle_round_trip(readonly):
    g, src, dst = _graph(readonly, seed=7, n=40, m=300)
    gi = pickle.loads(pickle.dumps(g._graph))
    assert gi._handle != g._graph._handle
    assert gi.is_readonly() == readonly and gi.number_of_edges() == 300
    assert np.array_equal(gi.src().numpy(), src) and np.array_equal(gi.dst().numpy(), dst)
    del g
    assert gi.in_degrees().sum().item() == 300


def test_bulk_construction_exports_without_permutation():
    # the engine's big-graph path: one AddEdges call, then the id-order edge
    # list read back once (zero-copy into torch) for the device CSR builder
    n, m = 100_000, 2_000_000
    rng = np.random.default_rng(11)
    src = torch.from_numpy(rng.integers(0, n, m))
    dst = torch.from_numpy(rng.integers(0, n, m))
    g = dgl.DGLGraph((src, dst))
    assert torch.equal(g._graph.src(), src) and torch.equal(g._graph.dst(), dst)
    assert torch.equal(g.in_degrees(), torch.bincount(dst, minlength=n))


@pytest.mark.parametrize("readonly", [False, True])
def test_parallel_csr_build_is_stable(readonly):
    """Past 2^20 edges the native CSR build places entries in parallel (rows in
    nnz-balanced ranges, input in chunks staged per range: O(n) reads); a
    row's slots must still come out in input (edge-id) order, or for the
    immutable index in (neighbour, edge id) order, with hub rows that straddle
    chunk boundaries."""
    n, m = 20_000, 3_000_000
    rng = np.random.default_rng(5)
    src = rng.integers(0, n, m)
    dst = np.where(rng.random(m) < 0.2, rng.integers(0, 3, m), rng.integers(0, n, m))
    g = dgl.DGLGraph((torch.from_numpy(src), torch.from_numpy(dst)), readonly=readonly)
    u, v, e = g.in_edges(g.nodes(), form="all")
    u, v, e = u.numpy(), v.numpy(), e.numpy()
    order = (np.lexsort((np.arange(m), src, dst)) if readonly
             else np.lexsort((np.arange(m), dst)))
    assert np.array_equal(v, dst[order]) and np.array_equal(u, src[order])
    assert np.array_equal(src[e], u) and np.array_equal(dst[e], v)
