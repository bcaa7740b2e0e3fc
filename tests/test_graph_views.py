"""Sparse views of a DGLGraph and their caches, after the reference's
tests/compute/test_graph.py (test_adjmat_cache :40-66, the known-answer
test_incmat :68-99, test_incmat_cache :101-128) and
tests/compute/test_graph_index.py:28-32 (mutable == immutable adjacency),
plus the engine's own cached g-SpMM adjacency: a mutation must invalidate it
(the next update_all sees the new edges, bit-exact against the oracle)."""
import math

import numpy as np
import pytest
import scipy.sparse as sp
import torch

import dgl
import dgl.function as fn
from oracle import oracle as O


def _dense(t):
    return t.to_dense().numpy()


def test_incmat_known_answer():
    g = dgl.DGLGraph()
    g.add_nodes(4)
    for u, v in ((0, 1), (0, 2), (0, 3), (2, 3), (1, 1)):
        g.add_edge(u, v)
    np.testing.assert_array_equal(_dense(g.incidence_matrix("in")),
                                  [[0, 0, 0, 0, 0], [1, 0, 0, 0, 1], [0, 1, 0, 0, 0],
                                   [0, 0, 1, 1, 0]])
    np.testing.assert_array_equal(_dense(g.incidence_matrix("out")),
                                  [[1, 1, 1, 0, 0], [0, 0, 0, 0, 1], [0, 0, 0, 1, 0],
                                   [0, 0, 0, 0, 0]])
    np.testing.assert_array_equal(_dense(g.incidence_matrix("both")),
                                  [[-1, -1, -1, 0, 0], [1, 0, 0, 0, 0], [0, 1, 0, -1, 0],
                                   [0, 0, 1, 1, 0]])
    with pytest.raises(dgl.DGLError):
        g.incidence_matrix("sideways")


def _random_graph(seed=0, n=1000):
    p = 10 * math.log(n) / n
    a = sp.random(n, n, p, random_state=seed, data_rvs=lambda k: np.ones(k))
    return dgl.DGLGraph(a), a


@pytest.mark.parametrize("view", ["adj", "inc"])
def test_view_cache(view):
    g, _ = _random_graph()
    if view == "adj":
        get = lambda other=False: g.adjacency_matrix(transpose=other)  # noqa: E731
    else:
        get = lambda other=False: g.incidence_matrix("both" if other else "in")  # noqa: E731
    m1 = get()
    assert get() is m1                  # cached
    assert get(True) is not m1          # different argument, different entry
    g.clear_cache()
    m2 = get()
    assert m2 is not m1                 # cleared by hand
    g.add_nodes(10)
    m3 = get()
    assert m3 is not m2                 # a mutation invalidates
    assert m3.shape[0] == g.number_of_nodes()


def test_adjacency_content_and_readonly_equal():
    g, a = _random_graph(seed=1, n=200)
    coo = a.tocoo()
    dense = np.zeros((200, 200))
    np.add.at(dense, (coo.col, coo.row), 1.0)  # rows = destinations
    np.testing.assert_array_equal(_dense(g.adjacency_matrix()), dense)
    np.testing.assert_array_equal(_dense(g.adjacency_matrix(transpose=True)), dense.T)
    ro = dgl.DGLGraph(a, readonly=True)
    np.testing.assert_array_equal(_dense(ro.adjacency_matrix()), dense)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_engine_adjacency_invalidated_by_mutation(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device(device)
    rng = np.random.default_rng(4)
    g = dgl.DGLGraph(multigraph=True)
    g.add_nodes(50)
    u, v = rng.integers(0, 50, 300), rng.integers(0, 50, 300)
    g.add_edges(u, v)
    H = rng.standard_normal((60, 8)).astype(np.float32)
    g.ndata["h"] = torch.from_numpy(H[:50]).to(dev)
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    first = g.sparse_adjacency(dev)
    assert g.sparse_adjacency(dev) is first
    np.testing.assert_array_equal(g.ndata["o"].cpu().numpy(), O.spmm_coo(50, v, u, H[:50]))
    # grow the graph: new nodes and edges, then message passing again
    g.add_nodes(10)
    u2, v2 = rng.integers(0, 60, 100), rng.integers(0, 60, 100)
    g.add_edges(u2, v2)
    g.ndata["h"] = torch.from_numpy(H).to(dev)
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    assert g.sparse_adjacency(dev) is not first
    uu, vv = np.concatenate([u, u2]), np.concatenate([v, v2])
    np.testing.assert_array_equal(g.ndata["o"].cpu().numpy(), O.spmm_coo(60, vv, uu, H))
