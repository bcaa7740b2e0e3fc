"""Graph structure index: the native graph of libdgl_hip.so behind a handle.

Same shape as the reference's python/dgl/graph_index.py (GraphIndex, 1027
lines): the structure lives in the library (src/graph/graph.cc mutable
adjacency, immutable_graph.cc sorted CSRs there; csrc/graph_index.cc here) and
every structural query is one ``graph_index._CAPI_*`` call through the
PackedFunc registry, with the reference's names, arguments and returns
(graph_apis.cc). So the engine's DGLGraph and the reference's own Python layer
bound to this library read the same index.

What this class adds on the Python side are caches, as the reference's
GraphIndex caches its adjacency matrices (graph_index.py:537 cached_member):
the edge list in id order as torch tensors (fetched once from the index with
``_CAPI_DGLGraphEdges``, zero-copy through DLPack) and the engine's g-SpMM CSRs
built from it per device (kernel.from_coo); all are dropped on mutation.
"""
from __future__ import absolute_import

import numpy as np
import torch

from . import _ffi, kernel
from .base import DGLError

__all__ = ["GraphIndex", "create_graph_index"]

_CAPI = _ffi.CAPINamespace("graph_index")


def _as_i64(x):
    if isinstance(x, torch.Tensor):
        return x.detach().to(dtype=torch.int64, device="cpu").reshape(-1).contiguous()
    if isinstance(x, slice):
        return torch.arange(x.start or 0, x.stop, x.step or 1, dtype=torch.int64)
    if isinstance(x, (int, np.integer)):
        return torch.tensor([int(x)], dtype=torch.int64)
    return torch.as_tensor(np.asarray(x, dtype=np.int64)).reshape(-1).contiguous()


def _triple(f):
    """(src, dst, eid) of an EdgeArray packed function (graph_apis.cc:21-36)."""
    return f(0), f(1), f(2)


def _call(api, *args):
    """A graph_index._CAPI_* call whose library error surfaces as DGLError."""
    return getattr(_CAPI, api)(*args)


class GraphIndex(object):
    """Directed (multi)graph with integer node ids 0..N-1 and edge ids 0..E-1,
    stored in the library's native index (mutable, or immutable when
    ``readonly``)."""

    def __init__(self, multigraph=False, readonly=False, handle=None):
        # a readonly index is created with its edges (create_graph_index)
        if handle is None:
            if readonly:
                handle = _call("_CAPI_DGLGraphCreate", torch.zeros(0, dtype=torch.int64),
                               torch.zeros(0, dtype=torch.int64),
                               torch.zeros(0, dtype=torch.int64), int(multigraph), 0, 1)
            else:
                handle = _call("_CAPI_DGLGraphCreateMutable", int(multigraph))
        self._handle = handle
        self._multigraph = bool(multigraph)
        self._readonly = bool(readonly)
        self._cache = {}
        self._sync_sizes()

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h:
            try:
                _call("_CAPI_DGLGraphFree", ("handle", h))
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass
            self._handle = None

    def _h(self):
        return ("handle", self._handle)

    def _sync_sizes(self):
        # sizes mirrored on the Python side: they are read on every
        # message-passing call, the index is only asked after a mutation
        self._n = _call("_CAPI_DGLGraphNumVertices", self._h())
        self._m = _call("_CAPI_DGLGraphNumEdges", self._h())

    # -- mutation ----------------------------------------------------------
    def _invalidate(self):
        self._cache = {}

    def add_nodes(self, num):
        if self._readonly:
            raise DGLError("readonly graph cannot be mutated")
        _call("_CAPI_DGLGraphAddVertices", self._h(), int(num))
        self._sync_sizes()
        self._invalidate()

    def add_edges(self, u, v):
        if self._readonly:
            raise DGLError("readonly graph cannot be mutated")
        u = _as_i64(u)
        v = _as_i64(v)
        if u.numel() == 1 and v.numel() > 1:
            u = u.expand(v.numel()).contiguous()
        elif v.numel() == 1 and u.numel() > 1:
            v = v.expand(u.numel()).contiguous()
        if u.numel() != v.numel():
            raise DGLError("Invalid edges: %d sources vs %d destinations" % (u.numel(), v.numel()))
        if u.numel() == 0:
            return
        hi = max(int(u.max()), int(v.max()))
        if int(min(u.min(), v.min())) < 0 or hi >= self._n:
            raise DGLError("Invalid node id in edges (graph has %d nodes)" % self._n)
        _call("_CAPI_DGLGraphAddEdges", self._h(), u, v)
        self._sync_sizes()
        self._invalidate()

    def clear(self):
        if self._readonly:
            raise DGLError("readonly graph cannot be mutated")
        _call("_CAPI_DGLGraphClear", self._h())
        self._sync_sizes()
        self._invalidate()

    def is_multigraph(self):
        return self._multigraph

    def is_readonly(self):
        return self._readonly

    # -- sizes / raw arrays ------------------------------------------------
    def number_of_nodes(self):
        return self._n

    def number_of_edges(self):
        return self._m

    def _id_order(self):
        key = ("edges_id_order",)
        if key not in self._cache:
            src, dst, eid = _triple(_call("_CAPI_DGLGraphEdges", self._h(), "eid"))
            if not self._readonly:
                eid = None  # a mutable graph's ids are its positions
            self._cache[key] = (src, dst, eid)
        return self._cache[key]

    def src(self):
        """Source of every edge, in edge-id order (int64, host)."""
        return self._id_order()[0]

    def dst(self):
        """Destination of every edge, in edge-id order (int64, host)."""
        return self._id_order()[1]

    def edges(self, order=None):
        """(src, dst, eid) of all edges (graph_index.py:409-431): ``order`` None
        is the index's own order (edge ids for a mutable graph, the out-CSR for
        an immutable one), 'eid' sorts by edge id, 'srcdst' by (src, dst)."""
        if order == "eid" or (order is None and not self._readonly):
            src, dst, _ = self._id_order()
            return src, dst, torch.arange(self._m, dtype=torch.int64)
        return _triple(_call("_CAPI_DGLGraphEdges", self._h(), order or ""))

    # -- cached CSRs --------------------------------------------------------
    def _slot_order(self):
        # ImmutableGraph keeps CSR sorted by (dst, src) (immutable_graph.cc:206-237);
        # the mutable graph's COO is in edge-id order (graph.cc:509-524).
        return kernel.ORDER_COL if self._readonly else kernel.ORDER_EID

    def adjacency(self, ctx):
        """The engine's g-SpMM adjacency (kernel.SparseAdj) of the whole graph
        on ``ctx``: rows = dst, cols = src, slots in the index's adjacency
        order (the reference's adjacency_matrix(transpose=False),
        graph_index.py:537-585); built from the id-order edge list by the
        library's CSR builder and cached per device until the next mutation."""
        ctx = torch.device(ctx)
        if ctx.type == "cuda" and ctx.index is None:
            ctx = torch.device("cuda", torch.cuda.current_device())
        key = ("adj", str(ctx))
        if key not in self._cache:
            src, dst, _ = self._id_order()
            # the native index validated every edge when it was added
            self._cache[key] = kernel.from_coo(self._n, self._n, dst, src, self._slot_order(), ctx,
                                               validate=False)
        return self._cache[key]

    def incidence_in(self, ctx):
        """Destination incidence (rows = dst, cols = eid) — the e2v reduction
        matrix of graph_index.py:629-635, as a CSR over edge ids."""
        ctx = torch.device(ctx)
        key = ("inc_in", str(ctx))
        if key not in self._cache:
            n, m = self._n, self._m
            eids = torch.arange(m, dtype=torch.int64)
            self._cache[key] = kernel.from_coo(n, m, self.dst(), eids, kernel.ORDER_EID, ctx)
        return self._cache[key]

    def get_adj(self, transpose, fmt):
        """``_CAPI_DGLGraphGetAdj``: [idx(2E), eid] for 'coo', [indptr, indices,
        eid] for 'csr' (graph.cc:506-554, immutable_graph.cc:553-575)."""
        f = _call("_CAPI_DGLGraphGetAdj", self._h(), int(bool(transpose)), fmt)
        return [f(i) for i in range(2 if fmt == "coo" else 3)]

    # -- queries ------------------------------------------------------------
    def has_nodes(self, vids):
        return _call("_CAPI_DGLGraphHasVertices", self._h(), _as_i64(vids))

    def in_degrees(self, v=None):
        v = torch.arange(self._n, dtype=torch.int64) if v is None else _as_i64(v)
        return _call("_CAPI_DGLGraphInDegrees", self._h(), v)

    def out_degrees(self, v=None):
        v = torch.arange(self._n, dtype=torch.int64) if v is None else _as_i64(v)
        return _call("_CAPI_DGLGraphOutDegrees", self._h(), v)

    def in_edges(self, v):
        """(src, dst, eid) of the in-edges of ``v`` (query order; each node's
        edges in the index's adjacency order)."""
        return _triple(_call("_CAPI_DGLGraphInEdges_2", self._h(), _as_i64(v)))

    def out_edges(self, u):
        """(src, dst, eid) of the out-edges of ``u``."""
        return _triple(_call("_CAPI_DGLGraphOutEdges_2", self._h(), _as_i64(u)))

    def predecessors(self, v, radius=1):
        """Distinct predecessors of node ``v`` (graph.cc:148-162)."""
        return _call("_CAPI_DGLGraphPredecessors", self._h(), int(v), int(radius))

    def successors(self, u, radius=1):
        """Distinct successors of node ``u`` (graph.cc:164-178)."""
        return _call("_CAPI_DGLGraphSuccessors", self._h(), int(u), int(radius))

    def find_edges(self, eid):
        eid = _as_i64(eid)
        if self._readonly:  # the immutable index has no FindEdges (graph_apis.cc)
            if eid.numel() and (int(eid.min()) < 0 or int(eid.max()) >= self._m):
                raise DGLError("Invalid edge id")
            src, dst, _ = self._id_order()
            return src[eid], dst[eid], eid
        return _triple(_call("_CAPI_DGLGraphFindEdges", self._h(), eid))

    def edge_ids(self, u, v):
        """All edges between each (u, v) pair, with broadcasting of a scalar
        end (graph.cc:205-249 EdgeIds); returns (src, dst, eid)."""
        u = _as_i64(u)
        v = _as_i64(v)
        if u.numel() != v.numel() and u.numel() != 1 and v.numel() != 1:
            raise DGLError("Invalid edges: %d vs %d" % (u.numel(), v.numel()))
        if u.numel() == 0 or v.numel() == 0:
            e = torch.zeros(0, dtype=torch.int64)
            return e, e, e
        hit = self.has_edges_between(u, v)
        if not bool(hit.all()):
            bad = int((hit == 0).nonzero()[0])
            raise DGLError("Edge (%d, %d) does not exist"
                           % (int(u[bad if u.numel() > 1 else 0]),
                              int(v[bad if v.numel() > 1 else 0])))
        return _triple(_call("_CAPI_DGLGraphEdgeIds", self._h(), u, v))

    def has_edges_between(self, u, v):
        return _call("_CAPI_DGLGraphHasEdgesBetween", self._h(), _as_i64(u), _as_i64(v))

    # -- pickling (graph_index.py:35-59): rebuildable from (n, multigraph, readonly, src, dst)
    def __getstate__(self):
        return (self._n, self._multigraph, self._readonly, self.src().numpy().copy(),
                self.dst().numpy().copy())

    def __setstate__(self, state):
        n, multi, ro, src, dst = state
        g = _from_edges(n, torch.as_tensor(src), torch.as_tensor(dst), multi, ro)
        self.__dict__.update(g.__dict__)
        g._handle = None  # ownership moved to self


def _from_edges(n, src, dst, multigraph, readonly):
    src, dst = _as_i64(src), _as_i64(dst)
    if readonly:
        # immutable index: in/out CSRs sorted per row (immutable_graph.cc:260-281)
        if src.numel() and (int(min(src.min(), dst.min())) < 0
                            or int(max(src.max(), dst.max())) >= n):
            raise DGLError("Invalid node id in edges (graph has %d nodes)" % n)
        h = _call("_CAPI_DGLGraphCreate", src, dst, torch.arange(src.numel(), dtype=torch.int64),
                  int(multigraph), int(n), 1)
        return GraphIndex(multigraph, True, handle=h)
    gi = GraphIndex(multigraph, False)
    gi.add_nodes(n)
    gi.add_edges(src, dst)
    return gi


def create_graph_index(graph_data=None, multigraph=False, readonly=False):
    """Build a GraphIndex from None, (src, dst), an edge list, a scipy sparse
    matrix, a networkx graph, or another GraphIndex (graph_index.py:950-998)."""
    if isinstance(graph_data, GraphIndex):
        return graph_data
    if graph_data is None:
        return GraphIndex(multigraph=multigraph, readonly=readonly)
    if isinstance(graph_data, tuple) and len(graph_data) == 2:
        src, dst = _as_i64(graph_data[0]), _as_i64(graph_data[1])
        n = 0 if src.numel() == 0 else int(max(src.max(), dst.max())) + 1
    elif isinstance(graph_data, (list,)):
        arr = np.asarray(graph_data, dtype=np.int64).reshape(-1, 2)
        n = 0 if arr.size == 0 else int(arr.max()) + 1
        src, dst = arr[:, 0], arr[:, 1]
    elif hasattr(graph_data, "tocoo"):
        coo = graph_data.tocoo()
        n = coo.shape[0]
        src, dst = coo.row.astype(np.int64), coo.col.astype(np.int64)
    elif hasattr(graph_data, "is_directed") and hasattr(graph_data, "edges"):
        import networkx as nx
        nxg = nx.convert_node_labels_to_integers(graph_data, ordering="sorted")
        if not nxg.is_directed():
            nxg = nxg.to_directed()
        n = nxg.number_of_nodes()
        elist = list(nxg.edges(data=True))
        if elist and "id" in elist[0][2]:
            elist.sort(key=lambda e: e[2]["id"])
        src = [e[0] for e in elist]
        dst = [e[1] for e in elist]
    else:
        raise DGLError("Unsupported graph data type: %s" % type(graph_data))
    return _from_edges(n, src, dst, multigraph, readonly)
