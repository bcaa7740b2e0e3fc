"""Graph structure index (edge lists + cached CSR adjacencies).

Mirrors the role of python/dgl/graph_index.py (GraphIndex, 1027 lines) for the
operations the message-passing path uses. The reference keeps the structure
in C++ (src/graph/graph.cc: adjacency lists; src/graph/immutable_graph.cc:
in/out CSR) behind ctypes handles. Here the canonical storage is the edge
list in edge-id order (src[e], dst[e]) — exactly the (row, col) pair list of
the reference's COO adjacency (graph.cc:509-524) — and every derived
structure is a CSR built by libdgl_hip.so and cached per device until the
next mutation (graph_index.py:537, 69-115).
"""
from __future__ import absolute_import

import numpy as np
import torch

from . import kernel
from .base import DGLError

__all__ = ["GraphIndex", "create_graph_index"]


def _as_i64(x):
    if isinstance(x, torch.Tensor):
        return x.detach().to(dtype=torch.int64, device="cpu").reshape(-1)
    if isinstance(x, slice):
        return torch.arange(x.start or 0, x.stop, x.step or 1, dtype=torch.int64)
    if isinstance(x, (int, np.integer)):
        return torch.tensor([int(x)], dtype=torch.int64)
    return torch.as_tensor(np.asarray(x, dtype=np.int64)).reshape(-1)


class GraphIndex(object):
    """Directed (multi)graph with integer node ids 0..N-1 and edge ids 0..E-1."""

    def __init__(self, multigraph=False, readonly=False):
        self._n = 0
        self._src_chunks = []
        self._dst_chunks = []
        self._src = torch.zeros(0, dtype=torch.int64)
        self._dst = torch.zeros(0, dtype=torch.int64)
        self._multigraph = bool(multigraph)
        self._readonly = bool(readonly)
        self._cache = {}

    # -- mutation ----------------------------------------------------------
    def _invalidate(self):
        self._cache = {}

    def _flush(self):
        if self._src_chunks:
            self._src = torch.cat([self._src] + self._src_chunks)
            self._dst = torch.cat([self._dst] + self._dst_chunks)
            self._src_chunks = []
            self._dst_chunks = []

    def add_nodes(self, num):
        if self._readonly:
            raise DGLError("readonly graph cannot be mutated")
        self._n += int(num)
        self._invalidate()

    def add_edges(self, u, v):
        if self._readonly:
            raise DGLError("readonly graph cannot be mutated")
        u = _as_i64(u)
        v = _as_i64(v)
        if u.numel() == 1 and v.numel() > 1:
            u = u.expand(v.numel())
        elif v.numel() == 1 and u.numel() > 1:
            v = v.expand(u.numel())
        if u.numel() != v.numel():
            raise DGLError("Invalid edges: %d sources vs %d destinations" % (u.numel(), v.numel()))
        if u.numel() == 0:
            return
        hi = max(int(u.max()), int(v.max()))
        if int(min(u.min(), v.min())) < 0 or hi >= self._n:
            raise DGLError("Invalid node id in edges (graph has %d nodes)" % self._n)
        self._src_chunks.append(u.clone())
        self._dst_chunks.append(v.clone())
        self._invalidate()

    def clear(self):
        self.__init__(self._multigraph, self._readonly)

    def is_multigraph(self):
        return self._multigraph

    def is_readonly(self):
        return self._readonly

    # -- sizes / raw arrays ------------------------------------------------
    def number_of_nodes(self):
        return self._n

    def number_of_edges(self):
        return self._src.numel() + sum(c.numel() for c in self._src_chunks)

    def src(self):
        self._flush()
        return self._src

    def dst(self):
        self._flush()
        return self._dst

    def edges(self, order=None):
        """(src, dst, eid) of all edges; order None/'eid' or 'srcdst'."""
        src, dst = self.src(), self.dst()
        eid = torch.arange(src.numel(), dtype=torch.int64)
        if order == "srcdst":
            key = src * max(self._n, 1) + dst
            perm = torch.sort(key, stable=True)[1]
            return src[perm], dst[perm], eid[perm]
        return src, dst, eid

    # -- cached CSRs --------------------------------------------------------
    def _slot_order(self):
        # ImmutableGraph keeps CSR sorted by (dst, src) (immutable_graph.cc:206-237);
        # the mutable graph's COO is in edge-id order (graph.cc:509-524).
        return kernel.ORDER_COL if self._readonly else kernel.ORDER_EID

    def _host_csr(self, kind):
        key = ("host", kind)
        if key not in self._cache:
            n = self._n
            if kind == "in":
                self._cache[key] = kernel.build_csr(n, n, self.dst(), self.src(),
                                                    kernel.ORDER_EID, "cpu", schedule=False)
            else:
                self._cache[key] = kernel.build_csr(n, n, self.src(), self.dst(),
                                                    kernel.ORDER_EID, "cpu", schedule=False)
        return self._cache[key]

    def adjacency(self, ctx):
        """SparseAdj of the whole graph on ``ctx``: rows = dst, cols = src
        (the reference's adjacency_matrix(transpose=False), graph_index.py:537-585)."""
        ctx = torch.device(ctx)
        if ctx.type == "cuda" and ctx.index is None:
            ctx = torch.device("cuda", torch.cuda.current_device())
        key = ("adj", str(ctx))
        if key not in self._cache:
            n = self._n
            src, dst, order = self.src(), self.dst(), self._slot_order()
            adj = kernel.from_coo(n, n, dst, src, order, ctx)
            self._cache[key] = adj
        return self._cache[key]

    def incidence_in(self, ctx):
        """Destination incidence (rows = dst, cols = eid) — the e2v reduction
        matrix of graph_index.py:629-635, as a CSR over edge ids."""
        ctx = torch.device(ctx)
        key = ("inc_in", str(ctx))
        if key not in self._cache:
            n, m = self._n, self.number_of_edges()
            eids = torch.arange(m, dtype=torch.int64)
            self._cache[key] = kernel.from_coo(n, m, self.dst(), eids, kernel.ORDER_EID, ctx)
        return self._cache[key]

    # -- queries ------------------------------------------------------------
    def has_nodes(self, vids):
        v = _as_i64(vids)
        return ((v >= 0) & (v < self._n)).to(torch.int64)

    def in_degrees(self, v=None):
        deg = self._host_csr("in").degrees()
        return deg if v is None else deg[_as_i64(v)]

    def out_degrees(self, v=None):
        deg = self._host_csr("out").degrees()
        return deg if v is None else deg[_as_i64(v)]

    def _gather_rows(self, kind, v):
        """Edges of rows ``v`` (query order; each row's edges in edge-id order)."""
        csr = self._host_csr(kind)
        v = _as_i64(v)
        if v.numel() and (int(v.min()) < 0 or int(v.max()) >= self._n):
            raise DGLError("Invalid node id")
        starts = csr.indptr[v]
        cnt = csr.indptr[v + 1] - starts
        rows = torch.repeat_interleave(v, cnt)
        base = torch.repeat_interleave(starts - torch.cumsum(cnt, 0) + cnt, cnt)
        slots = base + torch.arange(int(cnt.sum()), dtype=torch.int64)
        return rows, csr.indices[slots].long(), csr.eid[slots]

    def in_edges(self, v):
        """(src, dst, eid) of the in-edges of ``v``."""
        dst, src, eid = self._gather_rows("in", v)
        return src, dst, eid

    def out_edges(self, u):
        """(src, dst, eid) of the out-edges of ``u``."""
        src, dst, eid = self._gather_rows("out", u)
        return src, dst, eid

    def predecessors(self, v):
        return self.in_edges(v)[0]

    def successors(self, u):
        return self.out_edges(u)[1]

    def find_edges(self, eid):
        eid = _as_i64(eid)
        m = self.number_of_edges()
        if eid.numel() and (int(eid.min()) < 0 or int(eid.max()) >= m):
            raise DGLError("Invalid edge id")
        return self.src()[eid], self.dst()[eid], eid

    def _pairmap(self):
        """Edges sorted by (src, dst) key, stable in edge id: (keys, perm)."""
        key = ("pairmap",)
        if key not in self._cache:
            k = self.src() * max(self._n, 1) + self.dst()
            self._cache[key] = torch.sort(k, stable=True)
        return self._cache[key]

    def edge_ids(self, u, v):
        """All edges between each (u, v) pair, with broadcasting of a scalar
        end (graph.cc EdgeIds semantics); returns (src, dst, eid)."""
        u = _as_i64(u)
        v = _as_i64(v)
        if u.numel() == 1 and v.numel() > 1:
            u = u.expand(v.numel())
        elif v.numel() == 1 and u.numel() > 1:
            v = v.expand(u.numel())
        if u.numel() != v.numel():
            raise DGLError("Invalid edges: %d vs %d" % (u.numel(), v.numel()))
        if u.numel() == 0:
            e = torch.zeros(0, dtype=torch.int64)
            return e, e, e
        n = max(self._n, 1)
        sk, perm = self._pairmap()
        q = u * n + v
        lo = torch.searchsorted(sk, q, right=False)
        hi = torch.searchsorted(sk, q, right=True)
        cnt = hi - lo
        if bool((cnt == 0).any()):
            bad = int((cnt == 0).nonzero()[0])
            raise DGLError("Edge (%d, %d) does not exist" % (int(u[bad]), int(v[bad])))
        if not self._multigraph:
            cnt = torch.ones_like(cnt)
        base = torch.repeat_interleave(lo - torch.cumsum(cnt, 0) + cnt, cnt)
        slots = base + torch.arange(int(cnt.sum()), dtype=torch.int64)
        eid = perm[slots]
        return self.src()[eid], self.dst()[eid], eid

    def has_edges_between(self, u, v):
        u = _as_i64(u)
        v = _as_i64(v)
        n = max(self._n, 1)
        sk = self._pairmap()[0]
        q = u * n + v
        lo = torch.searchsorted(sk, q)
        hit = (lo < sk.numel()) & (sk[lo.clamp(max=max(sk.numel() - 1, 0))] == q) \
            if sk.numel() else torch.zeros_like(q, dtype=torch.bool)
        return hit.to(torch.int64)

    # -- pickling (graph_index.py:35-59): rebuildable from (n, multigraph, readonly, src, dst)
    def __getstate__(self):
        return (self._n, self._multigraph, self._readonly, self.src().numpy(), self.dst().numpy())

    def __setstate__(self, state):
        n, multi, ro, src, dst = state
        self.__init__(multi, False)
        self._n = n
        self._src = torch.as_tensor(src)
        self._dst = torch.as_tensor(dst)
        self._readonly = ro


def create_graph_index(graph_data=None, multigraph=False, readonly=False):
    """Build a GraphIndex from None, (src, dst), an edge list, a scipy sparse
    matrix, a networkx graph, or another GraphIndex (graph_index.py:950-998)."""
    if isinstance(graph_data, GraphIndex):
        return graph_data
    gi = GraphIndex(multigraph=multigraph, readonly=False)
    if graph_data is None:
        pass
    elif isinstance(graph_data, tuple) and len(graph_data) == 2:
        src, dst = _as_i64(graph_data[0]), _as_i64(graph_data[1])
        n = 0 if src.numel() == 0 else int(max(src.max(), dst.max())) + 1
        gi.add_nodes(n)
        gi.add_edges(src, dst)
    elif isinstance(graph_data, (list,)):
        arr = np.asarray(graph_data, dtype=np.int64).reshape(-1, 2)
        n = 0 if arr.size == 0 else int(arr.max()) + 1
        gi.add_nodes(n)
        gi.add_edges(arr[:, 0], arr[:, 1])
    elif hasattr(graph_data, "tocoo"):
        coo = graph_data.tocoo()
        gi.add_nodes(coo.shape[0])
        gi.add_edges(coo.row.astype(np.int64), coo.col.astype(np.int64))
    elif hasattr(graph_data, "is_directed") and hasattr(graph_data, "edges"):
        import networkx as nx
        nxg = nx.convert_node_labels_to_integers(graph_data, ordering="sorted")
        if not nxg.is_directed():
            nxg = nxg.to_directed()
        gi.add_nodes(nxg.number_of_nodes())
        elist = list(nxg.edges(data=True))
        if elist and "id" in elist[0][2]:
            elist.sort(key=lambda e: e[2]["id"])
        if elist:
            gi.add_edges([e[0] for e in elist], [e[1] for e in elist])
    else:
        raise DGLError("Unsupported graph data type: %s" % type(graph_data))
    gi._flush()
    gi._readonly = bool(readonly)
    return gi
