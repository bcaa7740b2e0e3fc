"""DGLGraph: the user-facing graph + message-passing API.

Same public surface and semantics as python/dgl/graph.py (DGLGraph, 2939
lines in the reference) for graph construction, feature storage and the
message-passing entry points the hot path starts from:
update_all (graph.py:2398-2441), send_and_recv (2089-2196), pull (2198-2299),
push (2301-2396), send / recv (1926-2087), apply_nodes / apply_edges
(1800-1924), adjacency_matrix (2721-2742).

Each message-passing call is lowered by runtime.scheduler onto the g-SpMM
kernels of libdgl_hip.so; see that module for the lowering rules.
"""
from __future__ import absolute_import

import torch

from . import kernel, utils
from .base import ALL, DGLError, is_all
from .frame import Frame
from .graph_index import create_graph_index
from .runtime import scheduler
from .view import EdgeView, NodeView

__all__ = ["DGLGraph"]


class DGLGraph(object):
    """Directed graph with node/edge features and message passing.

    Parameters
    ----------
    graph_data : None, networkx graph, scipy sparse matrix, edge list, (u, v)
    node_frame, edge_frame : Frame, optional
    multigraph : bool
    readonly : bool
    """

    def __init__(self, graph_data=None, node_frame=None, edge_frame=None,
                 multigraph=False, readonly=False):
        self._graph = create_graph_index(graph_data, multigraph, readonly)
        n, m = self._graph.number_of_nodes(), self._graph.number_of_edges()
        self._node_frame = node_frame if node_frame is not None else Frame(n)
        self._edge_frame = edge_frame if edge_frame is not None else Frame(m)
        self._msg_frame = Frame(m)
        self._msg_pending = torch.zeros(m, dtype=torch.bool)
        self._message_func = None
        self._reduce_func = None
        self._apply_node_func = None
        self._apply_edge_func = None

    # -- structure -------------------------------------------------------------
    def add_nodes(self, num, data=None):
        """Add ``num`` isolated nodes (optionally with features)."""
        self._graph.add_nodes(num)
        if data is None:
            self._node_frame.add_rows(num)
        else:
            lo = self._node_frame.num_rows
            self._node_frame.add_rows(num)
            self._node_frame.update_rows(torch.arange(lo, lo + num), data)

    def add_edge(self, u, v, data=None):
        """Add one edge u -> v."""
        self.add_edges([u], [v], data)

    def add_edges(self, u, v, data=None):
        """Add edges u[i] -> v[i] (a scalar end broadcasts)."""
        before = self._graph.number_of_edges()
        self._graph.add_edges(u, v)
        num = self._graph.number_of_edges() - before
        self._edge_frame.add_rows(num)
        self._msg_frame.add_rows(num)
        self._msg_pending = torch.cat([self._msg_pending, torch.zeros(num, dtype=torch.bool)])
        if data is not None:
            self._edge_frame.update_rows(torch.arange(before, before + num), data)

    def clear(self):
        """Remove all nodes, edges and features."""
        self._graph.clear()
        self._node_frame = Frame(0)
        self._edge_frame = Frame(0)
        self._msg_frame = Frame(0)
        self._msg_pending = torch.zeros(0, dtype=torch.bool)

    def clear_cache(self):
        """Drop cached adjacencies (rebuilt on next use)."""
        self._graph._invalidate()

    def number_of_nodes(self):
        return self._graph.number_of_nodes()

    def __len__(self):
        return self.number_of_nodes()

    def number_of_edges(self):
        return self._graph.number_of_edges()

    @property
    def is_multigraph(self):
        return self._graph.is_multigraph()

    @property
    def is_readonly(self):
        return self._graph.is_readonly()

    def has_node(self, vid):
        return 0 <= int(vid) < self.number_of_nodes()

    def __contains__(self, vid):
        return self.has_node(vid)

    def has_nodes(self, vids):
        return self._graph.has_nodes(vids)

    def has_edge_between(self, u, v):
        return bool(self._graph.has_edges_between([u], [v])[0])

    def has_edges_between(self, u, v):
        return self._graph.has_edges_between(u, v)

    def predecessors(self, v):
        return self._graph.predecessors(v)

    def successors(self, v):
        return self._graph.successors(v)

    def edge_id(self, u, v, force_multi=False):
        _, _, eid = self._graph.edge_ids([u], [v])
        return eid if (force_multi or self.is_multigraph) else int(eid[0])

    def edge_ids(self, u, v, force_multi=False):
        src, dst, eid = self._graph.edge_ids(u, v)
        return (src, dst, eid) if (force_multi or self.is_multigraph) else eid

    def find_edges(self, eid):
        src, dst, _ = self._graph.find_edges(eid)
        return src, dst

    def in_edges(self, v, form="uv"):
        return self._form(self._graph.in_edges(v), form)

    def out_edges(self, v, form="uv"):
        return self._form(self._graph.out_edges(v), form)

    def all_edges(self, form="uv", order=None):
        return self._form(self._graph.edges(order), form)

    @staticmethod
    def _form(edges, form):
        src, dst, eid = edges
        if form == "all":
            return src, dst, eid
        if form == "uv":
            return src, dst
        if form == "eid":
            return eid
        raise DGLError("Invalid form: %s" % form)

    def in_degree(self, v):
        return int(self._graph.in_degrees([v])[0])

    def in_degrees(self, v=ALL):
        return self._graph.in_degrees(None if is_all(v) else v)

    def out_degree(self, v):
        return int(self._graph.out_degrees([v])[0])

    def out_degrees(self, v=ALL):
        return self._graph.out_degrees(None if is_all(v) else v)

    def to_networkx(self, node_attrs=None, edge_attrs=None):
        """networkx (Multi)DiGraph of the structure (graph.py:1094-1135): every
        edge carries its id as the 'id' attribute; node_attrs / edge_attrs
        name feature columns copied as per-node / per-edge tensor rows."""
        import networkx as nx
        nxg = nx.MultiDiGraph() if self.is_multigraph else nx.DiGraph()
        n = self.number_of_nodes()
        nxg.add_nodes_from(range(n))
        src, dst = self._graph.src().tolist(), self._graph.dst().tolist()
        for e, (u, v) in enumerate(zip(src, dst)):
            nxg.add_edge(u, v, id=e)
        for attr in node_attrs or ():
            col = self._node_frame[attr]
            for i in range(n):
                nxg.nodes[i][attr] = col[i]
        if edge_attrs:
            cols = {attr: self._edge_frame[attr] for attr in edge_attrs}
            for _, _, d in nxg.edges(data=True):
                for attr, col in cols.items():
                    d[attr] = col[d["id"]]
        return nxg

    def from_networkx(self, nx_graph, node_attrs=None, edge_attrs=None):
        """Replace the structure by a networkx graph (graph.py:1136-1232)."""
        self.clear()
        self._graph = create_graph_index(nx_graph, self._graph.is_multigraph(), False)
        self._reset_frames()
        import networkx as nx
        nxg = nx.convert_node_labels_to_integers(nx_graph, ordering="sorted")
        if not nxg.is_directed():
            nxg = nxg.to_directed()
        if node_attrs:
            for attr in node_attrs:
                vals = [nxg.nodes[i][attr] for i in range(nxg.number_of_nodes())]
                self._node_frame[attr] = _batch(vals)
        if edge_attrs:
            elist = list(nxg.edges(data=True))
            if elist and "id" in elist[0][2]:
                elist.sort(key=lambda e: e[2]["id"])
            for attr in edge_attrs:
                self._edge_frame[attr] = _batch([e[2][attr] for e in elist])

    def from_scipy_sparse_matrix(self, spmat):
        """Replace the structure by a scipy sparse matrix: u = row, v = col."""
        self.clear()
        self._graph = create_graph_index(spmat, self._graph.is_multigraph(), False)
        self._reset_frames()

    def _reset_frames(self):
        n, m = self.number_of_nodes(), self.number_of_edges()
        self._node_frame = Frame(n)
        self._edge_frame = Frame(m)
        self._msg_frame = Frame(m)
        self._msg_pending = torch.zeros(m, dtype=torch.bool)

    # -- features --------------------------------------------------------------
    def node_attr_schemes(self):
        return self._node_frame.schemes()

    def edge_attr_schemes(self):
        return self._edge_frame.schemes()

    def set_n_initializer(self, initializer, field=None):
        self._node_frame.set_initializer(initializer, field)

    def set_e_initializer(self, initializer, field=None):
        self._edge_frame.set_initializer(initializer, field)

    @property
    def nodes(self):
        return NodeView(self)

    @property
    def ndata(self):
        return self.nodes[:].data

    @property
    def edges(self):
        return EdgeView(self)

    @property
    def edata(self):
        return self.edges[:].data

    def set_n_repr(self, data, u=ALL, inplace=False):
        if not isinstance(data, dict):
            raise DGLError("Expect dictionary type for feature data. Got %s" % type(data))
        if is_all(u):
            for k, val in data.items():
                self._node_frame[k] = val
        else:
            u = utils.toindex(u)
            for k, val in data.items():
                if val.shape[0] != len(u):
                    raise DGLError("Expect number of features to match number of nodes "
                                   "(len(u)). Got %d and %d instead." % (val.shape[0], len(u)))
            self._node_frame.update_rows(u, data, inplace)

    def get_n_repr(self, u=ALL):
        if len(self._node_frame) == 0:
            return {}
        if is_all(u):
            return dict(self._node_frame.items())
        return self._node_frame.select_rows(utils.toindex(u))

    def pop_n_repr(self, key):
        return self._node_frame.pop(key)

    def set_e_repr(self, data, edges=ALL, inplace=False):
        if not isinstance(data, dict):
            raise DGLError("Expect dictionary type for feature data. Got %s" % type(data))
        if is_all(edges):
            for k, val in data.items():
                self._edge_frame[k] = val
            return
        eid = self._resolve_edges(edges)
        self._edge_frame.update_rows(eid, data, inplace)

    def get_e_repr(self, edges=ALL):
        if len(self._edge_frame) == 0:
            return {}
        if is_all(edges):
            return dict(self._edge_frame.items())
        return self._edge_frame.select_rows(self._resolve_edges(edges))

    def pop_e_repr(self, key):
        return self._edge_frame.pop(key)

    def _resolve_edges(self, edges):
        if isinstance(edges, tuple):
            _, _, eid = self._graph.edge_ids(edges[0], edges[1])
            return eid
        return utils.toindex(edges)

    def _edge_triplet(self, edges):
        if is_all(edges):
            return self._graph.edges()
        if isinstance(edges, tuple):
            return self._graph.edge_ids(edges[0], edges[1])
        return self._graph.find_edges(utils.toindex(edges))

    # -- registered functions --------------------------------------------------
    def register_message_func(self, func):
        self._message_func = func

    def register_reduce_func(self, func):
        self._reduce_func = func

    def register_apply_node_func(self, func):
        self._apply_node_func = func

    def register_apply_edge_func(self, func):
        self._apply_edge_func = func

    def _defaults(self, message_func=None, reduce_func=None, apply_node_func=None):
        mf = self._message_func if message_func == "default" else message_func
        rf = self._reduce_func if reduce_func == "default" else reduce_func
        af = self._apply_node_func if apply_node_func == "default" else apply_node_func
        return mf, rf, af

    # -- computation -----------------------------------------------------------
    def apply_nodes(self, func="default", v=ALL, inplace=False):
        """Update node features with a node UDF."""
        if func == "default":
            func = self._apply_node_func
        if func is None:
            return
        v = None if is_all(v) else utils.toindex(v)
        scheduler.schedule_apply_nodes(self, v, func, inplace)

    def apply_edges(self, func="default", edges=ALL, inplace=False):
        """Update edge features with an edge UDF."""
        if func == "default":
            func = self._apply_edge_func
        assert func is not None
        if is_all(edges):
            scheduler.schedule_apply_edges(self, None, None, None, func, inplace)
        else:
            u, v, eid = self._edge_triplet(edges)
            scheduler.schedule_apply_edges(self, u, v, eid, func, inplace)

    def send(self, edges=ALL, message_func="default"):
        """Compute messages on ``edges`` and store them for a later recv."""
        if message_func == "default":
            message_func = self._message_func
        u, v, eid = self._edge_triplet(edges)
        if len(eid) == 0:
            return
        scheduler.schedule_send(self, u, v, eid, message_func)

    def recv(self, v=ALL, reduce_func="default", apply_node_func="default", inplace=False):
        """Reduce pending messages at ``v``."""
        _, reduce_func, apply_node_func = self._defaults(None, reduce_func, apply_node_func)
        assert reduce_func is not None
        v = torch.arange(self.number_of_nodes()) if is_all(v) else utils.toindex(v)
        if len(v) == 0:
            return
        scheduler.schedule_recv(self, v, reduce_func, apply_node_func, inplace)

    def send_and_recv(self, edges, message_func="default", reduce_func="default",
                      apply_node_func="default", inplace=False):
        """Send along ``edges`` and reduce at their destinations."""
        mf, rf, af = self._defaults(message_func, reduce_func, apply_node_func)
        assert mf is not None
        assert rf is not None
        u, v, eid = self._edge_triplet(edges)
        if len(u) == 0:
            return
        scheduler.schedule_snr(self, u, v, eid, mf, rf, af, inplace)

    def pull(self, v, message_func="default", reduce_func="default",
             apply_node_func="default", inplace=False):
        """Pull messages from the predecessors of ``v``."""
        mf, rf, af = self._defaults(message_func, reduce_func, apply_node_func)
        assert mf is not None
        assert rf is not None
        v = utils.toindex(v)
        if len(v) == 0:
            return
        scheduler.schedule_pull(self, v, mf, rf, af, inplace)

    def push(self, u, message_func="default", reduce_func="default",
             apply_node_func="default", inplace=False):
        """Push messages from ``u`` to its successors."""
        mf, rf, af = self._defaults(message_func, reduce_func, apply_node_func)
        assert mf is not None
        assert rf is not None
        u = utils.toindex(u)
        if len(u) == 0:
            return
        scheduler.schedule_push(self, u, mf, rf, af, inplace)

    def update_all(self, message_func="default", reduce_func="default",
                   apply_node_func="default"):
        """Send along every edge and reduce at every node."""
        mf, rf, af = self._defaults(message_func, reduce_func, apply_node_func)
        assert mf is not None
        assert rf is not None
        scheduler.schedule_update_all(self, mf, rf, af)

    # -- sparse views ----------------------------------------------------------
    def _cached_view(self, key, build):
        # per (view, arguments, ctx); cleared by mutation and clear_cache(),
        # as the reference's adjacency / incidence caches (graph_index.py:537-662)
        cache = self._graph._cache
        if key not in cache:
            cache[key] = build()
        return cache[key]

    def adjacency_matrix(self, transpose=False, ctx=torch.device("cpu")):
        """Adjacency as a torch sparse COO tensor (rows = dst unless transpose)
        in the reference's nnz order (graph.py:2721-2742); cached per
        (transpose, ctx) until the graph changes."""
        ctx = torch.device(ctx)
        return self._cached_view(("adjmat", bool(transpose), str(ctx)),
                                 lambda: self._adjacency_matrix(transpose, ctx))

    def _adjacency_matrix(self, transpose, ctx):
        # the index's COO (graph_index.py:565-583 -> _CAPI_DGLGraphGetAdj):
        # edge-id order for a mutable graph, in-CSR order for an immutable one
        idx = self._graph.get_adj(transpose, "coo")[0]
        n, m = self.number_of_nodes(), self.number_of_edges()
        return torch.sparse_coo_tensor(idx.reshape(2, m), torch.ones(m), (n, n)).to(ctx)

    def incidence_matrix(self, typestr, ctx=torch.device("cpu")):
        """'in' / 'out' / 'both' incidence matrix (graph_index.py:587-662);
        cached per (type, ctx) until the graph changes."""
        if typestr not in ("in", "out", "both"):
            raise DGLError("Invalid incidence matrix type: %s" % typestr)
        ctx = torch.device(ctx)
        return self._cached_view(("incmat", typestr, str(ctx)),
                                 lambda: self._incidence_matrix(typestr, ctx))

    def _incidence_matrix(self, typestr, ctx):
        src, dst, eid = self._graph.edges()
        n, m = self.number_of_nodes(), self.number_of_edges()
        if typestr == "in":
            idx, val = torch.stack([dst, eid]), torch.ones(m)
        elif typestr == "out":
            idx, val = torch.stack([src, eid]), torch.ones(m)
        elif typestr == "both":
            keep = src != dst
            idx = torch.cat([torch.stack([src[keep], eid[keep]]),
                             torch.stack([dst[keep], eid[keep]])], 1)
            val = torch.cat([-torch.ones(int(keep.sum())), torch.ones(int(keep.sum()))])
        else:
            raise DGLError("Invalid incidence matrix type: %s" % typestr)
        return torch.sparse_coo_tensor(idx, val, (n, m)).to(ctx)

    def sparse_adjacency(self, ctx):
        """The engine's cached g-SpMM adjacency (kernel.SparseAdj) on ``ctx``."""
        return self._graph.adjacency(ctx)

    def __repr__(self):
        return ("DGLGraph(num_nodes={n}, num_edges={m},\n         ndata_schemes={ns}\n"
                "         edata_schemes={es})").format(
                    n=self.number_of_nodes(), m=self.number_of_edges(),
                    ns=self.node_attr_schemes(), es=self.edge_attr_schemes())


def _batch(vals):
    if isinstance(vals[0], torch.Tensor):
        return torch.stack(vals, 0)
    return torch.tensor(vals)



