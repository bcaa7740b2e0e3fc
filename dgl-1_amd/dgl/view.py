"""``g.nodes`` / ``g.edges`` / ``g.ndata`` / ``g.edata`` views (python/dgl/view.py)."""
from __future__ import absolute_import

from collections import namedtuple
from collections.abc import MutableMapping

import torch

from .base import ALL, DGLError, is_all

__all__ = ["NodeView", "EdgeView", "NodeDataView", "EdgeDataView"]

NodeSpace = namedtuple("NodeSpace", ["data"])
EdgeSpace = namedtuple("EdgeSpace", ["data"])


def _full_slice(s):
    if not (s.start is None and s.stop is None and s.step is None):
        raise DGLError('Currently only full slice ":" is supported')


class NodeView(object):
    """``g.nodes``: call for all node ids, index for a data view."""

    __slots__ = ["_graph"]

    def __init__(self, graph):
        self._graph = graph

    def __len__(self):
        return self._graph.number_of_nodes()

    def __getitem__(self, nodes):
        if isinstance(nodes, slice):
            _full_slice(nodes)
            nodes = ALL
        return NodeSpace(data=NodeDataView(self._graph, nodes))

    def __call__(self):
        return torch.arange(0, len(self), dtype=torch.int64)


class NodeDataView(MutableMapping):
    """Feature dict of a node selection."""

    __slots__ = ["_graph", "_nodes"]

    def __init__(self, graph, nodes):
        self._graph = graph
        self._nodes = nodes

    def __getitem__(self, key):
        return self._graph.get_n_repr(self._nodes)[key]

    def __setitem__(self, key, val):
        self._graph.set_n_repr({key: val}, self._nodes)

    def __delitem__(self, key):
        if not is_all(self._nodes):
            raise DGLError("Delete feature data is not supported on only a subset of nodes. "
                           "Please use `del G.ndata[key]` instead.")
        self._graph.pop_n_repr(key)

    def __len__(self):
        return len(self._graph._node_frame)

    def __iter__(self):
        return iter(self._graph._node_frame)

    def __repr__(self):
        data = self._graph.get_n_repr(self._nodes)
        return repr({k: data[k] for k in self._graph._node_frame})


class EdgeView(object):
    """``g.edges``: call for (u, v) / (u, v, eid), index for a data view."""

    __slots__ = ["_graph"]

    def __init__(self, graph):
        self._graph = graph

    def __len__(self):
        return self._graph.number_of_edges()

    def __getitem__(self, edges):
        if isinstance(edges, slice):
            _full_slice(edges)
            edges = ALL
        return EdgeSpace(data=EdgeDataView(self._graph, edges))

    def __call__(self, *args, **kwargs):
        return self._graph.all_edges(*args, **kwargs)


class EdgeDataView(MutableMapping):
    """Feature dict of an edge selection."""

    __slots__ = ["_graph", "_edges"]

    def __init__(self, graph, edges):
        self._graph = graph
        self._edges = edges

    def __getitem__(self, key):
        return self._graph.get_e_repr(self._edges)[key]

    def __setitem__(self, key, val):
        self._graph.set_e_repr({key: val}, self._edges)

    def __delitem__(self, key):
        if not is_all(self._edges):
            raise DGLError("Delete feature data is not supported on only a subset of edges. "
                           "Please use `del G.edata[key]` instead.")
        self._graph.pop_e_repr(key)

    def __len__(self):
        return len(self._graph._edge_frame)

    def __iter__(self):
        return iter(self._graph._edge_frame)

    def __repr__(self):
        data = self._graph.get_e_repr(self._edges)
        return repr({k: data[k] for k in self._graph._edge_frame})
