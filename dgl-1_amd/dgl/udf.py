"""UDF batch views (python/dgl/udf.py:8-181): EdgeBatch and NodeBatch."""
from __future__ import absolute_import

__all__ = ["EdgeBatch", "NodeBatch", "LazyDict"]


class LazyDict(object):
    """Read-only mapping whose values are materialised on first access."""

    def __init__(self, fn, keys):
        self._fn = fn
        self._keys = list(keys)
        self._vals = {}

    def __getitem__(self, key):
        if key not in self._keys:
            raise KeyError(key)
        if key not in self._vals:
            self._vals[key] = self._fn(key)
        return self._vals[key]

    def __contains__(self, key):
        return key in self._keys

    def keys(self):
        return list(self._keys)

    def items(self):
        return [(k, self[k]) for k in self._keys]

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)


class EdgeBatch(object):
    """A batch of edges: ``src``, ``dst`` and ``data`` feature dicts."""

    def __init__(self, g, edges, src_data, edge_data, dst_data):
        self._g = g
        self._edges = edges
        self._src = src_data
        self._dst = dst_data
        self._data = edge_data

    @property
    def src(self):
        return self._src

    @property
    def dst(self):
        return self._dst

    @property
    def data(self):
        return self._data

    def edges(self):
        """(u, v, eid) tensors."""
        return self._edges

    def batch_size(self):
        return len(self._edges[2])

    def __len__(self):
        return self.batch_size()


class NodeBatch(object):
    """A batch of nodes: ``data`` features and, in reduce UDFs, ``mailbox``."""

    def __init__(self, g, nodes, data, msgs=None):
        self._g = g
        self._nodes = nodes
        self._data = data
        self._msgs = msgs

    @property
    def data(self):
        return self._data

    @property
    def mailbox(self):
        return self._msgs

    def nodes(self):
        return self._nodes

    def batch_size(self):
        return len(self._nodes)

    def __len__(self):
        return self.batch_size()
