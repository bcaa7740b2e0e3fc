"""Column storage for node / edge features.

Covers the semantics of python/dgl/frame.py the message-passing path relies
on: whole-column reads (READ_COL, executor.py:305-363), out-of-place column
replacement (WRITE_COL_/WRITE_DICT_, executor.py:871-923,1033-1080), row reads
and writes with initializer fill for new columns (FrameRef.update_rows /
update_column, frame.py:564-681; frame_like, frame.py:829-855).
"""
from __future__ import absolute_import

import torch

from .base import DGLError, dgl_warning
from .init import zero_initializer

__all__ = ["Frame"]


class Frame(object):
    """A dict of tensors sharing the first dimension ``num_rows``."""

    def __init__(self, num_rows=0):
        self._cols = {}
        self._num_rows = int(num_rows)
        self._inits = {}
        self._default_init = None
        self._warned = False

    # -- dict interface -----------------------------------------------------
    @property
    def num_rows(self):
        return self._num_rows

    def keys(self):
        return self._cols.keys()

    def values(self):
        return self._cols.values()

    def items(self):
        return self._cols.items()

    def __contains__(self, key):
        return key in self._cols

    def __len__(self):
        return len(self._cols)

    def __iter__(self):
        return iter(self._cols)

    def __getitem__(self, key):
        return self._cols[key]

    def __setitem__(self, key, val):
        if not isinstance(val, torch.Tensor):
            raise DGLError("Feature data must be a tensor, got %s" % type(val))
        if val.dim() == 0 or val.shape[0] != self._num_rows:
            raise DGLError("Expected feature of %d rows for '%s', got shape %s"
                           % (self._num_rows, key, tuple(val.shape)))
        self._cols[key] = val

    def __delitem__(self, key):
        del self._cols[key]

    def pop(self, key):
        return self._cols.pop(key)

    def clear(self):
        self._cols = {}

    def schemes(self):
        return {k: (tuple(v.shape[1:]), v.dtype) for k, v in self._cols.items()}

    # -- initializers (graph.py:1308-1402) ----------------------------------
    def set_initializer(self, init, field=None):
        if field is None:
            self._default_init = init
        else:
            self._inits[field] = init

    def get_initializer(self, field):
        init = self._inits.get(field, self._default_init)
        if init is None:
            if not self._warned:
                dgl_warning("Initializer is not set. Use zero initializer instead. To suppress "
                            "this warning, use `set_initializer` to explicitly specify which "
                            "initializer to use.")
                self._warned = True
            init = zero_initializer
        return init

    def _init_rows(self, key, shape, dtype, device, lo, hi):
        return self.get_initializer(key)((hi - lo,) + tuple(shape), dtype, device, slice(lo, hi))

    # -- row operations -----------------------------------------------------
    def add_rows(self, num):
        num = int(num)
        if num <= 0:
            return
        lo, hi = self._num_rows, self._num_rows + num
        for k, col in list(self._cols.items()):
            pad = self._init_rows(k, col.shape[1:], col.dtype, col.device, lo, hi)
            self._cols[k] = torch.cat([col, pad.to(col.device)], 0)
        self._num_rows = hi

    def select_rows(self, rows, keys=None):
        """dict of the given rows (``rows`` None = all rows)."""
        keys = self._cols.keys() if keys is None else keys
        out = {}
        for k in keys:
            col = self._cols[k]
            out[k] = col if rows is None else col.index_select(0, rows.to(col.device))
        return out

    def update_rows(self, rows, data, inplace=False):
        """Write ``data[k]`` at ``rows`` (``rows`` None = replace whole columns)."""
        for k, val in data.items():
            if rows is None:
                self[k] = val
                continue
            if k not in self._cols:
                full = self._init_rows(k, val.shape[1:], val.dtype, val.device, 0, self._num_rows)
                self._cols[k] = full.to(val.device)
            col = self._cols[k]
            idx = rows.to(col.device)
            if val.device != col.device:
                val = val.to(col.device)
            if val.dtype != col.dtype:
                val = val.to(col.dtype)
            if tuple(val.shape[1:]) != tuple(col.shape[1:]):
                raise DGLError("Cannot update column '%s' of shape %s with data of shape %s"
                               % (k, tuple(col.shape), tuple(val.shape)))
            if inplace:
                col.index_copy_(0, idx, val)
            else:
                self._cols[k] = col.index_copy(0, idx, val)
