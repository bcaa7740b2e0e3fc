"""Index helpers (the role of python/dgl/utils.py:Index / toindex, 90-115)."""
from __future__ import absolute_import

import numpy as np
import torch

from .base import DGLError, is_all

__all__ = ["toindex", "is_iterable", "relabel"]


def toindex(x):
    """Normalise node/edge ids to a 1-D int64 CPU tensor."""
    if isinstance(x, torch.Tensor):
        if x.dtype.is_floating_point:
            raise DGLError("Index data must be an integer tensor, got %s" % x.dtype)
        return x.detach().to(device="cpu", dtype=torch.int64).reshape(-1)
    if isinstance(x, slice):
        return torch.arange(x.start or 0, x.stop, x.step or 1, dtype=torch.int64)
    if isinstance(x, (int, np.integer)):
        return torch.tensor([int(x)], dtype=torch.int64)
    if is_all(x):
        raise DGLError("ALL must be resolved before toindex")
    arr = np.asarray(x)
    if arr.size and not np.issubdtype(arr.dtype, np.integer):
        raise DGLError("Index data must be integers")
    return torch.as_tensor(arr.astype(np.int64)).reshape(-1)


def is_iterable(obj):
    """True for lists/tuples (of builtins), not strings or tensors."""
    return isinstance(obj, (list, tuple))


def relabel(nodes_sorted_unique, ids):
    """Positions of ``ids`` inside the sorted unique id list
    (python/dgl/utils.py:321-361 build_relabel_map)."""
    return torch.searchsorted(nodes_sorted_unique, ids)
