"""Feature initializers (python/dgl/init.py:8-61)."""
from __future__ import absolute_import

import torch

__all__ = ["base_initializer", "zero_initializer"]


def base_initializer(shape, dtype, ctx, id_range):  # pylint: disable=unused-argument
    """Signature of a feature initializer: (shape, dtype, ctx, id_range) -> tensor."""
    raise NotImplementedError


def zero_initializer(shape, dtype, ctx, id_range):  # pylint: disable=unused-argument
    """Zero feature initializer."""
    return torch.zeros(shape, dtype=dtype, device=ctx)
