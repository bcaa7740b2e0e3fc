"""Tensor-backend plugin (python/dgl/backend/__init__.py:17-46, backend.py).

The reference selects its tensor framework with ``DGLBACKEND`` and routes the
hot path through three hooks of that plugin: ``get_preferred_sparse_format``,
``sparse_matrix`` and ``spmm`` (backend.py:77-148,558-572). This engine ships
a single backend, PyTorch-ROCm, whose ``spmm`` is the HIP g-SpMM.
"""
from __future__ import absolute_import

import os

from ..base import DGLError

_name = os.environ.get("DGLBACKEND", "pytorch").lower()
if _name != "pytorch":
    raise DGLError("Unsupported backend %s: this engine provides the pytorch (ROCm) backend "
                   "only" % _name)

from .pytorch import *  # noqa: E402,F401,F403


def load_backend(name="pytorch"):
    """Backend loader kept for API parity; only 'pytorch' exists."""
    if name != "pytorch":
        raise DGLError("Unsupported backend %s" % name)
