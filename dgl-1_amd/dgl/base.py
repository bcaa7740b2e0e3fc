"""Base symbols shared by the package (mirrors python/dgl/base.py:1-17)."""
from __future__ import absolute_import

import warnings

__all__ = ["ALL", "is_all", "DGLError", "dgl_warning"]

# Special symbol selecting all nodes or edges (python/dgl/base.py:9).
ALL = "__ALL__"


class DGLError(Exception):
    """Error raised by the engine (python/dgl/_ffi/base.py:21-23)."""


def is_all(arg):
    """True if ``arg`` is the ALL symbol."""
    return isinstance(arg, str) and arg == ALL


def dgl_warning(msg):
    """Emit a user warning (python/dgl/base.py:15-17)."""
    warnings.warn(msg)
