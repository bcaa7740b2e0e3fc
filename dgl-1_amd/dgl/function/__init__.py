"""DGL builtin functors (python/dgl/function/__init__.py)."""
# pylint: disable=redefined-builtin
from __future__ import absolute_import

from .message import *  # noqa: F401,F403
from .reducer import *  # noqa: F401,F403
from .base import *  # noqa: F401,F403
