"""Neural-network modules (python/dgl/nn/__init__.py)."""
from __future__ import absolute_import

from .pytorch import *  # noqa: F401,F403
