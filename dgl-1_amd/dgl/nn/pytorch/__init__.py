"""PyTorch NN modules (python/dgl/nn/pytorch/__init__.py)."""
from __future__ import absolute_import

from .gcn import GraphConvolutionLayer  # noqa: F401
