"""PyTorch NN modules (python/dgl/nn/pytorch/__init__.py) plus the conv
modules the north star names (GraphConv, GATConv) and SAGEConv / RelGraphConv."""
from __future__ import absolute_import

from .gcn import GraphConvolutionLayer  # noqa: F401
from .conv import GATConv, GraphConv, RelGraphConv, SAGEConv  # noqa: F401
from .linear import NodeLinear, bias_add, dense_mm, node_epilogue, sage_dense  # noqa: F401
from .loss import weighted_cross_entropy  # noqa: F401
