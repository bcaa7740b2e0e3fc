"""GraphConvolutionLayer (python/dgl/nn/pytorch/gcn.py:1-84): Linear node
update applied after ``update_all(copy_src, sum)`` (or ``send_and_recv`` on a
subset of edges), i.e. one g-SpMM plus the dense Linear on MFMA via torch."""
import torch.nn as nn

from ... import function as fn
from ...base import ALL, is_all


class NodeUpdateModule(nn.Module):
    """Linear + optional activation on ``node.data[node_field]``."""

    def __init__(self, node_field, in_feats, out_feats, activation=None):
        super(NodeUpdateModule, self).__init__()
        self.node_field = node_field
        self.linear = nn.Linear(in_feats, out_feats)
        self.activation = activation

    def forward(self, node):
        h = self.linear(node.data[self.node_field])
        if self.activation:
            h = self.activation(h)
        return {self.node_field: h}


class GraphConvolutionLayer(nn.Module):
    """One graph convolution (Kipf & Welling) over ``node_field``."""

    def __init__(self, node_field, in_feats, out_feats, activation, dropout=0):
        super(GraphConvolutionLayer, self).__init__()
        self.node_field = node_field
        self.dropout = nn.Dropout(p=dropout) if dropout else 0.
        self.update_func = NodeUpdateModule(node_field, in_feats, out_feats, activation)

    def forward(self, g, u=ALL, v=ALL):
        if self.dropout:
            field = self.node_field
            g.apply_nodes(lambda node: {field: self.dropout(node.data[field])})
        if is_all(u) and is_all(v):
            g.update_all(fn.copy_src(src=self.node_field, out="m"),
                         fn.sum(msg="m", out=self.node_field), self.update_func)
        else:
            g.send_and_recv((u, v), fn.copy_src(src=self.node_field, out="m"),
                            fn.sum(msg="m", out=self.node_field), self.update_func)
        return g
