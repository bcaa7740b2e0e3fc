"""Graph convolution modules on the engine's fused kernels.

The reference ships only GraphConvolutionLayer (python/dgl/nn/pytorch/gcn.py);
its GCN / GAT / R-GCN layers live in examples/pytorch/{gcn,gat,rgcn}. The
north star names ``nn.GraphConv`` / ``GATConv`` as the operator surface that
must drop in, so these modules package the example layers' computation (with
the later-DGL module names and arguments) on top of:

* GraphConv    : update_all(copy_src, sum) -> one g-SpMM (gcn_spmv.py:45-62)
* GATConv      : attention, dropout, per-head weighted sum and copy_edge
                 normaliser in one kernel (gat/train.py:61-96, kernel.gat_aggregate)
* SAGEConv     : update_all(copy_src, mean) -> g-SpMM mean
* RelGraphConv : typed-edge block-diagonal g-SpMM (rgcn/layers.py:121-132)
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import function as fn
from ... import kernel
from ...base import DGLError
from .linear import NodeLinear, sage_dense, bias_add

__all__ = ["GraphConv", "GATConv", "SAGEConv", "RelGraphConv"]


class GraphConv(nn.Module):
    """h' = act(D_dst^-1/2 A D_src^-1/2 h W + b) (norm='both'), 'right' = mean-style
    D_dst^-1, 'none' = plain sum. Weight is applied before aggregation when
    in_feats > out_feats (fewer bytes through the g-SpMM), after otherwise."""

    def __init__(self, in_feats, out_feats, norm="both", bias=True, activation=None):
        super(GraphConv, self).__init__()
        if norm not in ("both", "right", "none"):
            raise DGLError("Invalid norm %s" % norm)
        self.in_feats, self.out_feats, self.norm = in_feats, out_feats, norm
        self.weight = nn.Parameter(torch.Tensor(in_feats, out_feats))
        self.bias = nn.Parameter(torch.zeros(out_feats)) if bias else None
        self.activation = activation
        nn.init.xavier_uniform_(self.weight)

    def forward(self, g, feat):
        dev = feat.device
        if self.norm == "both":
            src_norm = g.out_degrees().float().clamp(min=1).pow(-0.5).to(dev).unsqueeze(1)
            feat = feat * src_norm
        if self.in_feats > self.out_feats:
            feat = feat @ self.weight
        g.ndata["_gc_h"] = feat
        g.update_all(fn.copy_src("_gc_h", "_gc_m"), fn.sum("_gc_m", "_gc_h"))
        rst = g.ndata.pop("_gc_h")
        if self.in_feats <= self.out_feats:
            rst = rst @ self.weight
        if self.norm != "none":
            deg = g.in_degrees().float().clamp(min=1).to(dev).unsqueeze(1)
            rst = rst * (deg.pow(-0.5) if self.norm == "both" else 1.0 / deg)
        if self.bias is not None:
            rst = bias_add(rst, self.bias)
        return self.activation(rst) if self.activation else rst


class GATConv(nn.Module):
    """Multi-head graph attention; returns (N, num_heads, out_feats)."""

    def __init__(self, in_feats, out_feats, num_heads, feat_drop=0., attn_drop=0.,
                 negative_slope=0.2, residual=False, activation=None):
        super(GATConv, self).__init__()
        self.num_heads, self.out_feats = num_heads, out_feats
        self.fc = nn.Linear(in_feats, num_heads * out_feats, bias=False)
        self.attn_l = nn.Parameter(torch.Tensor(1, num_heads, out_feats))
        self.attn_r = nn.Parameter(torch.Tensor(1, num_heads, out_feats))
        self.feat_drop = nn.Dropout(feat_drop) if feat_drop else None
        self.attn_drop = nn.Dropout(attn_drop) if attn_drop else None
        self.negative_slope = negative_slope
        self.res_fc = None
        if residual:
            self.res_fc = nn.Identity() if in_feats == num_heads * out_feats else \
                nn.Linear(in_feats, num_heads * out_feats, bias=False)
        self.activation = activation
        gain = nn.init.calculate_gain("relu")
        nn.init.xavier_normal_(self.fc.weight, gain=gain)
        nn.init.xavier_normal_(self.attn_l, gain=gain)
        nn.init.xavier_normal_(self.attn_r, gain=gain)

    def forward(self, g, feat):
        h = self.feat_drop(feat) if self.feat_drop is not None else feat
        ft = self.fc(h).view(-1, self.num_heads, self.out_feats)
        # (ft * attn).sum(-1) in the library's association (kernel.gat_logits):
        # with the same ft, gat_aggregate's blocked forward then recomputes
        # each source's logit from its gathered row instead of reading el
        el, er = kernel.gat_logits(ft, self.attn_l, self.attn_r)  # N x H x 1
        adj = g.sparse_adjacency(feat.device)
        # attention, its dropout, the weighted sum and the normaliser in one
        # kernel (kernel.gat_aggregate); the attention is kept, in CSR slot
        # order, only for the backward. Same per-element arithmetic as the
        # attention g-SDDMM + u_mul_e + copy_e g-SpMMs (bit for bit without
        # dropout); the dropout mask is the kernel's counter hash
        ft_sum, z = kernel.gat_aggregate(
            adj, ft, el, er, self.negative_slope, clamp=(-float("inf"), float("inf")),
            attn_drop=self.attn_drop.p if self.attn_drop is not None else 0.0,
            training=self.training)
        rst = ft_sum / z.clamp(min=1e-20)
        if self.res_fc is not None:
            rst = rst + self.res_fc(h).view(-1, self.num_heads, self.out_feats)
        return self.activation(rst) if self.activation else rst


class SAGEConv(nn.Module):
    """GraphSAGE with the mean aggregator: act(W_self h + W_neigh mean_{u->v} h_u)."""

    def __init__(self, in_feats, out_feats, bias=True, activation=None):
        super(SAGEConv, self).__init__()
        # NodeLinear: nn.Linear whose backward reductions over the node
        # dimension are chunked (split-K weight gradient, chunked bias sum)
        self.fc_self = NodeLinear(in_feats, out_feats, bias=bias)
        self.fc_neigh = NodeLinear(in_feats, out_feats, bias=False)
        self.activation = activation

    def forward(self, g, feat):
        def aggregate(x):
            g.ndata["_sage_h"] = x
            g.update_all(fn.copy_src("_sage_h", "_sage_m"), fn.mean("_sage_m", "_sage_n"))
            g.ndata.pop("_sage_h")
            return g.ndata.pop("_sage_n")
        # fc_neigh (no bias) commutes with the mean: the narrower side is
        # aggregated; both products and their sum fused (linear.sage_dense)
        return sage_dense(feat, aggregate, self.fc_self, self.fc_neigh, self.activation)


class RelGraphConv(nn.Module):
    """R-GCN layer with block-diagonal relation weights (num_bases blocks):
    h' = act(norm * sum_{e=(u->v)} blockdiag(W[etype_e]) h_u + h W_loop + b)."""

    def __init__(self, in_feat, out_feat, num_rels, num_bases, bias=True, activation=None,
                 self_loop=True, dropout=0.0):
        super(RelGraphConv, self).__init__()
        if in_feat % num_bases or out_feat % num_bases:
            raise DGLError("in/out features must be divisible by num_bases")
        self.weight = nn.Parameter(torch.Tensor(num_rels, num_bases, in_feat // num_bases,
                                                out_feat // num_bases))
        nn.init.xavier_uniform_(self.weight, gain=nn.init.calculate_gain("relu"))
        self.loop_weight = nn.Parameter(torch.Tensor(in_feat, out_feat)) if self_loop else None
        if self_loop:
            nn.init.xavier_uniform_(self.loop_weight, gain=nn.init.calculate_gain("relu"))
        self.bias = nn.Parameter(torch.zeros(out_feat)) if bias else None
        self.activation = activation
        self.dropout = nn.Dropout(dropout) if dropout else None

    def forward(self, g, feat, etype, norm=None):
        rst = kernel.typed_block_spmm(g.sparse_adjacency(feat.device), feat, self.weight, etype)
        if norm is not None:
            rst = rst * norm.reshape(-1, 1)
        if self.loop_weight is not None:
            loop = feat @ self.loop_weight
            rst = rst + (self.dropout(loop) if self.dropout is not None else loop)
        if self.bias is not None:
            rst = rst + self.bias
        return self.activation(rst) if self.activation else rst
