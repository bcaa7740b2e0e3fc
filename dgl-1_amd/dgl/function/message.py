"""Builtin message functions (python/dgl/function/message.py:1-257).

Each builtin is both a declarative descriptor the scheduler lowers to a
g-SpMM kernel and a plain callable used when messages must be materialised
(UDF reduce, send/recv). ``copy_u`` / ``u_mul_e`` / ``copy_e`` are the later
DGL names of ``copy_src`` / ``src_mul_edge`` / ``copy_edge``.
"""
from __future__ import absolute_import

import operator

from .base import BuiltinFunction

__all__ = ["src_mul_edge", "copy_src", "copy_edge", "copy_u", "u_mul_e", "copy_e"]


class MessageFunction(BuiltinFunction):
    """Base builtin message function."""

    def __call__(self, edges):
        raise NotImplementedError

    def is_spmv_supported(self, g):
        """Whether the reference would specialise this into an SPMV."""
        raise NotImplementedError

    @property
    def use_edge_feature(self):
        raise NotImplementedError


def _edge_feat_is_scalar(g, field):
    """(E,) or (E, 1) edge feature (message.py:37-44)."""
    shape = tuple(g.edata[field].shape)
    return len(shape) == 1 or (len(shape) == 2 and shape[1] == 1)


def _broadcast_mul(sdata, edata):
    # align ranks by appending unit dims, as message.py:81-95 does
    rank = max(sdata.dim(), edata.dim())
    sdata = sdata.reshape(tuple(sdata.shape) + (1,) * (rank - sdata.dim()))
    edata = edata.reshape(tuple(edata.shape) + (1,) * (rank - edata.dim()))
    return sdata * edata


class SrcMulEdgeMessageFunction(MessageFunction):
    """m = h_src * w_edge."""

    kernel_msg = "u_mul_e"

    def __init__(self, mul_op, src_field, edge_field, out_field):
        self.mul_op = mul_op
        self.src_field = src_field
        self.edge_field = edge_field
        self.out_field = out_field

    def is_spmv_supported(self, g):
        return _edge_feat_is_scalar(g, self.edge_field)

    def __call__(self, edges):
        return {self.out_field: _broadcast_mul(edges.src[self.src_field],
                                               edges.data[self.edge_field])}

    @property
    def name(self):
        return "src_mul_edge"

    @property
    def use_edge_feature(self):
        return True


class CopySrcMessageFunction(MessageFunction):
    """m = h_src."""

    kernel_msg = "copy_u"

    def __init__(self, src_field, out_field):
        self.src_field = src_field
        self.out_field = out_field
        self.edge_field = None

    def is_spmv_supported(self, g):
        return True

    def __call__(self, edges):
        return {self.out_field: edges.src[self.src_field]}

    @property
    def name(self):
        return "copy_src"

    @property
    def use_edge_feature(self):
        return False


class CopyEdgeMessageFunction(MessageFunction):
    """m = w_edge."""

    kernel_msg = "copy_e"

    def __init__(self, edge_field=None, out_field=None):
        self.src_field = None
        self.edge_field = edge_field
        self.out_field = out_field

    def is_spmv_supported(self, g):
        return False  # the reference never specialises copy_edge (message.py:156-171)

    def __call__(self, edges):
        return {self.out_field: edges.data[self.edge_field]}

    @property
    def name(self):
        return "copy_edge"

    @property
    def use_edge_feature(self):
        return True


def src_mul_edge(src, edge, out):
    """Message = source node feature ``src`` times edge feature ``edge``."""
    return SrcMulEdgeMessageFunction(operator.mul, src, edge, out)


def copy_src(src, out):
    """Message = source node feature ``src``."""
    return CopySrcMessageFunction(src, out)


def copy_edge(edge, out):
    """Message = edge feature ``edge``."""
    return CopyEdgeMessageFunction(edge, out)


def copy_u(u, out):
    """Alias of :func:`copy_src`."""
    return copy_src(u, out)


def u_mul_e(lhs_field, rhs_field, out):
    """Alias of :func:`src_mul_edge`."""
    return src_mul_edge(lhs_field, rhs_field, out)


def copy_e(e, out):
    """Alias of :func:`copy_edge`."""
    return copy_edge(e, out)
