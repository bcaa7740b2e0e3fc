"""Builtin reduce functions (python/dgl/function/reducer.py:1-97) plus ``mean``."""
# pylint: disable=redefined-builtin
from __future__ import absolute_import

import torch

from .base import BuiltinFunction

__all__ = ["sum", "max", "mean"]


class ReduceFunction(BuiltinFunction):
    """Base builtin reduce function."""

    def __call__(self, nodes):
        raise NotImplementedError

    def is_spmv_supported(self):
        raise NotImplementedError


class SimpleReduceFunction(ReduceFunction):
    """Aggregate one message field into one node field."""

    def __init__(self, name, reduce_op, msg_field, out_field):
        self._name = name
        self.reduce_op = reduce_op
        self.msg_field = msg_field
        self.out_field = out_field

    def is_spmv_supported(self):
        """Only ``sum`` is an SPMV in the reference (reducer.py:40-43)."""
        return self._name == "sum"

    def __call__(self, nodes):
        return {self.out_field: self.reduce_op(nodes.mailbox[self.msg_field], 1)}

    @property
    def name(self):
        return self._name

    @property
    def kernel_reduce(self):
        return self._name


def _max(x, dim):
    return torch.max(x, dim)[0]


def sum(msg, out):
    """Reduce by sum: ``{out: mailbox[msg].sum(1)}``."""
    return SimpleReduceFunction("sum", torch.sum, msg, out)


def max(msg, out):
    """Reduce by element-wise max: ``{out: mailbox[msg].max(1)}``."""
    return SimpleReduceFunction("max", _max, msg, out)


def mean(msg, out):
    """Reduce by mean: ``{out: mailbox[msg].mean(1)}`` (north-star extension)."""
    return SimpleReduceFunction("mean", torch.mean, msg, out)
