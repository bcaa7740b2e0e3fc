"""Builtin function base classes (python/dgl/function/base.py:1-38)."""
from __future__ import absolute_import

__all__ = ["BuiltinFunction", "BundledFunction"]


class BuiltinFunction(object):
    """Base class of declarative message / reduce functions."""

    @property
    def name(self):
        raise NotImplementedError


class BundledFunction(object):
    """Runs several functions and merges their output dicts (base.py:13-32)."""

    def __init__(self, fn_list):
        self.fn_list = list(fn_list)

    def __call__(self, *args, **kwargs):
        ret = {}
        for fn in self.fn_list:
            ret.update(fn(*args, **kwargs))
        return ret

    @property
    def name(self):
        return "bundled"
