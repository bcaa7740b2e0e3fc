"""IR variables (counterpart of python/dgl/runtime/ir/var.py).

A variable names a value flowing between executors. It is either concrete
(graph index, string, function, sparse matrix) or symbolic — a feature
tensor or feature dict that an executor fills in when the program runs.
"""
from __future__ import absolute_import

from .program import get_current_prog

__all__ = ["VarType", "Var", "new", "FEAT", "FEAT_DICT", "SPMAT", "IDX", "STR", "FUNC"]


class VarType(object):
    """Type codes (the reference's numbering)."""
    FEAT = 0        # feature tensor (symbolic)
    FEAT_DICT = 1   # dict / frame of feature tensors (symbolic)
    SPMAT = 2       # sparse matrix: a SparseAdj, or a callable device -> SparseAdj
    IDX = 3         # int64 index tensor, or None for "all"
    STR = 4
    FUNC = 5

    NAMES = ("Feat", "FeatDict", "SpMat", "Idx", "Str", "Func")


class Var(object):
    """A named IR value; ``data`` is None until bound or produced."""
    __slots__ = ("name", "typecode", "data")

    def __init__(self, name, typecode, data=None):
        self.name = name
        self.typecode = typecode
        self.data = data

    def typestr(self):
        return VarType.NAMES[self.typecode]

    def __str__(self):
        return '"%s"' % self.data if self.typecode == VarType.STR else self.name

    __repr__ = __str__


def new(typecode, data=None, name=None):
    """A fresh variable; unnamed ones are numbered per program (_z0, _z1, ...)."""
    if name is None:
        p = get_current_prog()
        if p is None:
            name = "_z"
        else:
            name = "_z%d" % p.varcount
            p.varcount += 1
    return Var(name, typecode, data)


def FEAT(data=None, name=None):
    return new(VarType.FEAT, data, name)


def FEAT_DICT(data=None, name=None):
    return new(VarType.FEAT_DICT, data, name)


def SPMAT(data=None, name=None):
    return new(VarType.SPMAT, data, name)


def IDX(data=None, name=None):
    return new(VarType.IDX, data, name)


def STR(data=None, name=None):
    return new(VarType.STR, data, name)


def FUNC(data=None, name=None):
    return new(VarType.FUNC, data, name)
