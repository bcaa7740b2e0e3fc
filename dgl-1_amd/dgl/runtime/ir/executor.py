"""Executors of the message-passing IR (counterpart of
python/dgl/runtime/ir/executor.py).

Each executor is one step of a lowered API call: it reads its argument
variables when the program runs and binds its result variable. The
upper-case functions (``SPMV``, ``EDGE_UDF``, ``WRITE_ROW_`` ...) issue an
executor into the current program and return the result variable, as in
the reference; the scheduler (scheduler.py) builds every API call from them.

The kernel executors run the engine's HIP g-SpMM (dgl.kernel.gspmm) where
the reference ran torch.sparse.mm:

* SPMV            : A @ B, i.e. update_all(copy_src, REDUCE) over the
                    adjacency (SPMVExecutor, executor.py:452-473); this
                    engine also takes max / mean in the same kernel
* SPMV_WITH_DATA  : A(edge data) @ B, i.e. src_mul_edge (executor.py:535-566)
* SPMV_E2V        : incidence @ messages, a builtin reducer over materialised
                    messages (the reference's e2v SPMV, spmv.py:229-292)
* DEGREE_BUCKETING: a reduce UDF over the mailbox, bucketed by in-degree
                    (degree_bucketing.py:13-84; the reference issues one
                    NODE_UDF per bucket plus MERGE_ROW, here one executor
                    runs the native bucketing schedule)

Mutating executors end in ``_`` and return no variable.
"""
from __future__ import absolute_import

import torch

from ... import kernel
from . import var
from .program import get_current_prog
from .registry import IR_REGISTRY
from .var import VarType

__all__ = ["OpCode", "Executor",
           "NODE_UDF", "EDGE_UDF", "SPMV", "SPMV_WITH_DATA", "SPMV_E2V",
           "DEGREE_BUCKETING", "READ", "READ_COL", "READ_ROW", "MERGE_ROW",
           "UPDATE_DICT", "NEW_DICT", "WRITE_", "WRITE_COL_", "WRITE_ROW_",
           "WRITE_DICT_", "APPEND_ROW_", "WRITE_ROW_INPLACE_", "CLEAR_FRAME_", "CALL_"]


class OpCode(object):
    """Opcodes (the reference's numbering; 10-11 and 28 are this engine's)."""
    NODE_UDF = 0
    EDGE_UDF = 1
    SPMV = 2
    SPMV_WITH_DATA = 3
    READ = 4
    READ_COL = 5
    READ_ROW = 6
    MERGE_ROW = 7
    UPDATE_DICT = 8
    NEW_DICT = 9
    SPMV_E2V = 10
    DEGREE_BUCKETING = 11
    # mutating (no result)
    WRITE_ = 21
    WRITE_COL_ = 22
    WRITE_ROW_ = 23
    WRITE_DICT_ = 24
    APPEND_ROW_ = 25
    WRITE_ROW_INPLACE_ = 26
    CLEAR_FRAME_ = 27
    CALL_ = 28


class Executor(object):
    """One IR step. ``args`` are Vars (None for an omitted optional one)."""
    OPCODE = None

    def __init__(self, *args, **kw):
        self.args = args
        self.ret = kw.get("ret")

    def opcode(self):
        return self.OPCODE

    def arg_vars(self):
        return list(self.args)

    def ret_var(self):
        return self.ret

    def _vals(self):
        return [None if a is None else a.data for a in self.args]

    def run(self):
        out = self.compute(*self._vals())
        if self.ret is not None:
            self.ret.data = out

    def compute(self, *vals):
        raise NotImplementedError


def _adj(spmat, like):
    """A SPMAT variable's matrix on the device of ``like``."""
    return spmat(like.device) if callable(spmat) else spmat


def _as_dict(fd):
    return fd if isinstance(fd, dict) else {k: fd[k] for k in fd.keys()}


class NodeUDFExecutor(Executor):
    OPCODE = OpCode.NODE_UDF

    def compute(self, fn, fdnode, fdmail=None):
        return fn(fdnode) if fdmail is None else fn(fdnode, fdmail)


class EdgeUDFExecutor(Executor):
    OPCODE = OpCode.EDGE_UDF

    def compute(self, fn, fdsrc, fdedge, fddst):
        return fn(fdsrc, fdedge, fddst)


class SPMVExecutor(Executor):
    """ret = REDUCE over in-edges of B[src] (copy_src; reduce a STR var)."""
    OPCODE = OpCode.SPMV

    def compute(self, spmat, B, reduce):
        return kernel.gspmm(_adj(spmat, B), "copy_u", reduce, B)


class SPMVWithDataExecutor(Executor):
    """ret = REDUCE over in-edges of A_data[e] * B[src] (src_mul_edge)."""
    OPCODE = OpCode.SPMV_WITH_DATA

    def compute(self, spmat, A_data, B, reduce):
        return kernel.gspmm(_adj(spmat, B), "u_mul_e", reduce, B, A_data)


class SPMVE2VExecutor(Executor):
    """ret = REDUCE over each receiver's materialised messages (copy_e over
    the incidence matrix); messages that are not float32 go to ``fallback``
    (degree bucketing of the builtin reducer)."""
    OPCODE = OpCode.SPMV_E2V

    def compute(self, spmat, msg, reduce, fallback=None):
        if msg.dtype != torch.float32 and fallback is not None:
            return fallback(msg)
        return kernel.gspmm(_adj(spmat, msg), "copy_e", reduce, None, msg)


class DegreeBucketingExecutor(Executor):
    """ret = dict of a reduce UDF's outputs for every receiver (bucketed)."""
    OPCODE = OpCode.DEGREE_BUCKETING

    def compute(self, fn, fdmail):
        return fn(fdmail)


class ReadExecutor(Executor):
    OPCODE = OpCode.READ

    def compute(self, fd, row, col):
        return fd.select_rows(row)[col] if hasattr(fd, "select_rows") else fd[col][row]


class ReadColExecutor(Executor):
    OPCODE = OpCode.READ_COL

    def compute(self, fd, col):
        return fd[col]


class ReadRowExecutor(Executor):
    OPCODE = OpCode.READ_ROW

    def compute(self, fd, row):
        if hasattr(fd, "select_rows"):
            return fd.select_rows(row)
        return {k: v if row is None else v.index_select(0, row.to(v.device))
                for k, v in fd.items()}


class MergeRowExecutor(Executor):
    """Rows of several dicts (each with its index vector) merged into one
    dict ordered by ascending index (the reference's bucket merge)."""
    OPCODE = OpCode.MERGE_ROW

    def compute(self, idx_list, fd_list):
        order = torch.argsort(torch.cat([torch.as_tensor(i) for i in idx_list]), stable=True)
        keys = fd_list[0].keys() if fd_list else []
        out = {}
        for k in keys:
            col = torch.cat([fd[k] for fd in fd_list], 0)
            out[k] = col.index_select(0, order.to(col.device))
        return out


class UpdateDictExecutor(Executor):
    OPCODE = OpCode.UPDATE_DICT

    def compute(self, fd1, fd2):
        out = dict(_as_dict(fd1))
        out.update(_as_dict(fd2))
        return out


class NewDictExecutor(Executor):
    OPCODE = OpCode.NEW_DICT

    def compute(self):
        return {}


class WriteExecutor(Executor):
    OPCODE = OpCode.WRITE_

    def compute(self, fd, row, col, val):
        fd.update_rows(row, {col: val})


class WriteColExecutor(Executor):
    OPCODE = OpCode.WRITE_COL_

    def compute(self, fd, col, val):
        fd[col] = val


class WriteRowExecutor(Executor):
    OPCODE = OpCode.WRITE_ROW_

    def compute(self, fd, row, val):
        fd.update_rows(row, val, False)


class WriteRowInplaceExecutor(Executor):
    OPCODE = OpCode.WRITE_ROW_INPLACE_

    def compute(self, fd, row, val):
        fd.update_rows(row, val, True)


class WriteDictExecutor(Executor):
    """Replace whole columns (update_all's write-back)."""
    OPCODE = OpCode.WRITE_DICT_

    def compute(self, fd, val):
        fd.update_rows(None, val)


class AppendRowExecutor(Executor):
    OPCODE = OpCode.APPEND_ROW_

    def compute(self, fd, val):
        n = next(iter(val.values())).shape[0] if val else 0
        lo = fd.num_rows
        fd.add_rows(n)
        fd.update_rows(torch.arange(lo, lo + n), val)


class ClearFrameExecutor(Executor):
    OPCODE = OpCode.CLEAR_FRAME_

    def compute(self, fd):
        fd.clear()


class CallExecutor(Executor):
    """A side effect of the API call at its place in the program (e.g.
    send/recv's pending-message bookkeeping)."""
    OPCODE = OpCode.CALL_

    def compute(self, fn):
        fn()


def _register(name, cls, args_type, ret_type):
    IR_REGISTRY[cls.OPCODE] = {"name": name, "args_type": args_type, "ret_type": ret_type,
                               "executor_cls": cls}


T = VarType
_register("NODE_UDF", NodeUDFExecutor, [T.FUNC, T.FEAT_DICT, T.FEAT_DICT], T.FEAT_DICT)
_register("EDGE_UDF", EdgeUDFExecutor, [T.FUNC, T.FEAT_DICT, T.FEAT_DICT, T.FEAT_DICT],
          T.FEAT_DICT)
_register("SPMV", SPMVExecutor, [T.SPMAT, T.FEAT, T.STR], T.FEAT)
_register("SPMV_WITH_DATA", SPMVWithDataExecutor, [T.SPMAT, T.FEAT, T.FEAT, T.STR], T.FEAT)
_register("SPMV_E2V", SPMVE2VExecutor, [T.SPMAT, T.FEAT, T.STR, T.FUNC], T.FEAT)
_register("DEGREE_BUCKETING", DegreeBucketingExecutor, [T.FUNC, T.FEAT_DICT], T.FEAT_DICT)
_register("READ", ReadExecutor, [T.FEAT_DICT, T.IDX, T.STR], T.FEAT)
_register("READ_COL", ReadColExecutor, [T.FEAT_DICT, T.STR], T.FEAT)
_register("READ_ROW", ReadRowExecutor, [T.FEAT_DICT, T.IDX], T.FEAT_DICT)
_register("MERGE_ROW", MergeRowExecutor, [T.IDX, T.FEAT_DICT], T.FEAT_DICT)
_register("UPDATE_DICT", UpdateDictExecutor, [T.FEAT_DICT, T.FEAT_DICT], T.FEAT_DICT)
_register("NEW_DICT", NewDictExecutor, [], T.FEAT_DICT)
_register("WRITE_", WriteExecutor, [T.FEAT_DICT, T.IDX, T.STR, T.FEAT], None)
_register("WRITE_COL_", WriteColExecutor, [T.FEAT_DICT, T.STR, T.FEAT], None)
_register("WRITE_ROW_", WriteRowExecutor, [T.FEAT_DICT, T.IDX, T.FEAT_DICT], None)
_register("WRITE_DICT_", WriteDictExecutor, [T.FEAT_DICT, T.FEAT_DICT], None)
_register("APPEND_ROW_", AppendRowExecutor, [T.FEAT_DICT, T.FEAT_DICT], None)
_register("WRITE_ROW_INPLACE_", WriteRowInplaceExecutor, [T.FEAT_DICT, T.IDX, T.FEAT_DICT],
          None)
_register("CLEAR_FRAME_", ClearFrameExecutor, [T.FEAT_DICT], None)
_register("CALL_", CallExecutor, [T.FUNC], None)
del T


def _issue(cls, args, ret=True):
    """Issue ``cls(*args)`` into the current program; the result variable."""
    p = get_current_prog()
    if p is None:
        raise RuntimeError("no current IR program: issue executors inside ir.prog()")
    r = None
    if ret:
        r = var.new(IR_REGISTRY[cls.OPCODE]["ret_type"])
    p.issue(cls(*args, ret=r))
    return r


def NODE_UDF(fn, fdnode, fdmail=None):
    return _issue(NodeUDFExecutor, (fn, fdnode, fdmail))


def EDGE_UDF(fn, fdsrc, fdedge, fddst):
    return _issue(EdgeUDFExecutor, (fn, fdsrc, fdedge, fddst))


def SPMV(spA, B, reduce=None):
    return _issue(SPMVExecutor, (spA, B, reduce if reduce is not None else var.STR("sum")))


def SPMV_WITH_DATA(spA, A_data, B, reduce=None):
    return _issue(SPMVWithDataExecutor,
                  (spA, A_data, B, reduce if reduce is not None else var.STR("sum")))


def SPMV_E2V(spA, msg, reduce, fallback=None):
    return _issue(SPMVE2VExecutor, (spA, msg, reduce, fallback))


def DEGREE_BUCKETING(fn, fdmail):
    return _issue(DegreeBucketingExecutor, (fn, fdmail))


def READ(fd, row, col):
    return _issue(ReadExecutor, (fd, row, col))


def READ_COL(fd, col):
    return _issue(ReadColExecutor, (fd, col))


def READ_ROW(fd, row):
    return _issue(ReadRowExecutor, (fd, row))


def MERGE_ROW(idx_list, fd_list):
    return _issue(MergeRowExecutor, (idx_list, fd_list))


def UPDATE_DICT(fd1, fd2):
    return _issue(UpdateDictExecutor, (fd1, fd2))


def NEW_DICT():
    return _issue(NewDictExecutor, ())


def WRITE_(fd, row, col, val):
    _issue(WriteExecutor, (fd, row, col, val), ret=False)


def WRITE_COL_(fd, col, val):
    _issue(WriteColExecutor, (fd, col, val), ret=False)


def WRITE_ROW_(fd, row, val):
    _issue(WriteRowExecutor, (fd, row, val), ret=False)


def WRITE_ROW_INPLACE_(fd, row, val):
    _issue(WriteRowInplaceExecutor, (fd, row, val), ret=False)


def WRITE_DICT_(fd, val):
    _issue(WriteDictExecutor, (fd, val), ret=False)


def APPEND_ROW_(fd, val):
    _issue(AppendRowExecutor, (fd, val), ret=False)


def CLEAR_FRAME_(fd):
    _issue(ClearFrameExecutor, (fd,), ret=False)


def CALL_(fn):
    _issue(CallExecutor, (fn,), ret=False)
