"""Programs: the executor list one API call lowers to (counterpart of
python/dgl/runtime/ir/program.py:9-78).

The scheduler issues executors into the current thread's program; the
runtime then runs them in order (dgl.runtime.runtime.Runtime). Programs
nest: an API call made inside a user's ``with ir.prog() as p`` block runs
its own program, and every executor it ran is appended to ``p.trace``, so
the user can inspect the schedule the call took (``p.opcodes()``,
``p.pprint()``).
"""
from __future__ import absolute_import

import threading
from contextlib import contextmanager

from .registry import op_name

__all__ = ["Prog", "get_current_prog", "set_current_prog", "prog"]


class Prog(object):
    """An ordered list of executors.

    execs : issued, in issue order (what Runtime.run executes)
    trace : executors that have run, this program's and its children's
    """

    def __init__(self):
        self.execs = []
        self.trace = []
        self.varcount = 0

    def issue(self, exe):
        self.execs.append(exe)

    def opcodes(self):
        """Names of the executors that ran (or were issued, before a run)."""
        return [op_name(e.opcode()) for e in (self.trace or self.execs)]

    def pprint_exe(self, exe):
        args = ", ".join(str(a) for a in exe.arg_vars() if a is not None)
        ret = exe.ret_var()
        if ret is None:
            return "%s(%s)" % (op_name(exe.opcode()), args)
        return "%s %s = %s(%s)" % (ret.typestr(), ret.name, op_name(exe.opcode()), args)

    def pprint(self):
        text = "\n".join(self.pprint_exe(e) for e in (self.trace or self.execs))
        print(text)
        return text


class _Current(threading.local):
    def __init__(self):
        super(_Current, self).__init__()
        self.prog = None


_CURRENT = _Current()


def get_current_prog():
    return _CURRENT.prog


def set_current_prog(program):
    _CURRENT.prog = program


@contextmanager
def prog():
    """A new program, current for the block; the enclosing one (if any) is
    restored afterwards and inherits this one's trace."""
    parent = _CURRENT.prog
    p = Prog()
    _CURRENT.prog = p
    try:
        yield p
    finally:
        _CURRENT.prog = parent
        if parent is not None:
            parent.trace.extend(p.trace)
