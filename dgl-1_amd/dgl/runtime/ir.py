"""Execution trace of a scheduled call (the debugging role of the reference's
mini-IR dump, python/dgl/runtime/ir/program.py:28-46).

The reference lowers each API call into a thread-local list of executors
(READ_COL, SPMV, WRITE_COL_, ...) and runs them. Here the scheduler calls the
executors directly; when a ``prog()`` context is active each executed op is
recorded so the chosen schedule can be inspected with ``pprint``.
"""
from __future__ import absolute_import

import contextlib
import threading

__all__ = ["prog", "record", "current"]

_local = threading.local()


class Prog(object):
    """Recorded ops of one or more API calls."""

    def __init__(self):
        self.ops = []

    def opcodes(self):
        return [op for op, _ in self.ops]

    def pprint(self):
        lines = []
        for i, (op, info) in enumerate(self.ops):
            args = ", ".join("%s=%s" % kv for kv in sorted(info.items()))
            lines.append("%3d: %s(%s)" % (i, op, args))
        text = "\n".join(lines)
        print(text)
        return text


def current():
    stack = getattr(_local, "stack", None)
    return stack[-1] if stack else None


@contextlib.contextmanager
def prog():
    """Record the ops executed inside the block: ``with ir.prog() as p: ...``."""
    stack = getattr(_local, "stack", None)
    if stack is None:
        stack = _local.stack = []
    p = Prog()
    stack.append(p)
    try:
        yield p
    finally:
        stack.pop()


def record(op, **info):
    p = current()
    if p is not None:
        p.ops.append((op, info))
