"""The mini runtime (counterpart of python/dgl/runtime/runtime.py:6-10):
runs a program's executors in issue order."""
from __future__ import absolute_import

__all__ = ["Runtime"]


class Runtime(object):
    @staticmethod
    def run(prog):
        for exe in prog.execs:
            exe.run()
            prog.trace.append(exe)
