"""The message-passing mini-IR: variables, executors, programs
(counterpart of python/dgl/runtime/ir/)."""
from __future__ import absolute_import

from . import var  # noqa: F401
from .executor import *  # noqa: F401,F403
from .executor import Executor, OpCode  # noqa: F401
from .program import Prog, get_current_prog, prog, set_current_prog  # noqa: F401
from .registry import IR_REGISTRY, op_name  # noqa: F401
