"""dgl — MI355X-native message-passing engine with the DGL 0.1.3 API.

``import dgl`` resolves here when ``dgl-1_amd/`` is on ``sys.path``. The
package keeps the reference's operator surface (DGLGraph, dgl.function,
the scheduler, the backend plugin, the C-ABI registry) and executes builtin
message passing on hand-written HIP g-SpMM kernels (libdgl_hip.so).
"""
from __future__ import absolute_import

__version__ = "0.1.3+mi355x"

from . import function  # noqa: F401
from . import backend  # noqa: F401
from . import init  # noqa: F401
from . import kernel  # noqa: F401
from .base import ALL, DGLError  # noqa: F401
from .graph import DGLGraph  # noqa: F401
from .udf import EdgeBatch, NodeBatch  # noqa: F401
from .runtime import ir  # noqa: F401
from . import nn  # noqa: F401
from ._ffi import list_global_names as list_global_func_names  # noqa: F401
