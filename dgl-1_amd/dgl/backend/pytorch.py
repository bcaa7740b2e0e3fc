"""PyTorch-ROCm backend (python/dgl/backend/pytorch/tensor.py).

The hot-path hooks (tensor.py:26-51,145-146) are re-implemented on the
engine: ``sparse_matrix`` builds a :class:`SparseMatrix` over the engine's CSR
and ``spmm`` runs the HIP g-SpMM (autograd included). The remaining helpers
are the plain tensor utilities the reference's backend exposes.
"""
from __future__ import absolute_import

import torch

from .. import kernel
from ..base import DGLError

__all__ = ["get_preferred_sparse_format", "sparse_matrix", "sparse_matrix_indices", "spmm",
           "SparseMatrix", "cpu", "tensor", "shape", "dtype", "ndim", "context", "astype",
           "asnumpy", "copy_to", "zeros", "zeros_like", "ones", "arange", "cat", "stack",
           "reshape", "unsqueeze", "squeeze", "sum", "max", "mean", "is_tensor",
           "data_type_dict", "float32", "float64", "int32", "int64"]

float32, float64, int32, int64 = torch.float32, torch.float64, torch.int32, torch.int64


def data_type_dict():
    return {"float16": torch.float16, "float32": torch.float32, "float64": torch.float64,
            "uint8": torch.uint8, "int8": torch.int8, "int16": torch.int16,
            "int32": torch.int32, "int64": torch.int64}


def cpu():
    return torch.device("cpu")


def get_preferred_sparse_format():
    """The engine's kernels consume CSR (the reference's PyTorch backend said 'coo')."""
    return "csr"


class SparseMatrix(object):
    """A (rows x cols) sparse matrix for ``spmm``: engine CSR + optional values.

    Slot order follows the input: COO entries keep their nnz order (the order
    torch.sparse.mm consumes an uncoalesced COO), CSR entries their given order.
    """

    def __init__(self, adj, data, num_nnz, row, col):
        self.adj = adj
        self.data = data
        self.nnz = num_nnz
        self._row = row
        self._col = col

    @property
    def shape(self):
        return self.adj.shape

    def indices(self):
        return torch.stack([self._row, self._col])


def sparse_matrix(data, index, shape, force_format=False):  # pylint: disable=unused-argument
    """Build a sparse matrix from ('coo', idx[2, nnz]) or ('csr', indices, indptr)."""
    fmt = index[0]
    if fmt == "coo":
        idx = index[1]
        row, col = idx[0].to(torch.int64), idx[1].to(torch.int64)
    elif fmt == "csr":
        indices, indptr = index[1].to(torch.int64), index[2].to(torch.int64)
        row = torch.repeat_interleave(torch.arange(len(indptr) - 1, device=indptr.device),
                                      indptr[1:] - indptr[:-1])
        col = indices
    else:
        raise TypeError("Unsupported sparse format %s" % fmt)
    dev = data.device if isinstance(data, torch.Tensor) else row.device
    adj = kernel.from_coo(int(shape[0]), int(shape[1]), row.cpu(), col.cpu(), kernel.ORDER_EID,
                          dev)
    return SparseMatrix(adj, data, row.numel(), row, col), None


def sparse_matrix_indices(spmat):
    return ("coo", spmat.indices())


def _is_all_ones(data):
    return data is None or bool((data == 1).all())


def spmm(x, y):
    """x (SparseMatrix) @ y (dense [cols, F] or [cols]) on the engine's g-SpMM."""
    if not isinstance(x, SparseMatrix):
        raise DGLError("spmm expects a SparseMatrix built by sparse_matrix()")
    if y.dtype != torch.float32:
        raise DGLError("g-SpMM computes in float32; got %s" % y.dtype)
    adj = x.adj.to(y.device)
    if x.data is not None and x.data.requires_grad or not _is_all_ones(x.data):
        return kernel.gspmm(adj, "u_mul_e", "sum", y, x.data.to(y.device))
    return kernel.gspmm(adj, "copy_u", "sum", y)


def is_tensor(obj):
    return isinstance(obj, torch.Tensor)


def tensor(data, dtype=None):
    return torch.tensor(data, dtype=dtype)


def shape(x):
    return x.shape


def dtype(x):
    return x.dtype


def ndim(x):
    return x.dim()


def context(x):
    return x.device


def astype(x, ty):
    return x.type(ty)


def asnumpy(x):
    return x.detach().cpu().numpy()


def copy_to(x, ctx):
    return x.to(ctx)


def zeros(shape_, dtype_, ctx):
    return torch.zeros(shape_, dtype=dtype_, device=ctx)


def zeros_like(x):
    return torch.zeros_like(x)


def ones(shape_, dtype_, ctx):
    return torch.ones(shape_, dtype=dtype_, device=ctx)


def arange(start, stop):
    return torch.arange(start, stop, dtype=torch.int64)


def cat(seq, dim):
    return torch.cat(seq, dim=dim)


def stack(seq, dim):
    return torch.stack(seq, dim=dim)


def reshape(x, shape_):
    return x.reshape(shape_)


def unsqueeze(x, dim):
    return x.unsqueeze(dim)


def squeeze(x, dim):
    return x.squeeze(dim)


def sum(x, dim):  # pylint: disable=redefined-builtin
    return x.sum(dim)


def max(x, dim):  # pylint: disable=redefined-builtin
    return x.max(dim)[0]


def mean(x, dim):
    return x.mean(dim)
