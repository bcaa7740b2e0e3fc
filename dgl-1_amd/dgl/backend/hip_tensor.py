"""The reference-side binding of libdgl_hip.so for the tensor-backend route
(boundary b1): what a maintainer of the reference puts in place of
``sparse_matrix`` / ``sparse_matrix_indices`` / ``spmm`` in
python/dgl/backend/pytorch/tensor.py:45-51,145-146.

It is plain ctypes over the C-ABI (include/dgl_hip.h) and torch — nothing
from this engine's Python package — so it drops into the reference as it
stands. The adjacency the reference builds once and caches per context
(GraphIndex.adjacency_matrix, python/dgl/graph_index.py:537-585, whose
``idx`` already lives on the context) becomes, on its first product on a
device, a CSR built on that device (dglhip_coo_to_csr_device) and its launch
plan (dglhip_spmm_plan_create); every later ``spmm`` on that matrix runs the
plan (dglhip_spmm_plan_run): the source-blocked schedule, the heavy-row
split and the short-row tiers, with no per-call upload, sort or host sync.
Whether the values are the adjacency's ones (copy_src) or edge weights
(src_mul_edge) is decided once, when the matrix is made. The backward of
``spmm`` with respect to the dense operand is the product over the
transposed CSR (built on first use), as torch.sparse.mm's autograd does.
Results equal torch.sparse.mm on the same uncoalesced COO bit for bit
(tests/test_hip_tensor_binding.py).
"""
import ctypes
import os

import torch as th

_vp, _i64, _int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
_EDGE_BY_EID = 1


def _load():
    path = os.environ.get("DGL_LIBRARY_PATH", "")
    if not path.endswith(".so"):
        here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        path = os.path.join(here, "lib", "libdgl_hip.so")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    sig = {
        "DGLGetLastError": (ctypes.c_char_p, []),
        "dglhip_coo_to_csr_workspace_bytes": (_i64, [_i64, _i64, _i64, _int]),
        "dglhip_coo_to_csr_device": (_int, [_i64, _i64, _i64, _vp, _vp, _int, _vp, _vp, _vp, _vp,
                                            _i64, _vp]),
        "dglhip_coo_to_csr_host": (_int, [_i64, _i64, _i64, _vp, _vp, _int, _vp, _vp, _vp]),
        "dglhip_spmm_plan_create": (_int, [_int, _int, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                                           ctypes.POINTER(_vp)]),
        "dglhip_spmm_plan_free": (_int, [_vp]),
        "dglhip_spmm_plan_workspace": (_int, [_vp, _int, _int, _i64, _i64, _i64, _i64, _int, _vp,
                                              _vp, ctypes.POINTER(_i64)]),
        "dglhip_spmm_plan_run": (_int, [_vp, _int, _int, _i64, _vp, _i64, _i64, _vp, _i64, _int,
                                        _vp, _vp, _vp, _vp, _i64, _vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


_lib = _load()


def _check(rc):
    if rc != 0:
        raise RuntimeError(_lib.DGLGetLastError().decode())


def _stream(dev):
    return th.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None


def _p(t):
    return None if t is None else t.data_ptr()


class _CSR(object):
    """One orientation of the matrix on one device: CSR arrays + launch plan."""

    def __init__(self, rows, cols, r, c, dev):
        nnz = r.numel()
        self.num_rows, self.num_cols = rows, cols
        self.indptr = th.empty(rows + 1, dtype=th.int64, device=dev)
        self.indices = th.empty(nnz, dtype=th.int32, device=dev)
        self.eid = th.empty(nnz, dtype=th.int64, device=dev)  # the COO position of each slot
        r, c = r.to(dev, th.int64).contiguous(), c.to(dev, th.int64).contiguous()
        if dev.type == "cuda":
            nb = _lib.dglhip_coo_to_csr_workspace_bytes(rows, cols, nnz, 0)
            ws = th.empty(max(nb, 1), dtype=th.uint8, device=dev)
            _check(_lib.dglhip_coo_to_csr_device(rows, cols, nnz, _p(r), _p(c), 0,
                                                 _p(self.indptr), _p(self.indices), _p(self.eid),
                                                 _p(ws), nb, _stream(dev)))
            kind = (10, dev.index if dev.index is not None else th.cuda.current_device())
        else:
            _check(_lib.dglhip_coo_to_csr_host(rows, cols, nnz, _p(r), _p(c), 0, _p(self.indptr),
                                               _p(self.indices), _p(self.eid)))
            kind = (1, 0)
        h = _vp()
        _check(_lib.dglhip_spmm_plan_create(kind[0], kind[1], rows, cols, nnz, _p(self.indptr),
                                            _p(self.indices) if nnz else None, None, None,
                                            _stream(dev), ctypes.byref(h)))
        self.plan = h.value

    def __del__(self):
        if getattr(self, "plan", None):
            _lib.dglhip_spmm_plan_free(self.plan)
            self.plan = None

    def product(self, y, weights):
        """out = A y (u_mul_e with the weights by edge id, else copy_u), sum."""
        y = y.contiguous()
        dev, F = y.device, y.shape[1]
        msg, elen = (1, 1) if weights is not None else (0, 0)
        out = th.empty(self.num_rows, F, dtype=th.float32, device=dev)
        nb = _i64()
        _check(_lib.dglhip_spmm_plan_workspace(self.plan, msg, 0, F, 0, y.shape[0], elen,
                                               _EDGE_BY_EID, _p(self.eid), _stream(dev),
                                               ctypes.byref(nb)))
        ws = th.empty(nb.value, dtype=th.uint8, device=dev) if nb.value else None
        _check(_lib.dglhip_spmm_plan_run(self.plan, msg, 0, F, _p(y), 0, y.shape[0],
                                         _p(weights), elen, _EDGE_BY_EID, _p(self.eid), _p(out),
                                         None, _p(ws), nb.value, _stream(dev)))
        return out


class HipSparseMatrix(object):
    """What sparse_matrix returns: the COO (index, values, shape) as the
    reference passes it, plus per-device CSRs and plans built on first use."""

    def __init__(self, data, idx, shape):
        self.idx, self.data, self.shape = idx, data, (int(shape[0]), int(shape[1]))
        # ones (the adjacency: copy_src) or edge weights (src_mul_edge),
        # decided once per matrix, not per product
        self.weights = None if bool((data == 1).all()) else data.reshape(-1).float().contiguous()
        self._dev = {}

    def csr(self, dev, transpose=False):
        key = (str(dev), transpose)
        if key not in self._dev:
            r, c = (self.idx[1], self.idx[0]) if transpose else (self.idx[0], self.idx[1])
            rows, cols = (self.shape[1], self.shape[0]) if transpose else self.shape
            self._dev[key] = _CSR(rows, cols, r, c, dev)
        return self._dev[key]

    def weights_on(self, dev):
        w = self.weights
        return None if w is None else w.to(dev)

    def _indices(self):
        return self.idx


class _HipSpMM(th.autograd.Function):
    @staticmethod
    def forward(ctx, mat, y):
        ctx.mat = mat
        return mat.csr(y.device).product(y, mat.weights_on(y.device))

    @staticmethod
    def backward(ctx, dy):
        mat = ctx.mat
        return None, mat.csr(dy.device, transpose=True).product(dy, mat.weights_on(dy.device))


def get_preferred_sparse_format():
    return "coo"


def sparse_matrix(data, index, shape, force_format=False):
    fmt = index[0]
    if fmt != 'coo':
        raise TypeError('Pytorch backend only supports COO format. But got %s.' % fmt)
    return HipSparseMatrix(data, index[1], shape), None


def sparse_matrix_indices(spmat):
    return ('coo', spmat._indices())


def spmm(x, y):
    return _HipSpMM.apply(x, y)
