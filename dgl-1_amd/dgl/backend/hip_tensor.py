"""The reference-side binding of libdgl_hip.so for the tensor-backend route
(boundary b1): what a maintainer of the reference puts in place of
``sparse_matrix`` / ``sparse_matrix_indices`` / ``spmm`` in
python/dgl/backend/pytorch/tensor.py:45-51,145-146.

It is plain ctypes over the C-ABI (include/dgl_hip.h) and torch — nothing
from this engine's Python package — so it drops into the reference as it
stands.

Structure and values are kept apart. The structure (the COO index) is what
the reference builds once and caches per context
(GraphIndex.adjacency_matrix, python/dgl/graph_index.py:537-585); on its
first product on a device it becomes a CSR built on that device
(dglhip_coo_to_csr_device) plus its launch plan (dglhip_spmm_plan_create),
one per orientation. That structure is cached on the index tensor itself
(a weak map keyed by the tensor's identity and version), so the per-call
rebuild of SPMVWithDataExecutor.run
(python/dgl/runtime/ir/executor.py:544-548: ``sparse_matrix_indices`` of the
cached adjacency, then ``sparse_matrix(A_data, spidx, shape)``) finds the
same CSRs and plans: no sort, no plan build, no host sync on the second call.

The values are per matrix: the adjacency's ones (copy_src: the plan's copy_u
product) or edge weights (src_mul_edge: u_mul_e by edge id). Which one is
decided without a device sync except for the first matrix made on an index
(that is the adjacency itself, once per graph and device); a weighted product
whose weights happen to be ones gives the copy_u bits anyway
(fma(1, h, acc) == acc + h).

Autograd follows torch.sparse.mm on ``th.sparse_coo_tensor(idx, data)``
(tensor.py:45-51,145-146):
  * dY = A^T dC, the product over the transposed CSR (same bits as torch's
    CPU kernel on the uncoalesced COO);
  * d(data)[e] = <dC[idx[0, e]], Y[idx[1, e]]> for every COO position e,
    duplicates included (torch gives every duplicate the full dot), the
    g-SDDMM dot (dglhip_gsddmm_device, fp32, features in order) over whichever
    orientation walks the edge ids more nearly in order (a*b == b*a, so both
    give the same bits).
"""
import ctypes
import os
import weakref

import torch as th

_vp, _i64, _int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
_EDGE_BY_EID = 1
_SDDMM_DOT = 0


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
        "dglhip_gsddmm_device": (_int, [_int, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                        _vp]),
        "dglhip_gsddmm_host": (_int, [_int, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                      _int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


_lib = _load()

# How many CSR + plan builds this process has made (a test reads it to show
# that the executor's per-call rebuild reuses the cached structure).
builds = 0


def _check(rc):
    if rc != 0:
        raise RuntimeError(_lib.DGLGetLastError().decode())


def _stream(dev):
    return th.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None


def _p(t):
    return None if t is None else t.data_ptr()


def _dense_f32(y):
    # torch.sparse.mm raises on a dense operand of another dtype; so do we,
    # rather than read its bytes as float32
    if y.dtype != th.float32:
        raise RuntimeError("expected scalar type Float but found %s" % y.dtype)
    return y.contiguous()


class _CSR(object):
    """One orientation of the matrix on one device: CSR arrays + launch plan."""

    def __init__(self, rows, cols, r, c, dev):
        global builds
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
        self._loc = None
        builds += 1

    def __del__(self):
        plan, self.plan = getattr(self, "plan", None), None
        if plan and _lib is not None:  # module globals may be gone at interpreter shutdown
            try:
                _lib.dglhip_spmm_plan_free(plan)
            except Exception:  # noqa: BLE001 - never raise from a finaliser
                pass

    @property
    def eid_locality(self):
        """Fraction of consecutive slots whose COO positions are consecutive:
        how sequential per-edge stores at out[eid] are along this CSR (one
        reduction + sync, once per CSR)."""
        if self._loc is None:
            n = self.eid.numel()
            self._loc = 1.0 if n < 2 else \
                float((self.eid[1:] == self.eid[:-1] + 1).sum().item()) / (n - 1)
        return self._loc

    def product(self, y, weights):
        """out = A y (u_mul_e with the weights by edge id, else copy_u), sum."""
        y = _dense_f32(y)
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

    def edge_dot(self, lhs, rhs, nnz):
        """out[eid[k]] = <lhs[row of k], rhs[indices[k]]> (fp32, features in
        order) for every slot k: one value per COO position."""
        lhs, rhs = _dense_f32(lhs), _dense_f32(rhs)
        dev, F = lhs.device, lhs.shape[1]
        out = th.empty(nnz, dtype=th.float32, device=dev)
        if nnz == 0:
            return out
        args = (_SDDMM_DOT, self.num_rows, F, 1, _p(self.indptr), _p(self.indices), _p(self.eid),
                _p(lhs), _p(rhs), _p(out))
        if dev.type == "cuda":
            _check(_lib.dglhip_gsddmm_device(*(args + (_stream(dev),))))
        else:
            _check(_lib.dglhip_gsddmm_host(*(args + (0,))))
        return out


class _Structure(object):
    """The per-device CSRs (both orientations) of one COO index; shared by
    every matrix made on that index tensor."""

    def __init__(self, idx, shape):
        # the index itself is not held: the cache entry must not keep its key alive
        self.shape, self.version = shape, idx._version
        self.nnz = int(idx.shape[1])
        self.dev = {}

    def csr(self, idx, dev, transpose=False):
        key = (str(dev), transpose)
        if key not in self.dev:
            r, c = (idx[1], idx[0]) if transpose else (idx[0], idx[1])
            rows, cols = (self.shape[1], self.shape[0]) if transpose else self.shape
            self.dev[key] = _CSR(rows, cols, r, c, dev)
        return self.dev[key]


# id(idx) -> (weakref to idx, _Structure); an entry leaves with its tensor.
_structures = {}


def _drop(key, ref):
    hit = _structures.get(key)
    if hit is not None and hit[0] is ref:
        del _structures[key]


def _structure_of(idx, shape):
    """(structure, new): the cached structure of this index tensor, or a new
    one when the tensor is new, has been written in place or is used with
    another shape."""
    key = id(idx)
    hit = _structures.get(key)
    if hit is not None and hit[0]() is idx:
        st = hit[1]
        if st.version == idx._version and st.shape == shape:
            return st, False
    st = _Structure(idx, shape)
    ref = weakref.ref(idx, lambda r, k=key: _drop(k, r))
    _structures[key] = (ref, st)
    return st, True


class HipSparseMatrix(object):
    """What sparse_matrix returns: the COO (index, values, shape) as the
    reference passes it; its CSRs and plans live on the index's structure."""

    def __init__(self, data, idx, shape):
        self.idx, self.data, self.shape = idx, data, (int(shape[0]), int(shape[1]))
        self._st, new = _structure_of(idx, self.shape)
        if data.dim() != 1 or data.shape[0] != self._st.nnz:
            data = data.reshape(-1)
            if data.shape[0] != self._st.nnz:
                raise RuntimeError("sparse_matrix: %d values for %d indices"
                                   % (data.shape[0], self._st.nnz))
        # ones (the adjacency: copy_src) or edge weights (src_mul_edge). Only
        # the first matrix on an index pays a value check (a host sync); a
        # rebuild on a cached index (SPMVWithDataExecutor) is taken as weighted
        # without one, and so is data that asks for a gradient.
        if data.requires_grad or not new:
            self.ones = False
        else:
            self.ones = bool((data == 1).all())

    def csr(self, dev, transpose=False):
        return self._st.csr(self.idx, dev, transpose)

    def weights_on(self, dev, data=None):
        if self.ones:
            return None
        w = self.data if data is None else data
        return w.detach().reshape(-1).to(dev, th.float32).contiguous()

    def _indices(self):
        return self.idx


class _HipSpMM(th.autograd.Function):
    @staticmethod
    def forward(ctx, mat, data, y):
        ctx.mat = mat
        w = mat.weights_on(y.device, data)
        ctx.save_for_backward(y, w if w is not None else th.empty(0))
        ctx.data_shape, ctx.data_dtype = data.shape, data.dtype
        return mat.csr(y.device).product(y, w)

    @staticmethod
    def backward(ctx, dc):
        mat = ctx.mat
        y, w = ctx.saved_tensors
        w = None if mat.ones else w
        dc = dc.contiguous()
        dy = dd = None
        if ctx.needs_input_grad[2]:
            dy = mat.csr(dc.device, transpose=True).product(dc, w)
        if ctx.needs_input_grad[1]:
            fwd = mat.csr(dc.device)
            bwd = mat.csr(dc.device, transpose=True)
            # stores at out[eid] along the orientation whose slots walk the
            # COO positions more nearly in order (the same bits either way)
            if bwd.eid_locality > max(0.5, 2.0 * fwd.eid_locality):
                dd = bwd.edge_dot(y, dc, mat._st.nnz)
            else:
                dd = fwd.edge_dot(dc, y, mat._st.nnz)
            dd = dd.reshape(ctx.data_shape).to(ctx.data_dtype)
        return None, dd, dy


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
    return _HipSpMM.apply(x, x.data, y)
