"""TEST ORACLE — test infrastructure only, never imported by the product.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, as the checker or the timed CPU baseline.

Python front-end of the plain-C restatement in spmm_oracle.c (see its header
for the reference file:line each routine follows and for how the third-party
arithmetic is pinned), plus pure-numpy restatements for small cases.
"""
from __future__ import absolute_import

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    """Compile spmm_oracle.c with gcc (oracle/Makefile)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.isfile(_SO):
            build()
        _lib = ctypes.CDLL(_SO)
        P = ctypes.c_void_p
        I = ctypes.c_int64
        _lib.oracle_spmm_coo.argtypes = [I, I, I, P, P, P, P, P]
        _lib.oracle_coo_to_csr.argtypes = [I, I, P, P, P, P, P]
        _lib.oracle_spmm_csr.argtypes = [I, I, P, P, P, P, P, P, ctypes.c_int]
        _lib.oracle_max_mailbox.argtypes = [I, I, P, P, P, P]
        _lib.oracle_mean_mailbox.argtypes = [I, I, P, P, P, P]
        _lib.oracle_sddmm_dot.argtypes = [I, I, P, P, P, P, P]
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def spmm_coo(num_rows, row, col, H, val=None):
    """torch.sparse.mm(sparse_coo_tensor([row; col], val|ones), H) restated."""
    H = _f32(H)
    F = H.shape[1] if H.ndim == 2 else 1
    row, col, val = _i64(row), _i64(col), _f32(val)
    out = np.empty((num_rows, F), np.float32)
    lib().oracle_spmm_coo(num_rows, F, len(row), _p(row), _p(col), _p(val), _p(H), _p(out))
    return out


def coo_to_csr(num_rows, row, col):
    """Stable grouping by row: (indptr, indices, pos) — CSR in nnz order."""
    row, col = _i64(row), _i64(col)
    nnz = len(row)
    indptr = np.empty(num_rows + 1, np.int64)
    indices = np.empty(nnz, np.int64)
    pos = np.empty(nnz, np.int64)
    lib().oracle_coo_to_csr(num_rows, nnz, _p(row), _p(col), _p(indptr), _p(indices), _p(pos))
    return indptr, indices, pos


def spmm_csr(indptr, indices, pos, H, val=None, num_threads=None):
    """Same product from the grouped form, OpenMP over rows (CPU baseline)."""
    H = _f32(H)
    indptr, indices, pos, val = _i64(indptr), _i64(indices), _i64(pos), _f32(val)
    R = len(indptr) - 1
    out = np.empty((R, H.shape[1]), np.float32)
    nt = num_threads or os.cpu_count() or 1
    lib().oracle_spmm_csr(R, H.shape[1], _p(indptr), _p(indices), _p(pos), _p(val), _p(H),
                          _p(out), int(nt))
    return out


def max_mailbox(num_rows, row, msg):
    """Degree-bucketing max of messages msg[e] grouped by row[e]."""
    indptr, _, pos = coo_to_csr(num_rows, row, np.zeros(len(row), np.int64))
    msg = _f32(msg)
    out = np.empty((num_rows, msg.shape[1]), np.float32)
    lib().oracle_max_mailbox(num_rows, msg.shape[1], _p(indptr), _p(pos), _p(msg), _p(out))
    return out


def mean_mailbox(num_rows, row, msg):
    """Degree-bucketing mean (double accumulation; tolerance reference)."""
    indptr, _, pos = coo_to_csr(num_rows, row, np.zeros(len(row), np.int64))
    msg = _f32(msg)
    out = np.empty((num_rows, msg.shape[1]), np.float32)
    lib().oracle_mean_mailbox(num_rows, msg.shape[1], _p(indptr), _p(pos), _p(msg), _p(out))
    return out


def sddmm_dot(row, col, A, B):
    """out[e] = <A[row[e]], B[col[e]]> in double (tolerance reference)."""
    row, col, A, B = _i64(row), _i64(col), _f32(A), _f32(B)
    out = np.empty(len(row), np.float32)
    lib().oracle_sddmm_dot(len(row), A.shape[1], _p(row), _p(col), _p(A), _p(B), _p(out))
    return out


# -- pure numpy restatement (small cases only) --------------------------------
def spmm_coo_py(num_rows, row, col, H, val=None):
    """Loop-for-loop restatement of the nnz-order fma chain (tiny inputs)."""
    H = np.asarray(H, np.float32)
    out = np.zeros((num_rows, H.shape[1]), np.float32)
    for e in range(len(row)):
        w = np.float64(1.0 if val is None else val[e])
        r = row[e]
        out[r] = (out[r].astype(np.float64) + w * H[col[e]].astype(np.float64)).astype(np.float32)
    return out
