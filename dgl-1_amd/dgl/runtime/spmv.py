"""Kernel specialisation analysis and adjacency builders.

Counterpart of python/dgl/runtime/spmv.py. The reference decides whether a
(message, reduce) pair can become ``SPMV(adj, H)`` (analyze_v2v_spmv,
spmv.py:11-55) and otherwise materialises messages and reduces them with an
incidence-matrix SPMV (analyze_e2v_spmv, spmv.py:57-81) or degree bucketing.

Here the lowering target is the g-SpMM kernel family, which covers every
builtin pair, so a pair is *kernel-eligible* when its operands fit the kernel:
float32 features, and for edge features either one scalar per edge (the
reference's own SPMV condition, message.py:37-44) or exactly the node
feature's shape. Pairs the reference would specialise are executed with the
reference's arithmetic bit for bit; the others (copy_edge, max, mean, vector
edge weights) are fused instead of materialised.
"""
from __future__ import absolute_import

import torch

from .. import kernel
from ..base import DGLError

__all__ = ["analyze_v2v", "build_adj_uv", "build_inc_eid", "build_inc_dst", "kernel_feat_ok"]


def kernel_feat_ok(mfn, nf, ef):
    """Can the g-SpMM kernel consume this message function's operands?"""
    name = mfn.kernel_msg
    if name in ("copy_u", "u_mul_e"):
        if mfn.src_field not in nf:
            return False
        u = nf[mfn.src_field]
        if u.dtype != torch.float32:
            return False
    if name in ("u_mul_e", "copy_e"):
        if mfn.edge_field not in ef:
            return False
        e = ef[mfn.edge_field]
        if e.dtype != torch.float32:
            return False
        if name == "u_mul_e":
            u = nf[mfn.src_field]
            try:
                kernel._edge_len(e.shape[1:], u.shape[1:])
            except DGLError:
                return False
            if e.device != u.device:
                return False
    return True


def analyze_v2v(mfuncs, rfuncs, nf, ef):
    """Split builtin lists into kernel pairs and leftovers.

    Returns (pairs, mfunc_left, rfunc_left) with the pairing rule of
    spmv.py:11-55 (reducer ↔ message by message field).
    """
    by_field = {m.out_field: m for m in mfuncs}
    pairs, mleft, rleft, touched = [], [], [], set()
    for rfn in rfuncs:
        if rfn.msg_field not in by_field:
            raise DGLError('Reduce function requires message field "%s", but no message '
                           'function generates it.' % rfn.msg_field)
        mfn = by_field[rfn.msg_field]
        if kernel_feat_ok(mfn, nf, ef):
            pairs.append((mfn, rfn))
        else:
            if rfn.msg_field not in touched:
                touched.add(rfn.msg_field)
                mleft.append(mfn)
            rleft.append(rfn)
    return pairs, mleft, rleft


def _relabel(recv_nodes, v):
    return torch.searchsorted(recv_nodes, v)


def build_adj_uv(num_nodes, u, v, eid, recv_nodes, device):
    """(|recv|, N) adjacency of the given edges (spmv.py:154-227): rows are the
    destinations relabelled into sorted-unique ``recv_nodes``, columns global
    source ids, slots in the given edge order. Its ``eid`` values are the
    edges' global ids so edge features are read in place."""
    rows = _relabel(recv_nodes, v)
    adj = kernel.from_coo(len(recv_nodes), num_nodes, rows, u, kernel.ORDER_EID, device)
    return _remap_eid(adj, eid)


def build_inc_eid(m, eid, v, recv_nodes, device):
    """(|recv|, m) incidence of messages by edge id (spmv.py:249-314): slot k
    of row ``searchsorted(recv_nodes, v[k])`` is column ``eid[k]``, and its
    slot eid is ``eid[k]`` too, so copy_e over it reads the message frame's
    rows in place (no gathered copy of the pending messages). Receivers
    without messages are empty rows (0 for sum, the initializer)."""
    eid = torch.as_tensor(eid, dtype=torch.int64)
    rows = _relabel(recv_nodes, v)
    adj = kernel.from_coo(len(recv_nodes), m, rows, eid, kernel.ORDER_EID, device)
    return _remap_eid(adj, eid)


def build_inc_dst(v, recv_nodes, device):
    """(|recv|, len(v)) incidence of message positions (spmv.py:316-353):
    build_inc_eid over positions 0..len(v)-1, as the reference defines it."""
    return build_inc_eid(len(v), torch.arange(len(v), dtype=torch.int64), v, recv_nodes,
                         device)


class _RemappedAdj(kernel.SparseAdj):
    """SparseAdj whose slot eids are translated through ``eid_map``."""

    def __init__(self, base, eid_map):
        fwd = _remap_csr(base.fwd, eid_map)

        def tb(dev):
            return _remap_csr(base.bwd.to(dev), eid_map)

        super(_RemappedAdj, self).__init__(fwd, tb, base.shape)


def _remap_csr(csr, eid_map):
    m = eid_map.to(csr.device)
    return kernel.CSR(csr.indptr, csr.indices, m[csr.eid], csr.num_cols, csr.row_order,
                      csr._host_indptr)


def _remap_eid(adj, eid):
    eid = torch.as_tensor(eid, dtype=torch.int64)
    n = len(eid)
    if n and bool((eid == torch.arange(n, dtype=torch.int64)).all()):
        return adj
    return _RemappedAdj(adj, eid)
