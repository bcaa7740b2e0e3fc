"""Scheduler: lowers message-passing API calls onto g-SpMM kernels.

Counterpart of python/dgl/runtime/scheduler.py (schedule_update_all
:158-198, schedule_snr :111-156, schedule_pull :309-361, schedule_push
:279-307, schedule_recv :58-109, schedule_send :26-56, schedule_apply_nodes /
apply_edges, _gen_send_reduce :470-570, _apply_with_accum :398-426).

Lowering rules (same decisions and result layout as the reference):
  * builtin (message, reduce) pairs with kernel-compatible operands ->
    ``SPMV``: one g-SpMM over the (cached) destination-major adjacency;
  * everything else -> messages are materialised on the triggered edges
    (EDGE_UDF), then builtin reducers run as e2v g-SpMM (copy_e over the
    incidence CSR) and UDF reducers through degree bucketing;
  * reduced rows are in sorted-unique receiver order; an apply function sees
    the node data updated with the reduced values (_apply_with_accum);
  * update_all replaces whole columns (WRITE_DICT_), the others write rows.
"""
from __future__ import absolute_import

import torch

from .. import kernel
from ..base import DGLError
from ..function.base import BuiltinFunction, BundledFunction
from ..udf import EdgeBatch, LazyDict, NodeBatch
from ..utils import is_iterable
from . import degree_bucketing, ir, spmv

__all__ = ["schedule_update_all", "schedule_snr", "schedule_pull", "schedule_push",
           "schedule_recv", "schedule_send", "schedule_apply_nodes", "schedule_apply_edges"]


def _standardize(func, what):
    """UDF, builtin, or list of builtins -> UDF or list (scheduler.py:370-396)."""
    if is_iterable(func):
        for fn in func:
            if not isinstance(fn, BuiltinFunction):
                raise DGLError("If specify multiple message/reduce functions, all of them "
                               "must be builtin")
        return list(func)
    if isinstance(func, BuiltinFunction):
        return [func]
    if not callable(func):
        raise DGLError("User-defined %s function must be callable. Got: %s" % (what, func))
    return func


def _edge_batch(g, u, v, eid):
    nf, ef = g._node_frame, g._edge_frame
    src = LazyDict(lambda k: nf[k].index_select(0, u.to(nf[k].device)), nf.keys())
    dst = LazyDict(lambda k: nf[k].index_select(0, v.to(nf[k].device)), nf.keys())
    edata = LazyDict(lambda k: ef[k].index_select(0, eid.to(ef[k].device)), ef.keys())
    return EdgeBatch(g, (u, v, eid), src, edata, dst)


def _materialize(g, mfunc, u, v, eid):
    """EDGE_UDF over the triggered edges (scheduler.py:572-583)."""
    ir.record("EDGE_UDF", num_edges=len(eid))
    if is_iterable(mfunc):
        mfunc = BundledFunction(mfunc)
    return mfunc(_edge_batch(g, u, v, eid))


def _msg_operands(g, mfn):
    """(ufeat, efeat) for a kernel message on the graph's frames."""
    nf, ef = g._node_frame, g._edge_frame
    ufeat = nf[mfn.src_field] if mfn.kernel_msg != "copy_e" else None
    efeat = ef[mfn.edge_field] if mfn.kernel_msg != "copy_u" else None
    return ufeat, efeat


class _Edges(object):
    """The triggered edges (u, v, eid); for update_all they are produced only
    if messages must be materialised (the kernel path never needs them)."""

    def __init__(self, fn):
        self._fn = fn
        self._val = None

    def get(self):
        if self._val is None:
            self._val = self._fn()
        return self._val


def _send_reduce(g, mfunc, rfunc, edges, recv_nodes, whole_graph):
    """Returns the reduced feature dict (rows = recv_nodes)."""
    nf, ef = g._node_frame, g._edge_frame
    mfunc = _standardize(mfunc, "message")
    rfunc = _standardize(rfunc, "reduce")
    out = {}
    adj_cache = {}

    def adjacency(dev):
        key = str(dev)
        if key not in adj_cache:
            if whole_graph:
                adj_cache[key] = g._graph.adjacency(dev)
            else:
                u, v, eid = edges.get()
                adj_cache[key] = spmv.build_adj_uv(g.number_of_nodes(), u, v, eid, recv_nodes,
                                                   dev)
        return adj_cache[key]

    if is_iterable(mfunc) and is_iterable(rfunc):
        pairs, mfunc, rfunc = spmv.analyze_v2v(mfunc, rfunc, nf, ef)
        for mfn, rfn in pairs:
            ufeat, efeat = _msg_operands(g, mfn)
            dev = (ufeat if ufeat is not None else efeat).device
            ir.record("SPMV", msg=mfn.kernel_msg, reduce=rfn.kernel_reduce,
                      src=mfn.src_field, edge=mfn.edge_field, out=rfn.out_field)
            out[rfn.out_field] = kernel.gspmm(adjacency(dev), mfn.kernel_msg,
                                              rfn.kernel_reduce, ufeat, efeat)
        if not mfunc:
            return out
    u, v, eid = edges.get()
    msgs = _materialize(g, mfunc, u, v, eid)
    if is_iterable(rfunc):
        for rfn in rfunc:
            if rfn.msg_field not in msgs:
                raise DGLError('Reduce function requires message field "%s", but no message '
                               'function generates it.' % rfn.msg_field)
            m = msgs[rfn.msg_field]
            if m.dtype == torch.float32:
                ir.record("SPMV_E2V", reduce=rfn.kernel_reduce, msg=rfn.msg_field,
                          out=rfn.out_field)
                if whole_graph:
                    inc = g._graph.incidence_in(m.device)
                else:
                    inc = spmv.build_inc_dst(v, recv_nodes, m.device)
                out[rfn.out_field] = kernel.gspmm(inc, "copy_e", rfn.kernel_reduce, None, m)
            else:  # non-float32 messages: builtin reducer as a UDF
                ir.record("DEGREE_BUCKETING", reduce=rfn.name, num_msgs=len(v))
                out.update(degree_bucketing.bucket_reduce(g, rfn, recv_nodes, v,
                                                          {rfn.msg_field: m}, nf))
        return out
    ir.record("DEGREE_BUCKETING", reduce="udf", num_msgs=len(v))
    out.update(degree_bucketing.bucket_reduce(g, rfunc, recv_nodes, v, msgs, nf))
    return out


def _apply_with_accum(g, nodes, reduced, apply_func):
    """Apply function over node data updated with the reduced values."""
    if not apply_func:
        return reduced
    ir.record("NODE_UDF", num_nodes=g.number_of_nodes() if nodes is None else len(nodes))
    nf = g._node_frame
    data = nf.select_rows(None if nodes is None else nodes)
    data.update(reduced)
    ids = torch.arange(g.number_of_nodes()) if nodes is None else nodes
    applied = apply_func(NodeBatch(g, ids, data))
    final = dict(reduced)
    final.update(applied)
    return final


def schedule_update_all(g, message_func, reduce_func, apply_func):
    """update_all: send on every edge, reduce at every node."""
    if g.number_of_edges() == 0:
        if apply_func is not None:
            schedule_apply_nodes(g, None, apply_func, inplace=False)
        return
    edges = _Edges(g._graph.edges)
    recv = torch.arange(g.number_of_nodes(), dtype=torch.int64)
    reduced = _send_reduce(g, message_func, reduce_func, edges, recv, True)
    final = _apply_with_accum(g, None, reduced, apply_func)
    ir.record("WRITE_DICT_", keys=sorted(final.keys()))
    g._node_frame.update_rows(None, final)


def schedule_snr(g, u, v, eid, message_func, reduce_func, apply_func, inplace):
    """send_and_recv on the given edges."""
    recv = torch.unique(v, sorted=True)
    reduced = _send_reduce(g, message_func, reduce_func, _Edges(lambda: (u, v, eid)), recv,
                           False)
    final = _apply_with_accum(g, recv, reduced, apply_func)
    ir.record("WRITE_ROW_", num_rows=len(recv), inplace=inplace)
    g._node_frame.update_rows(recv, final, inplace)


def schedule_pull(g, pull_nodes, message_func, reduce_func, apply_func, inplace):
    """pull: receivers are ``pull_nodes`` (including ones without in-edges)."""
    u, v, eid = g._graph.in_edges(pull_nodes)
    if len(eid) == 0:
        if apply_func is not None:
            schedule_apply_nodes(g, pull_nodes, apply_func, inplace)
        return
    recv = torch.unique(pull_nodes, sorted=True)
    reduced = _send_reduce(g, message_func, reduce_func, _Edges(lambda: (u, v, eid)), recv,
                           False)
    final = _apply_with_accum(g, recv, reduced, apply_func)
    ir.record("WRITE_ROW_", num_rows=len(recv), inplace=inplace)
    g._node_frame.update_rows(recv, final, inplace)


def schedule_push(g, push_nodes, message_func, reduce_func, apply_func, inplace):
    """push: send_and_recv along the out-edges of ``push_nodes``."""
    u, v, eid = g._graph.out_edges(push_nodes)
    if len(eid) == 0:
        return
    schedule_snr(g, u, v, eid, message_func, reduce_func, apply_func, inplace)


def schedule_send(g, u, v, eid, message_func):
    """send: materialise messages into the message frame (scheduler.py:26-56)."""
    msgs = _materialize(g, _standardize(message_func, "message"), u, v, eid)
    g._msg_frame.update_rows(eid, msgs)
    g._msg_pending[eid] = True


def schedule_recv(g, recv_nodes, reduce_func, apply_func, inplace):
    """recv: reduce pending messages on the in-edges of ``recv_nodes``."""
    src, dst, eid = g._graph.in_edges(recv_nodes)
    if len(eid):
        keep = g._msg_pending[eid]
        src, dst, eid = src[keep], dst[keep], eid[keep]
    if len(eid) == 0:
        if apply_func is not None:
            schedule_apply_nodes(g, recv_nodes, apply_func, inplace)
        return
    recv = torch.unique(recv_nodes, sorted=True)
    rfunc = _standardize(reduce_func, "reduce")
    msgs = g._msg_frame.select_rows(eid)
    out = {}
    if is_iterable(rfunc):
        for rfn in rfunc:
            m = msgs[rfn.msg_field]
            if m.dtype == torch.float32:
                ir.record("SPMV_E2V", reduce=rfn.kernel_reduce, msg=rfn.msg_field)
                inc = spmv.build_inc_dst(dst, recv, m.device)
                out[rfn.out_field] = kernel.gspmm(inc, "copy_e", rfn.kernel_reduce, None, m)
            else:
                out.update(degree_bucketing.bucket_reduce(g, rfn, recv, dst,
                                                          {rfn.msg_field: m}, g._node_frame))
    else:
        ir.record("DEGREE_BUCKETING", reduce="udf", num_msgs=len(dst))
        out = degree_bucketing.bucket_reduce(g, rfunc, recv, dst, msgs, g._node_frame)
    final = _apply_with_accum(g, recv, out, apply_func)
    g._node_frame.update_rows(recv, final, inplace)
    g._msg_pending[eid] = False
    if not bool(g._msg_pending.any()):
        g._msg_frame.clear()


def schedule_apply_nodes(g, v, apply_func, inplace):
    """apply_nodes over ``v`` (None = all nodes)."""
    nf = g._node_frame
    ids = torch.arange(g.number_of_nodes()) if v is None else v
    ir.record("NODE_UDF", num_nodes=len(ids))
    out = apply_func(NodeBatch(g, ids, nf.select_rows(v)))
    nf.update_rows(v, out, inplace)


def schedule_apply_edges(g, u, v, eid, apply_func, inplace):
    """apply_edges over the given edges (``eid`` None = all edges)."""
    ef = g._edge_frame
    if eid is None:
        u, v, eid = g._graph.edges()
        rows = None
    else:
        rows = eid
    ir.record("EDGE_UDF", num_edges=len(eid))
    out = apply_func(_edge_batch(g, u, v, eid))
    ef.update_rows(rows, out, inplace)
