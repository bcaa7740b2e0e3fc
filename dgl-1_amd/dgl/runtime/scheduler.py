"""Scheduler: lowers message-passing API calls into IR programs.

Counterpart of python/dgl/runtime/scheduler.py (schedule_update_all
:158-198, schedule_snr :111-156, schedule_pull :309-361, schedule_push
:279-307, schedule_recv :58-109, schedule_send :26-56, schedule_apply_nodes /
apply_edges, _gen_send_reduce :470-570, _apply_with_accum :398-426).

Every public schedule_* call issues executors (runtime/ir/executor.py) into a
fresh program and runs it (runtime/runtime.py), as the reference does.
Lowering rules (same decisions and result layout as the reference):
  * builtin (message, reduce) pairs with kernel-compatible operands ->
    ``SPMV`` / ``SPMV_WITH_DATA`` (copy_edge: ``SPMV_E2V`` over the
    adjacency): one g-SpMM over the (cached) destination-major adjacency;
  * everything else -> messages are materialised on the triggered edges
    (``EDGE_UDF``), then builtin reducers run as e2v g-SpMM (``SPMV_E2V``,
    copy_e over the incidence CSR) and UDF reducers through degree bucketing
    (``DEGREE_BUCKETING``);
  * reduced rows are in sorted-unique receiver order; an apply function sees
    the node data updated with the reduced values (``NODE_UDF`` over
    ``UPDATE_DICT(READ_ROW(nf, recv), reduced)``, _apply_with_accum);
  * update_all replaces whole columns (``WRITE_DICT_``), the others write rows
    (``WRITE_ROW_`` / ``WRITE_ROW_INPLACE_``).
"""
from __future__ import absolute_import

import functools

import torch

from ..base import DGLError
from ..function.base import BuiltinFunction, BundledFunction
from ..udf import EdgeBatch, LazyDict, NodeBatch
from ..utils import is_iterable
from . import degree_bucketing, ir, spmv
from .ir import var
from .runtime import Runtime

__all__ = ["schedule_update_all", "schedule_snr", "schedule_pull", "schedule_push",
           "schedule_recv", "schedule_send", "schedule_apply_nodes", "schedule_apply_edges"]


def _program(fn):
    """A public schedule_* entry: lower the call into a new program, run it."""
    @functools.wraps(fn)
    def wrapper(*args, **kw):
        with ir.prog() as p:
            fn(*args, **kw)
            Runtime.run(p)
    return wrapper


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


def _edge_vars(g, u, v, eid):
    """(src, edge, dst) feature-dict variables of the triggered edges: lazy
    row gathers from the frames, taken when an executor reads them."""
    nf, ef = g._node_frame, g._edge_frame
    src = LazyDict(lambda k: nf[k].index_select(0, u.to(nf[k].device)), nf.keys())
    dst = LazyDict(lambda k: nf[k].index_select(0, v.to(nf[k].device)), nf.keys())
    edata = LazyDict(lambda k: ef[k].index_select(0, eid.to(ef[k].device)), ef.keys())
    return var.FEAT_DICT(src, "src"), var.FEAT_DICT(edata, "edata"), var.FEAT_DICT(dst, "dst")


def _edge_udf(g, func, u, v, eid):
    """EDGE_UDF over the triggered edges (scheduler.py:572-583)."""
    if is_iterable(func):
        func = BundledFunction(func)
    fn = var.FUNC(lambda src, edata, dst: func(EdgeBatch(g, (u, v, eid), src, edata, dst)),
                  "edge_func")
    return ir.EDGE_UDF(fn, *_edge_vars(g, u, v, eid))


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


def _all_nodes(g, recv_nodes):
    """Receiver ids; None stands for every node (update_all), whose id list is
    made only when a UDF or fallback reducer needs it: the kernel path of a
    whole-graph update_all touches no O(N) host array."""
    if recv_nodes is None:
        return torch.arange(g.number_of_nodes(), dtype=torch.int64)
    return recv_nodes


def _bucket_fn(g, rfunc, recv_nodes, msg_dst):
    return var.FUNC(lambda msgs: degree_bucketing.bucket_reduce(
        g, rfunc, _all_nodes(g, recv_nodes), msg_dst, msgs, g._node_frame), "reduce_func")


def _builtin_over_messages(g, rfn, msgs, inc, recv_nodes, msg_dst, out, msg_eid=None):
    """A builtin reducer over materialised messages: SPMV_E2V (copy_e over the
    incidence matrix), or degree bucketing when the messages are not float32.
    ``msg_eid``: ``msgs`` is the whole message frame and the incidence
    matrix's columns are edge ids (build_inc_eid); the fallback then takes the
    rows of those edges."""
    def check():
        if rfn.msg_field not in msgs.data:
            raise DGLError('Reduce function requires message field "%s", but no message '
                           'function generates it.' % rfn.msg_field)
    ir.CALL_(var.FUNC(check, "check_msg"))
    m = ir.READ_COL(msgs, var.STR(rfn.msg_field))
    fallback = var.FUNC(lambda mt: degree_bucketing.bucket_reduce(
        g, rfn, _all_nodes(g, recv_nodes), msg_dst,
        {rfn.msg_field: mt if msg_eid is None else mt[msg_eid.to(mt.device)]},
        g._node_frame)[rfn.out_field],
        "bucket_" + rfn.name)
    r = ir.SPMV_E2V(inc, m, var.STR(rfn.kernel_reduce), fallback)
    ir.WRITE_COL_(out, var.STR(rfn.out_field), r)


def _send_reduce(g, mfunc, rfunc, edges, recv_nodes, whole_graph):
    """Issue the send + reduce; returns the FEAT_DICT variable of the reduced
    features (rows = recv_nodes)."""
    nf, ef = g._node_frame, g._edge_frame
    nf_var, ef_var = var.FEAT_DICT(nf, "nf"), var.FEAT_DICT(ef, "ef")
    mfunc = _standardize(mfunc, "message")
    rfunc = _standardize(rfunc, "reduce")
    out = ir.NEW_DICT()
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
        spmat = var.SPMAT(adjacency, "adj")
        for mfn, rfn in pairs:
            red = var.STR(rfn.kernel_reduce)
            if mfn.kernel_msg == "copy_u":
                r = ir.SPMV(spmat, ir.READ_COL(nf_var, var.STR(mfn.src_field)), red)
            elif mfn.kernel_msg == "u_mul_e":
                r = ir.SPMV_WITH_DATA(spmat, ir.READ_COL(ef_var, var.STR(mfn.edge_field)),
                                      ir.READ_COL(nf_var, var.STR(mfn.src_field)), red)
            else:  # copy_e over the adjacency: edge values by the slots' edge ids
                r = ir.SPMV_E2V(spmat, ir.READ_COL(ef_var, var.STR(mfn.edge_field)), red)
            ir.WRITE_COL_(out, var.STR(rfn.out_field), r)
        if not mfunc:
            return out
    u, v, eid = edges.get()
    msgs = _edge_udf(g, mfunc, u, v, eid)
    if is_iterable(rfunc):
        if whole_graph:
            inc = var.SPMAT(lambda dev: g._graph.incidence_in(dev), "inc")
        else:
            inc = var.SPMAT(lambda dev: spmv.build_inc_dst(v, recv_nodes, dev), "inc")
        for rfn in rfunc:
            _builtin_over_messages(g, rfn, msgs, inc, recv_nodes, v, out)
        return out
    return ir.UPDATE_DICT(out, ir.DEGREE_BUCKETING(_bucket_fn(g, rfunc, recv_nodes, v), msgs))


def _apply_with_accum(g, nodes, reduced, apply_func):
    """Apply function over node data updated with the reduced values."""
    if not apply_func:
        return reduced
    ids = _all_nodes(g, nodes)
    data = ir.UPDATE_DICT(ir.READ_ROW(var.FEAT_DICT(g._node_frame, "nf"), var.IDX(nodes)),
                          reduced)
    fn = var.FUNC(lambda nd: apply_func(NodeBatch(g, ids, nd)), "apply_func")
    return ir.UPDATE_DICT(reduced, ir.NODE_UDF(fn, data))


def _write_rows(g, rows, final, inplace):
    nf_var = var.FEAT_DICT(g._node_frame, "nf")
    if inplace:
        ir.WRITE_ROW_INPLACE_(nf_var, var.IDX(rows), final)
    else:
        ir.WRITE_ROW_(nf_var, var.IDX(rows), final)


@_program
def schedule_update_all(g, message_func, reduce_func, apply_func):
    """update_all: send on every edge, reduce at every node."""
    if g.number_of_edges() == 0:
        if apply_func is not None:
            _apply_nodes(g, None, apply_func, inplace=False)
        return
    edges = _Edges(g._graph.edges)
    reduced = _send_reduce(g, message_func, reduce_func, edges, None, True)
    final = _apply_with_accum(g, None, reduced, apply_func)
    ir.WRITE_DICT_(var.FEAT_DICT(g._node_frame, "nf"), final)


def _snr(g, u, v, eid, message_func, reduce_func, apply_func, inplace):
    recv = torch.unique(v, sorted=True)
    reduced = _send_reduce(g, message_func, reduce_func, _Edges(lambda: (u, v, eid)), recv,
                           False)
    _write_rows(g, recv, _apply_with_accum(g, recv, reduced, apply_func), inplace)


@_program
def schedule_snr(g, u, v, eid, message_func, reduce_func, apply_func, inplace):
    """send_and_recv on the given edges."""
    _snr(g, u, v, eid, message_func, reduce_func, apply_func, inplace)


@_program
def schedule_pull(g, pull_nodes, message_func, reduce_func, apply_func, inplace):
    """pull: receivers are ``pull_nodes`` (including ones without in-edges)."""
    u, v, eid = g._graph.in_edges(pull_nodes)
    if len(eid) == 0:
        if apply_func is not None:
            _apply_nodes(g, pull_nodes, apply_func, inplace)
        return
    recv = torch.unique(pull_nodes, sorted=True)
    reduced = _send_reduce(g, message_func, reduce_func, _Edges(lambda: (u, v, eid)), recv,
                           False)
    _write_rows(g, recv, _apply_with_accum(g, recv, reduced, apply_func), inplace)


@_program
def schedule_push(g, push_nodes, message_func, reduce_func, apply_func, inplace):
    """push: send_and_recv along the out-edges of ``push_nodes``."""
    u, v, eid = g._graph.out_edges(push_nodes)
    if len(eid) == 0:
        return
    _snr(g, u, v, eid, message_func, reduce_func, apply_func, inplace)


@_program
def schedule_send(g, u, v, eid, message_func):
    """send: materialise messages into the message frame (scheduler.py:26-56)."""
    msgs = _edge_udf(g, _standardize(message_func, "message"), u, v, eid)
    ir.WRITE_ROW_(var.FEAT_DICT(g._msg_frame, "mf"), var.IDX(eid), msgs)

    def mark():
        g._msg_pending[eid] = True
    ir.CALL_(var.FUNC(mark, "mark_pending"))


@_program
def schedule_recv(g, recv_nodes, reduce_func, apply_func, inplace):
    """recv: reduce pending messages on the in-edges of ``recv_nodes``."""
    src, dst, eid = g._graph.in_edges(recv_nodes)
    if len(eid):
        keep = g._msg_pending[eid]
        src, dst, eid = src[keep], dst[keep], eid[keep]
    if len(eid) == 0:
        if apply_func is not None:
            _apply_nodes(g, recv_nodes, apply_func, inplace)
        return
    recv = torch.unique(recv_nodes, sorted=True)
    rfunc = _standardize(reduce_func, "reduce")
    out = ir.NEW_DICT()
    if is_iterable(rfunc):
        # the reference's e2v route (scheduler.py:451-456): incidence by edge id
        # over the whole message frame, read in place
        mf = var.FEAT_DICT(g._msg_frame, "mf")
        m = g._msg_frame.num_rows
        inc = var.SPMAT(lambda dev: spmv.build_inc_eid(m, eid, dst, recv, dev), "inc")
        for rfn in rfunc:
            _builtin_over_messages(g, rfn, mf, inc, recv, dst, out, msg_eid=eid)
    else:
        msgs = ir.READ_ROW(var.FEAT_DICT(g._msg_frame, "mf"), var.IDX(eid))
        out = ir.UPDATE_DICT(out, ir.DEGREE_BUCKETING(_bucket_fn(g, rfunc, recv, dst), msgs))
    _write_rows(g, recv, _apply_with_accum(g, recv, out, apply_func), inplace)

    def consume():
        g._msg_pending[eid] = False
        if not bool(g._msg_pending.any()):
            g._msg_frame.clear()
    ir.CALL_(var.FUNC(consume, "consume_pending"))


def _apply_nodes(g, v, apply_func, inplace):
    ids = _all_nodes(g, v)
    fn = var.FUNC(lambda nd: apply_func(NodeBatch(g, ids, nd)), "apply_func")
    out = ir.NODE_UDF(fn, ir.READ_ROW(var.FEAT_DICT(g._node_frame, "nf"), var.IDX(v)))
    _write_rows(g, v, out, inplace)


@_program
def schedule_apply_nodes(g, v, apply_func, inplace):
    """apply_nodes over ``v`` (None = all nodes)."""
    _apply_nodes(g, v, apply_func, inplace)


@_program
def schedule_apply_edges(g, u, v, eid, apply_func, inplace):
    """apply_edges over the given edges (``eid`` None = all edges)."""
    if eid is None:
        u, v, eid = g._graph.edges()
        rows = None
    else:
        rows = eid
    out = _edge_udf(g, apply_func, u, v, eid)
    ef_var = var.FEAT_DICT(g._edge_frame, "ef")
    if inplace:
        ir.WRITE_ROW_INPLACE_(ef_var, var.IDX(rows), out)
    else:
        ir.WRITE_ROW_(ef_var, var.IDX(rows), out)
