"""Degree bucketing for user-defined reduce functions.

Counterpart of python/dgl/runtime/degree_bucketing.py:13-190 and the native
``sched::DegreeBucketing`` (src/scheduler/scheduler.cc:13-93): receiving
nodes are grouped by in-degree so each bucket's mailbox is a dense
(n_bucket, degree, *feat) tensor the UDF can reduce over dim 1. A node's
messages appear in the order of the triggered edge list (scheduler.cc:22-33
appends message ids per destination in edge order). Buckets are processed in
ascending degree and the results are merged back in receiving-node order
(MERGE_ROW, executor.py:600-663); receiving nodes without messages get the
frame initializer's value (degree_bucketing.py:72-78).

Builtin reducers never come here: they run as g-SpMM kernels. The bucket
schedule itself is computed natively (dglhip_degree_bucketing_host).
"""
from __future__ import absolute_import

import ctypes

import torch

from .._ffi import LIB, check_call, ptr
from ..udf import NodeBatch

__all__ = ["bucket_reduce"]


def bucket_reduce(g, reduce_udf, recv_nodes, msg_dst, msgs, node_frame):
    """Run ``reduce_udf`` over degree buckets.

    recv_nodes : sorted unique node ids (CPU int64) receiving the reduction
    msg_dst    : destination node of every message (CPU int64, message order)
    msgs       : dict of message tensors, first dim = len(msg_dst)
    returns    : dict of reduced features, first dim = len(recv_nodes)
    """
    n_recv = len(recv_nodes)
    pos = torch.searchsorted(recv_nodes, msg_dst).contiguous()
    n_msgs = pos.numel()
    nb = ctypes.c_int64()
    bdeg = torch.empty(max(n_recv, 1), dtype=torch.int64)
    bptr = torch.empty(n_recv + 1, dtype=torch.int64)
    bnodes = torch.empty(max(n_recv, 1), dtype=torch.int64)
    mids_all = torch.empty(max(n_msgs, 1), dtype=torch.int64)
    check_call(LIB.dglhip_degree_bucketing_host(n_msgs, ptr(pos), n_recv, ctypes.byref(nb),
                                                ptr(bdeg), ptr(bptr), ptr(bnodes),
                                                ptr(mids_all)))
    results = {}
    positions = []
    outs = []
    moff = 0
    for b in range(nb.value):
        d = int(bdeg[b])
        members = bnodes[int(bptr[b]):int(bptr[b + 1])]
        mids = mids_all[moff:moff + d * len(members)]
        moff += d * len(members)
        nodes = recv_nodes[members]
        mailbox = {}
        for k, t in msgs.items():
            sel = t.index_select(0, mids.to(t.device))
            mailbox[k] = sel.reshape((len(members), d) + tuple(t.shape[1:]))
        data = node_frame.select_rows(nodes)
        out = reduce_udf(NodeBatch(g, nodes, data, mailbox))
        positions.append(members)
        outs.append(out)
    if not outs:
        return results
    has_msg = torch.zeros(n_recv, dtype=torch.bool)
    has_msg[bnodes[:int(bptr[nb.value])]] = True
    zero_deg = (~has_msg).nonzero(as_tuple=True)[0]
    allpos = torch.cat(positions + [zero_deg])
    inv = torch.empty_like(allpos)
    inv[allpos] = torch.arange(len(allpos))
    for key in outs[0].keys():
        parts = [o[key] for o in outs]
        ref = parts[0]
        if len(zero_deg):
            init = node_frame.get_initializer(key)
            fill = init((len(zero_deg),) + tuple(ref.shape[1:]), ref.dtype, ref.device,
                        slice(0, len(zero_deg)))
            parts.append(fill.to(ref.device))
        cat = torch.cat(parts, 0)
        results[key] = cat.index_select(0, inv.to(cat.device))
    return results
