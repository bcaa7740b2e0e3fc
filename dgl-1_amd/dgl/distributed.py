"""Full-graph message passing sharded by a 1-D node partition (new design).

The reference has no multi-device code at all. This module
adds the north star's scale-out path: destination rows are split into P
contiguous ranges balanced by in-edge count, one process per GPU
(torch.distributed over RCCL / xGMI, gloo on CPU for tests).

* Forward of update_all(copy_src, sum): halo exchange of the source rows,
  then the local g-SpMM over the rank's rows. For power-law graphs whose
  halo covers most nodes (Reddit-/RMAT-shaped: SURVEY.md §8e) the exchange
  is one all-gather of the row-padded feature blocks
  (``all_gather_into_tensor``, a ring over the xGMI links).
* Backward: the all-gather's adjoint, a reduce-scatter (sum) of the source
  gradients produced by the local transposed g-SpMM.

Column ids of the local CSR are remapped once (at partition time) from global
node ids to positions in the padded all-gather buffer, so the kernel runs
unchanged. Row results are bit-identical to the single-GPU product: each
local row accumulates exactly the same edges in the same edge-id order.

Pipelined forward (``pipeline_chunks = C > 0``, inference / benchmarking):
each row's slots are grouped into segments — sources this rank owns first,
then the remote sources of halo chunk 1..C — so the own segment is reduced
while the halo is still in flight, and each remote segment as soon as its
chunk's all-gather (on a separate HIP stream) lands. The row's fma chain is
continued segment by segment (dglhip_gspmm_ranges_device, accumulate), so
the result is one sequential chain in (segment, edge-id) order: deterministic
and within fp32 tolerance of the edge-id-order chain (bit-identical when edge
ids already run in source order, as in bench.py's graphs).
"""
from __future__ import absolute_import

import torch
import torch.distributed as dist

from . import kernel

__all__ = ["balanced_bounds", "PartitionedGraph"]


def balanced_bounds(in_degrees, num_parts):
    """Contiguous destination-row ranges with ~equal in-edge counts:
    int64[P+1] boundaries over node ids."""
    deg = torch.as_tensor(in_degrees, dtype=torch.int64).cpu()
    n = deg.numel()
    cum = torch.cumsum(deg, 0)
    total = int(cum[-1]) if n else 0
    bounds = [0]
    for p in range(1, num_parts):
        target = total * p // num_parts
        b = int(torch.searchsorted(cum, torch.tensor(target), right=True)) if n else 0
        bounds.append(max(bounds[-1], min(b, n)))
    bounds.append(n)
    return torch.tensor(bounds, dtype=torch.int64)


class _AllGatherRows(torch.autograd.Function):
    """Padded row blocks of every rank -> one (P * max_rows, F) tensor."""

    @staticmethod
    def forward(ctx, h_local, max_rows, group):
        ctx.group = group
        ctx.n_local = h_local.shape[0]
        ctx.max_rows = max_rows
        world = dist.get_world_size(group)
        pad = h_local.new_zeros((max_rows,) + tuple(h_local.shape[1:]))
        pad[:h_local.shape[0]] = h_local
        full = h_local.new_empty((world * max_rows,) + tuple(h_local.shape[1:]))
        dist.all_gather_into_tensor(full, pad.contiguous(), group=group)
        return full

    @staticmethod
    def backward(ctx, dfull):
        out = dfull.new_empty((ctx.max_rows,) + tuple(dfull.shape[1:]))
        dist.reduce_scatter_tensor(out, dfull.contiguous(), op=dist.ReduceOp.SUM, group=ctx.group)
        return out[:ctx.n_local], None, None


class PartitionedGraph(object):
    """This rank's shard of a graph for full-graph message passing.

    Parameters
    ----------
    num_nodes : global node count
    src, dst  : the rank's edges (dst inside its range), global ids, in
                global edge-id order (the order kept inside each CSR row)
    bounds    : int64[P+1] row ranges (balanced_bounds)
    device    : where the shard lives
    group     : torch.distributed process group (default world)
    """

    def __init__(self, num_nodes, src, dst, bounds, device, group=None, pipeline_chunks=0,
                 rank=None, world=None):
        self.group = group
        # explicit rank/world: single-process studies of one rank's share (no collectives)
        self.rank = dist.get_rank(group) if rank is None else int(rank)
        self.world = dist.get_world_size(group) if world is None else int(world)
        self._emulated = rank is not None
        self.bounds = torch.as_tensor(bounds, dtype=torch.int64).cpu()
        self.lo = int(self.bounds[self.rank])
        self.hi = int(self.bounds[self.rank + 1])
        self.num_nodes = int(num_nodes)
        self.num_local = self.hi - self.lo
        self.max_rows = int((self.bounds[1:] - self.bounds[:-1]).max())
        device = torch.device(device)
        src = torch.as_tensor(src, dtype=torch.int64).to(device)
        dst = torch.as_tensor(dst, dtype=torch.int64).to(device)
        b = self.bounds.to(device)
        owner = torch.searchsorted(b, src, right=True) - 1
        cols = owner * self.max_rows + (src - b[owner])
        self.num_edges = int(src.numel())
        self.device = device
        self.chunks = int(pipeline_chunks)
        if self.chunks > 0:
            self._build_pipeline(src, dst, b, owner)
            self.adj = None
        else:
            self.adj = kernel.from_coo(self.num_local, self.world * self.max_rows,
                                       dst - self.lo, cols, kernel.ORDER_EID, device)

    def _build_pipeline(self, src, dst, b, owner):
        C, P, R = self.chunks, self.world, self.num_local
        cr = -(-self.max_rows // C)  # rows per halo chunk
        self.chunk_rows = cr
        j = src - b[owner]                      # index inside the owner's block
        c = j // cr
        own = owner == self.rank
        # own sources index h_local directly; remote ones the chunked halo buffer
        cols = torch.where(own, j, c * (P * cr) + owner * cr + (j - c * cr))
        seg = torch.where(own, torch.zeros_like(c), c + 1)
        S = C + 1
        vrow = (dst - self.lo) * S + seg
        csr = kernel.build_csr(R * S, max(P * cr * C, R), vrow, cols, kernel.ORDER_EID,
                               self.device, schedule=False)
        ip = csr.indptr
        self.seg_ranges = [(ip[s:R * S:S].contiguous(), ip[s + 1:R * S + 1:S].contiguous())
                           for s in range(S)]
        self.pipe_csr = csr
        self.halo = None
        # overlap needs an asynchronous collective backend (RCCL); gloo runs inline
        overlap = (not self._emulated and self.device.type == "cuda"
                   and dist.get_backend(self.group) == "nccl")
        self.comm_stream = torch.cuda.Stream(self.device) if overlap else None

    def gather_halo(self, h_local):
        """All-gather of the padded row blocks (RCCL all_gather_into_tensor)."""
        return _AllGatherRows.apply(h_local, self.max_rows, self.group)

    def update_all(self, h_local, msg="copy_u", reduce="sum", efeat=None):
        """Local rows of update_all(msg, reduce) given this rank's node features."""
        if self.chunks > 0:
            if msg != "copy_u" or reduce != "sum" or h_local.requires_grad:
                raise ValueError("the pipelined forward covers copy_u + sum without autograd")
            return self._pipelined_copy_sum(h_local)
        full = self.gather_halo(h_local)
        return kernel.gspmm(self.adj, msg, reduce, full, efeat)

    def _pipelined_copy_sum(self, h_local):
        C, P, cr = self.chunks, self.world, self.chunk_rows
        F = h_local.shape[1]
        dev = self.device
        if self.halo is None or self.halo.shape[1] != F:
            self.halo = torch.empty(C * P * cr, F, device=dev)
            self.hpad = torch.zeros(C * cr, F, device=dev)
        self.hpad[:self.num_local].copy_(h_local)
        out = torch.empty(self.num_local, F, device=dev)
        ind = self.pipe_csr.indices
        beg, end = self.seg_ranges[0]
        events = []
        if self.comm_stream is not None:
            ready = torch.cuda.Event()
            ready.record()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ready)
                for c in range(C):
                    dist.all_gather_into_tensor(self.halo[c * P * cr:(c + 1) * P * cr],
                                                self.hpad[c * cr:(c + 1) * cr],
                                                group=self.group)
                    ev = torch.cuda.Event()
                    ev.record(self.comm_stream)
                    events.append(ev)
        # own sources while the halo is in flight
        kernel.gspmm_ranges("copy_u", beg, end, False, ind, out, ufeat=h_local.contiguous())
        for c in range(C):
            if self.comm_stream is not None:
                torch.cuda.current_stream(dev).wait_event(events[c])
            elif not self._emulated:
                dist.all_gather_into_tensor(self.halo[c * P * cr:(c + 1) * P * cr],
                                            self.hpad[c * cr:(c + 1) * cr], group=self.group)
            beg, end = self.seg_ranges[c + 1]
            kernel.gspmm_ranges("copy_u", beg, end, True, ind, out, ufeat=self.halo)
        if self.comm_stream is not None:
            self.halo.record_stream(torch.cuda.current_stream(dev))
        return out
