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
* Graphs with locality (halo below half of N) use a sparse
  halo instead: each rank receives only the remote rows its CSR references,
  one all-to-allv (``all_to_all_single`` with split sizes) per layer; the
  backward is the reverse all-to-allv with sum-on-receive. The request lists
  are exchanged once, at partition time. ``halo="auto"`` takes the
  all-to-allv when it at least halves what a rank receives: the largest rank
  halo against the (P-1) padded blocks of an all-gather (one all-reduce MAX,
  so every rank decides alike). RMAT graphs land here: half their vertices
  have no out-edges, and a rank's halo is about 0.2 N at P = 2..8, against
  (P-1)/P N for the all-gather; Reddit-like graphs reference almost every node
  and keep the all-gather.

Column ids of the local CSR are remapped once (at partition time) from global
node ids to positions in the padded all-gather buffer, so the kernel runs
unchanged. Row results are bit-identical to the single-GPU product: each
local row accumulates exactly the same edges in the same edge-id order.

Pipelined path (``pipeline_chunks = C > 0``, copy_u with sum or mean,
differentiable: _PipelinedAggregate). With the all-to-allv halo, every peer's request list is cut into C parts and
the exchange runs as C all-to-allv calls on a side stream: the own sources are
reduced while chunk 1 is in flight, and the received rows of chunk c as soon
as it lands, so only the last chunk's rows are reduced after the exchange
ends (with one exchange, the whole halo segment ran after it). With the all-gather:
each row's slots are grouped into segments — sources this rank owns first,
then the remote sources of halo chunk 1..C — so the own segment is reduced
while the halo is still in flight, and each remote segment as soon as its
chunk's all-gather (on a separate HIP stream) lands. The row's fma chain is
continued segment by segment: each segment is a CSR of its own, reduced with
DGLHIP_REDUCE_SUM_ACCUM (out += ..., the chain continuing from out), so it
keeps the degree-descending schedule and heavy-row chunking of a plain
g-SpMM. The result is one sequential chain in (segment, edge-id) order:
deterministic and within fp32 tolerance of the edge-id-order chain
(bit-identical when edge ids already run in source order, as in bench.py's
graphs, and no row is chunked). The backward runs the segments' transposes:
each halo chunk's gradient rows are computed and sent back to their owners
(reduce-scatter of the chunk's landing rows / reverse all-to-allv) on the
comm stream while the next chunk's transposed product runs, and the own
segment's product overlaps the last exchange; the received gradients are
then added in chunk (and peer) order, so the result is deterministic.
"""
from __future__ import absolute_import

import torch
import torch.distributed as dist

from . import kernel

__all__ = ["balanced_bounds", "PartitionedGraph"]


def _pack(x, halo_dtype):
    """Feature rows as sent over the wire: fp32 as they are, or rounded to
    bf16 and carried as a float16 view (the collectives only move these bytes;
    every backend takes float16, not all take bfloat16)."""
    if halo_dtype is None:
        return x
    return x.to(halo_dtype).view(torch.float16)


def _unpack(x, halo_dtype):
    if halo_dtype is None:
        return x
    return x.view(halo_dtype).float()


def _chunk_parts(lengths, C):
    """Split each of P lists (lengths int64[P]) into C consecutive parts of
    near-equal size: int64[C+1, P] start offsets inside each list. Both ends
    of an all-to-allv compute the same split from the same length."""
    lengths = torch.as_tensor(lengths, dtype=torch.int64).cpu()
    c = torch.arange(C + 1, dtype=torch.int64).unsqueeze(1)
    return (lengths.unsqueeze(0) * c) // C


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
    """Padded row blocks of every rank -> one (P * max_rows, F) tensor. The
    gradients go back in fp32 (a reduce-scatter sums them)."""

    @staticmethod
    def forward(ctx, h_local, max_rows, group, halo_dtype=None):
        ctx.group = group
        ctx.n_local = h_local.shape[0]
        ctx.max_rows = max_rows
        world = dist.get_world_size(group)
        pad = h_local.new_zeros((max_rows,) + tuple(h_local.shape[1:]))
        pad[:h_local.shape[0]] = h_local
        pad = _pack(pad, halo_dtype).contiguous()
        full = pad.new_empty((world * max_rows,) + tuple(pad.shape[1:]))
        dist.all_gather_into_tensor(full, pad, group=group)
        return _unpack(full, halo_dtype)

    @staticmethod
    def backward(ctx, dfull):
        out = dfull.new_empty((ctx.max_rows,) + tuple(dfull.shape[1:]))
        dist.reduce_scatter_tensor(out, dfull.contiguous(), op=dist.ReduceOp.SUM, group=ctx.group)
        return out[:ctx.n_local], None, None, None


class _AllToAllRows(torch.autograd.Function):
    """Sparse halo: rows h_local[send_idx] go to their requesting ranks
    (send_splits), the rows this rank requested come back in owner order
    (recv_splits). Backward: reverse all-to-allv of the fp32 gradients, then
    sum-on-receive one peer at a time (indices are unique within a peer, so
    the adds are ordered)."""

    @staticmethod
    def forward(ctx, h_local, send_idx, send_splits, recv_splits, group, halo_dtype=None):
        ctx.save_for_backward(send_idx)
        ctx.splits = (send_splits, recv_splits)
        ctx.group = group
        ctx.n_local = h_local.shape[0]
        ctx.halo_dtype = halo_dtype
        tail = tuple(h_local.shape[1:])
        send = _pack(h_local.index_select(0, send_idx), halo_dtype).contiguous()
        recv = send.new_empty((sum(recv_splits),) + tail)
        dist.all_to_all_single(recv, send, recv_splits, send_splits, group=group)
        return _unpack(recv, halo_dtype)

    @staticmethod
    def backward(ctx, drecv):
        send_idx, = ctx.saved_tensors
        send_splits, recv_splits = ctx.splits
        tail = tuple(drecv.shape[1:])
        # gradients travel in fp32 whatever the forward's wire type, as in the
        # all-gather mode's reduce-scatter (halo_dtype rounds features only)
        wire = drecv.float().contiguous()
        dsend = wire.new_empty((sum(send_splits),) + tail)
        dist.all_to_all_single(dsend, wire, send_splits, recv_splits, group=ctx.group)
        dh = drecv.new_zeros((ctx.n_local,) + tail)
        off = 0
        for n in send_splits:
            if n:
                dh.index_add_(0, send_idx[off:off + n], dsend[off:off + n])
            off += n
        return dh, None, None, None, None, None


class _PipelinedAggregate(torch.autograd.Function):
    """update_all(copy_u, sum | mean) over a PartitionedGraph with the halo
    exchange cut into chunks and overlapped with the local g-SpMM segments,
    in both directions (full-graph training at N > 1, the layer of
    examples/pytorch/gcn/gcn_spmv.py:45-62 sharded; its backward is
    SURVEY.md §3.2's dH = Aᵀ·dC).

    Forward: PartitionedGraph._pipelined_* (own segment while the exchange
    is in flight, each chunk's segment as it lands), then the mean's divisor.
    Backward: each halo chunk's transposed product, returned to the owners
    (reduce-scatter / reverse all-to-allv on the comm stream) while the next
    chunk's product runs; the own segment's transposed product overlaps the
    last exchange; the received gradients are added in chunk order."""

    @staticmethod
    def forward(ctx, h_local, pg, mean, add_to=None):
        out = pg._pipelined_sum(h_local.detach())
        if add_to is not None:
            # add_to + sum / deg in one pass (addcdiv: the quotient, then the
            # sum of two terms -- the bits of add_to + (sum / deg))
            add_to.addcdiv_(out, pg._mean_divisor(out.dtype))
            ctx.mark_dirty(add_to)
            out = add_to
        elif mean:
            out = out / pg._mean_divisor(out.dtype)
        ctx.pg, ctx.mean = pg, mean or add_to is not None
        ctx.has_add = add_to is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        pg = ctx.pg
        dout = dout.contiguous()
        d_add = dout if (ctx.has_add and ctx.needs_input_grad[3]) else None
        if ctx.mean:
            dout = (dout / pg._mean_divisor(dout.dtype)).contiguous()
        return pg._pipelined_backward(dout), None, None, d_add


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
    halo      : "allgather" (padded row blocks of every rank), "alltoall"
                (only the referenced remote rows) or "auto": alltoall when it
                at least halves what a rank receives, i.e. when
                2 * (largest rank halo) <= (P - 1) * max_rows (the rows of the
                all-gather's P - 1 remote padded blocks), decided by one
                all-reduce MAX so every rank picks the same collective
    halo_dtype: None (fp32 rows, bit-exact results) or torch.bfloat16: remote
                rows travel rounded to bf16, half the exchange volume
                (SURVEY.md §8e); the local reduction stays fp32. Opt-in: the
                rows' results then carry bf16 rounding of the remote inputs.
                Gradients travel in fp32 in every halo mode.
    overlap   : pipelined path only: run the chunk exchanges on a side stream
                that the segments' products wait on by event. None (default):
                with RCCL on a ROCm device; True: also with gloo on a ROCm
                device (gloo orders its device copies against the stream a
                collective is issued on, so the same events and stream
                bookkeeping run as under RCCL: the one-GPU test of that path);
                False: inline on the current stream.
    """

    def __init__(self, num_nodes, src, dst, bounds, device, group=None, pipeline_chunks=0,
                 rank=None, world=None, halo="auto", halo_dtype=None, overlap=None):
        if halo_dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError("halo_dtype must be None, torch.float32 or torch.bfloat16")
        self.halo_dtype = None if halo_dtype == torch.float32 else halo_dtype
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
        self.num_edges = int(src.numel())
        self.device = device
        # in-degree of each local row (all of a row's in-edges live on this
        # rank): the mean reducer's divisor
        self.in_deg = torch.bincount(dst - self.lo, minlength=self.num_local)
        self._seg_t = None  # transposed segment CSRs, built by the first backward
        self.chunks = int(pipeline_chunks)
        self.adj = None
        self.halo = None
        if halo not in ("auto", "allgather", "alltoall"):
            raise ValueError("halo must be auto, allgather or alltoall")
        own = owner == self.rank
        if halo != "allgather":
            need = torch.unique(src[~own])       # sorted global ids = owner order
            if halo == "auto" and self._emulated:  # single-rank study: this rank's halo
                gather_rows = (self.world - 1) * self.max_rows
                halo = "alltoall" if 2 * need.numel() <= gather_rows else "allgather"
            elif halo == "auto":
                # the all-to-allv when it at least halves what a rank receives:
                # largest halo vs the (P-1) padded blocks of an all-gather (one
                # all-reduce MAX, so every rank decides alike)
                top = torch.tensor([need.numel()], dtype=torch.int64, device=self._coll_dev())
                dist.all_reduce(top, op=dist.ReduceOp.MAX, group=group)
                gather_rows = (self.world - 1) * self.max_rows
                halo = "alltoall" if 2 * int(top) <= gather_rows else "allgather"
        self.halo_mode = halo
        self.comm_stream = None
        if halo == "alltoall":
            self._build_alltoall(src, dst, b, owner, own, need)
        elif self.chunks > 0:
            self._build_pipeline(src, dst, b, owner)
        else:
            cols = owner * self.max_rows + (src - b[owner])
            self.adj = kernel.from_coo(self.num_local, self.world * self.max_rows,
                                       dst - self.lo, cols, kernel.ORDER_EID, device)
        if self.chunks > 0:
            if overlap is None:
                # by default only with an asynchronous collective backend (RCCL)
                overlap = (not self._emulated and self.device.type == "cuda"
                           and dist.get_backend(self.group) == "nccl")
            elif overlap and (self._emulated or self.device.type != "cuda"):
                raise ValueError("overlap needs a ROCm device and real peers")
            self.comm_stream = torch.cuda.Stream(self.device) if overlap else None
        elif overlap:
            raise ValueError("overlap applies to the pipelined path (pipeline_chunks > 0)")

    def _coll_dev(self):
        """Device the process group's collectives take tensors on."""
        return self.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")

    def _build_alltoall(self, src, dst, b, owner, own, need):
        P, R = self.world, self.num_local
        bd = b.to(need.device)
        need_owner = torch.searchsorted(bd, need, right=True) - 1
        recv_splits = torch.bincount(need_owner, minlength=P).cpu()
        if self._emulated:  # no peers to ask: only this rank's receive side
            self.send_idx, self.send_splits = None, None
            self.recv_splits = recv_splits.tolist()
            self.num_halo = int(need.numel())
            self._build_alltoall_csrs(src, dst, own, need, need_owner)
            return
        cdev = self._coll_dev()
        # tell every owner how many of its rows this rank needs, then which
        send_splits = torch.empty(P, dtype=torch.int64, device=cdev)
        dist.all_to_all_single(send_splits, recv_splits.to(cdev), group=self.group)
        send_splits = send_splits.cpu()
        req = torch.empty(int(send_splits.sum()), dtype=torch.int64, device=cdev)
        dist.all_to_all_single(req, need.to(cdev), send_splits.tolist(),
                               recv_splits.tolist(), group=self.group)
        self.send_idx = (req.to(self.device) - self.lo).contiguous()
        self.send_splits = send_splits.tolist()
        self.recv_splits = recv_splits.tolist()
        self.num_halo = int(need.numel())
        if self.chunks > 0:
            # chunk c of the rows sent to peer q: part c of q's request list
            parts = _chunk_parts(send_splits, self.chunks)
            starts = torch.cumsum(send_splits, 0) - send_splits
            idx = []
            for c in range(self.chunks):
                sel = [self.send_idx[int(starts[q] + parts[c, q]):int(starts[q] + parts[c + 1, q])]
                       for q in range(P)]
                idx.append(torch.cat(sel).contiguous())
            self.chunk_send_idx = idx
            self.chunk_send_splits = (parts[1:] - parts[:-1]).tolist()
        self._build_alltoall_csrs(src, dst, own, need, need_owner)

    def _build_alltoall_csrs(self, src, dst, own, need, need_owner):
        R = self.num_local
        pos = torch.searchsorted(need, src)
        if self.chunks > 0:
            # pipelined forward: own sources (columns of h_local) reduced while the
            # exchange is in flight, then the rows of halo chunk 1..C (columns of
            # that chunk's receive buffer) continue each row's chain
            C, P = self.chunks, self.world
            lens = torch.as_tensor(self.recv_splits, dtype=torch.int64)
            parts = _chunk_parts(lens, C)                       # [C+1, P]
            self.chunk_recv_splits = (parts[1:] - parts[:-1]).tolist()
            # need entry i: owner p, offset j in p's list -> chunk, slot in chunk buffer
            first = (torch.cumsum(lens, 0) - lens).to(need.device)
            j = torch.arange(need.numel(), device=need.device) - first[need_owner]
            pd = parts.to(need.device)
            chunk = (j.unsqueeze(0) >= pd[1:-1, need_owner]).sum(0) if C > 1 else \
                torch.zeros_like(j)
            sizes = parts[1:] - parts[:-1]                      # [C, P]
            base = (torch.cumsum(sizes, 1) - sizes).to(need.device)  # chunk buffer offsets
            slot = base[chunk, need_owner] + (j - pd[chunk, need_owner])
            lrow = dst - self.lo
            rem = ~own
            seg_of = chunk[pos[rem]]
            cols = slot[pos[rem]]
            self.seg_csrs = [kernel.build_csr(R, R, lrow[own], (src - self.lo)[own],
                                              kernel.ORDER_EID, self.device)]
            for c in range(C):
                m = seg_of == c
                self.seg_csrs.append(kernel.build_csr(
                    R, max(int(sizes[c].sum()), 1), lrow[rem][m], cols[m], kernel.ORDER_EID,
                    self.device))
        else:
            # columns: own sources -> [0, R), remote -> R + position in `need`
            cols = torch.where(own, src - self.lo, R + pos)
            self.adj = kernel.from_coo(R, R + self.num_halo, dst - self.lo, cols,
                                       kernel.ORDER_EID, self.device)

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
        # one CSR per segment (standard rows: degree-descending schedule and,
        # under kernel.set_row_split, heavy rows chunked), edge order kept
        lrow = dst - self.lo
        self.seg_csrs = []
        for sidx in range(C + 1):
            m = seg == sidx
            ncols = R if sidx == 0 else P * cr * C  # h_local / the halo buffer
            self.seg_csrs.append(kernel.build_csr(R, ncols, lrow[m], cols[m], kernel.ORDER_EID,
                                                  self.device))
            del m
        self.halo = None

    def gather_halo(self, h_local):
        """Source rows the local CSR's columns index: all-gather of the padded
        row blocks (RCCL all_gather_into_tensor), or [h_local | requested remote
        rows] through one all-to-allv."""
        if self.halo_mode == "alltoall":
            recv = _AllToAllRows.apply(h_local, self.send_idx, self.send_splits,
                                       self.recv_splits, self.group, self.halo_dtype)
            return torch.cat([h_local, recv], 0)
        full = _AllGatherRows.apply(h_local, self.max_rows, self.group, self.halo_dtype)
        if self.halo_dtype is not None:
            # the own block stays exact: splice the local rows back in
            lo = self.rank * self.max_rows
            full = torch.cat([full[:lo], h_local, full[lo + self.num_local:]], 0)
        return full

    def set_halo_dtype(self, halo_dtype):
        """Switch the wire type of remote rows (None / torch.float32 or
        torch.bfloat16); landing buffers are reallocated on the next call."""
        if halo_dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError("halo_dtype must be None, torch.float32 or torch.bfloat16")
        if self._emulated:
            raise ValueError("an emulated rank keeps the halo_dtype it was built with")
        self.halo_dtype = None if halo_dtype == torch.float32 else halo_dtype
        self.halo = None

    def update_all(self, h_local, msg="copy_u", reduce="sum", efeat=None):
        """Local rows of update_all(msg, reduce) given this rank's node features.

        Pipelined (pipeline_chunks > 0): copy_u with sum or mean, differentiable
        in h_local; the backward overlaps each chunk's reverse exchange with the
        next chunk's transposed g-SpMM (_PipelinedAggregate)."""
        if self.chunks > 0:
            if msg not in ("copy_u", "copy_src") or reduce not in ("sum", "mean"):
                raise ValueError("the pipelined path covers copy_u with sum or mean")
            if efeat is not None:
                raise ValueError("copy_u takes no edge features")
            return _PipelinedAggregate.apply(h_local, self, reduce == "mean")
        full = self.gather_halo(h_local)
        return kernel.gspmm(self.adj, msg, reduce, full, efeat)

    def mean_add(self, h_local, out):
        """out <- out + update_all(h_local, copy_u, mean), in place and
        differentiable in h_local: the bits of that sum of two tensors, without
        a pass of its own (the pipelined path adds in the mean's division, the
        exchanged one in the g-SpMM's store: kernel.gspmm_mean_add). GraphSAGE's
        fc_self(h) + mean(...) (nn.pytorch.sage_dense's ``add_into``)."""
        if self.chunks > 0:
            return _PipelinedAggregate.apply(h_local, self, True, out)
        return kernel.gspmm_mean_add(self.adj, self.gather_halo(h_local), out)

    def _pipelined_sum(self, h_local):
        if self.halo_mode == "alltoall":
            return self._pipelined_alltoall_sum(h_local)
        return self._pipelined_copy_sum(h_local)

    def _mean_divisor(self, dtype):
        d = getattr(self, "_deg_f", None)
        if d is None or d.dtype != dtype:
            d = self._deg_f = self.in_deg.clamp(min=1).to(dtype).unsqueeze(1)
        return d

    def _transposed_segments(self):
        """Per segment of the pipelined forward, the CSR of its transpose: rows
        are the segment's source rows (h_local for the own segment; one
        chunk's landing rows for a halo segment, rebased to the chunk), slots
        in the forward's edge order (kernel.coo_of recovers it)."""
        if self._seg_t is None:
            R, C = self.num_local, self.chunks
            segs = []
            for i, csr in enumerate(self.seg_csrs):
                row, col = kernel.coo_of(csr)
                if i == 0:
                    base, nrows = 0, R
                elif self.halo_mode == "alltoall":
                    base, nrows = 0, sum(self.chunk_recv_splits[i - 1])
                else:
                    cw = self.world * self.chunk_rows  # landing rows of one chunk
                    base, nrows = (i - 1) * cw, cw
                segs.append(kernel.build_csr(max(nrows, 1), R, col - base, row,
                                             kernel.ORDER_EID, self.device))
                del row, col
            self._seg_t = segs
        return self._seg_t

    def _pipelined_backward(self, dout):
        """dh_local for d(out) = dout: every segment's transposed product, the
        halo chunks' gradients returned to their owners (reduce-scatter of the
        chunk's landing rows, or the reverse all-to-allv then sum-on-receive
        one peer at a time), the own segment reduced while they travel.
        Gradients travel in fp32 whatever the forward's wire type."""
        if self._emulated:
            raise ValueError("an emulated rank has no peers to return gradients to")
        R, C, P = self.num_local, self.chunks, self.world
        F = dout.shape[1]
        dev = self.device
        segs = self._transposed_segments()
        comm = self.comm_stream
        main = torch.cuda.current_stream(dev) if comm is not None else None
        landed, events, keep = [], [], []
        for c in range(C):
            t = segs[c + 1]
            d_rows = torch.empty(t.num_rows, F, device=dev)
            kernel.gspmm_into(t, d_rows, dout, accumulate=False)
            if self.halo_mode == "alltoall":
                nsend = sum(self.chunk_send_splits[c])
                recv = torch.empty(nsend, F, device=dev)
                n_in = sum(self.chunk_recv_splits[c])
                src_rows = d_rows[:n_in]

                def run(recv=recv, src_rows=src_rows, c=c):
                    dist.all_to_all_single(recv, src_rows, self.chunk_send_splits[c],
                                           self.chunk_recv_splits[c], group=self.group)
            else:
                recv = torch.empty(self.chunk_rows, F, device=dev)

                def run(recv=recv, d_rows=d_rows):
                    dist.reduce_scatter_tensor(recv, d_rows, op=dist.ReduceOp.SUM,
                                               group=self.group)
            if comm is not None:
                ev = torch.cuda.Event()
                ev.record(main)
                with torch.cuda.stream(comm):
                    comm.wait_event(ev)
                    run()
                    done = torch.cuda.Event()
                    done.record(comm)
                events.append(done)
                keep.append(d_rows)
            else:
                run()
            landed.append(recv)
        # own sources while the last chunks travel
        dh = torch.empty(R, F, device=dev)
        kernel.gspmm_into(segs[0], dh, dout, accumulate=False)
        cr = getattr(self, "chunk_rows", 0)
        for c in range(C):
            if comm is not None:
                main.wait_event(events[c])
                landed[c].record_stream(main)
            if self.halo_mode == "alltoall":
                off = 0
                idx = self.chunk_send_idx[c]
                for n in self.chunk_send_splits[c]:
                    if n:  # row ids are unique within a peer: ordered adds
                        dh.index_add_(0, idx[off:off + n], landed[c][off:off + n])
                    off += n
            else:
                lo, hi = c * cr, min((c + 1) * cr, R)
                if hi > lo:
                    dh[lo:hi] += landed[c][:hi - lo]
        if comm is not None:
            for t in keep:
                t.record_stream(comm)
            dout.record_stream(comm)
        return dh

    def _pipelined_copy_sum(self, h_local):
        C, P, cr = self.chunks, self.world, self.chunk_rows
        F = h_local.shape[1]
        dev = self.device
        hd = self.halo_dtype
        if self.halo is None or self.halo.shape[1] != F:
            # the landing rows: fp32, or bf16 bits in a float16 view that the
            # kernel reads as bf16 (no fp32 copy of the halo)
            self.halo = torch.empty(C * P * cr, F, device=dev,
                                    dtype=torch.float32 if hd is None else torch.float16)
            if self._emulated:  # compute-only study: no gather ever lands, use finite rows
                (self.halo if hd is None else self.halo.view(hd)).uniform_(-1, 1)
            self.hpads = {}
        h_local = h_local.contiguous()
        R = self.num_local
        sends = []
        for c in range(C):
            lo, hi = c * cr, min((c + 1) * cr, R)
            if hi - lo == cr:  # a full chunk: rows of h_local as they are
                sends.append(h_local[lo:hi])
                continue
            pad = self.hpads.get(c)  # partial / empty chunk: zero-padded copy
            if pad is None:
                pad = self.hpads[c] = torch.zeros(cr, F, device=dev)
            if hi > lo:
                pad[:hi - lo].copy_(h_local[lo:hi])
            sends.append(pad)
        out = torch.empty(R, F, device=dev)
        events, wires = [], []
        land = self.halo
        rows = self.halo if hd is None else self.halo.view(hd)

        def gather(c):
            wire = _pack(sends[c], hd).contiguous()
            dist.all_gather_into_tensor(land[c * P * cr:(c + 1) * P * cr], wire,
                                        group=self.group)
            wires.append(wire)

        if self.comm_stream is not None:
            ready = torch.cuda.Event()
            ready.record()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ready)
                for c in range(C):
                    gather(c)
                    ev = torch.cuda.Event()
                    ev.record(self.comm_stream)
                    events.append(ev)
        # own sources while the halo is in flight
        kernel.gspmm_into(self.seg_csrs[0], out, h_local, accumulate=False)
        for c in range(C):
            if self.comm_stream is not None:
                torch.cuda.current_stream(dev).wait_event(events[c])
            elif not self._emulated:
                gather(c)
            kernel.gspmm_into(self.seg_csrs[c + 1], out, rows, accumulate=True)
        if self.comm_stream is not None:
            self.halo.record_stream(torch.cuda.current_stream(dev))
            for t in wires:
                t.record_stream(self.comm_stream)
            h_local.record_stream(self.comm_stream)
        return out

    def _pipelined_alltoall_sum(self, h_local):
        dev = self.device
        C = self.chunks
        h_local = h_local.contiguous()
        F = h_local.shape[1]
        out = torch.empty(self.num_local, F, device=dev)
        hd = self.halo_dtype
        nrecv = [sum(x) for x in self.chunk_recv_splits]
        wire_dtype = torch.float32 if hd is None else torch.float16
        if self._emulated:  # compute-only study: resident random receive buffers
            if self.halo is None or self.halo[0].shape[1] != F:
                self.halo = [_pack(torch.rand(n, F, device=dev) * 2 - 1, hd) for n in nrecv]
            recvs = self.halo
        else:
            recvs = [torch.empty((n, F), dtype=wire_dtype, device=dev) for n in nrecv]
        main = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        events, sends = [], []

        def exchange(c):
            send = _pack(h_local.index_select(0, self.chunk_send_idx[c]), hd).contiguous()
            dist.all_to_all_single(recvs[c], send, self.chunk_recv_splits[c],
                                   self.chunk_send_splits[c], group=self.group)
            sends.append(send)

        if not self._emulated and self.comm_stream is not None:
            ready = torch.cuda.Event()
            ready.record()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ready)
                for c in range(C):
                    exchange(c)
                    ev = torch.cuda.Event()
                    ev.record(self.comm_stream)
                    events.append(ev)
        # own sources while the exchange is in flight
        kernel.gspmm_into(self.seg_csrs[0], out, h_local, accumulate=False)
        for c in range(C):
            if events:
                main.wait_event(events[c])
                recvs[c].record_stream(main)
            elif not self._emulated:
                exchange(c)
            if nrecv[c]:
                kernel.gspmm_into(self.seg_csrs[c + 1], out,
                                  recvs[c] if hd is None else recvs[c].view(hd),
                                  accumulate=True)
        if events:
            h_local.record_stream(self.comm_stream)
            for t in sends:
                t.record_stream(self.comm_stream)
        return out
