"""NodeLinear: the dense per-node Linear that follows a g-SpMM, shaped for
full-graph node counts (millions of rows, a few hundred features).

The forward is one GEMM (hipBLASLt, MFMA). The backward's reductions over
the node dimension are what PyTorch handles badly at these shapes: on
RMAT-24 (16.7M rows, F=128) autograd of nn.Linear spent 64 ms per bias
gradient (a column reduce) and 14 ms per weight gradient (one GEMM with
K = 16.7M and a 128 x 128 output, too few tiles to fill 256 CUs).
Here both are cut into C row chunks (tools/colsum_study.py, 16.7M x 128 on
the MI355X; profiles/r01/colsum_study.json):

* dW = dYᵀ·X as a batched GEMM over the chunks (split-K), the C partial
  128 x 128 products summed in chunk order: 14.6 -> 4.4 ms;
* db = per-chunk column sums, then their sum: 1.4 ms (a GEMV dYᵀ·1 took
  177 ms in rocBLAS, ones·dY as a GEMM 9.3 ms).

Results equal nn.Linear's to fp32 summation tolerance (the association of the
sums over rows differs; both are implementation-defined in the reference's
torch backend).
"""
import math

import torch
import torch.nn as nn

from ..._handoff import GradHandoff, is_output, output_ref, take

__all__ = ["NodeLinear", "sage_dense", "bias_add", "dense_mm", "node_epilogue"]

_ROWS_PER_CHUNK = 1 << 16
_SMALL_ROWS_PER_CHUNK = 1 << 11


def _splitk_tn(a, b):
    """aᵀ·b for tall a (n, p), b (n, q): split-K over row chunks, summed in order."""
    n = a.shape[0]
    chunks = min(256, n // _ROWS_PER_CHUNK)
    if 1 < chunks < 32:
        # a few 64K-row chunks leave too few tiles for 256 CUs: 2K-row chunks
        # (r06, GCN on the 232,965-row graph: the 602 x 128 weight gradient
        # 0.83 -> 0.34 ms, the 128 x 41 one 0.42 -> 0.06 ms against torch's
        # unsplit GEMM; tools/gemm_probe.py, profiles/r06/gemm_probe_splitk.json)
        chunks = min(256, n // _SMALL_ROWS_PER_CHUNK)
    if chunks <= 1:
        # below two 64K-row chunks: 2K-row chunks, so a small output still gets
        # workgroups (Pubmed's 19,717 x 500 -> 64 x 500 weight gradient ran on
        # one workgroup in torch's GEMM: 0.14 ms)
        chunks = n // _SMALL_ROWS_PER_CHUNK
    if chunks <= 1:
        return a.t().matmul(b)
    k = n // chunks
    m = k * chunks
    A = a[:m].reshape(chunks, k, a.shape[1]).transpose(1, 2)
    B = b[:m].reshape(chunks, k, b.shape[1])
    out = torch.bmm(A, B).sum(0)
    if m < n:
        out = out + a[m:].t().matmul(b[m:])
    return out


def _colsum(a):
    """a.sum(0) for tall a, as per-chunk column sums summed in chunk order."""
    n = a.shape[0]
    chunks = min(256, n // _ROWS_PER_CHUNK)
    if chunks <= 1:
        return a.sum(0)
    k = n // chunks
    m = k * chunks
    out = a[:m].reshape(chunks, k, a.shape[1]).sum(1).sum(0)
    if m < n:
        out = out + a[m:].sum(0)
    return out


def _given_colsum(ctx, dy):
    """dy's column sums as the consumer's backward handed them over with dy
    (the loss kernel, which sums them as it stores dy; a GradHandoff keyed on
    that very tensor), else computed here."""
    given, ctx.dy_colsum = getattr(ctx, "dy_colsum", None), None
    cs = take(given, dy)
    return cs if cs is not None else _colsum(dy)


class _NodeLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        if bias is not None:
            out = torch.addmm(bias, x, weight.t())
        else:
            out = x.matmul(weight.t())
        ctx.out_ref = output_ref(out)
        ctx.wants_dy_colsum = ctx.has_bias and ctx.needs_input_grad[2]
        ctx.dy_colsum = None
        return out

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = dy.matmul(weight)
        if ctx.needs_input_grad[1]:
            dw = _splitk_tn(dy, x.contiguous())
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _given_colsum(ctx, dy)
        return dx, dw, db


class _DenseMMFn(torch.autograd.Function):
    """x·w (w: in x out, the GCN layer's weight layout) whose weight gradient
    xᵀ·dy is the split-K product (_splitk_tn) instead of autograd's one GEMM
    with K = the node count (too few output tiles to fill the chip)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return torch.mm(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy.mm(w.t()) if ctx.needs_input_grad[0] else None
        dw = _splitk_tn(x.contiguous(), dy) if ctx.needs_input_grad[1] else None
        return dx, dw


class _NodeEpilogueFn(torch.autograd.Function):
    """act(x * row_scale + bias) in one pass each way (rowops.hip,
    dglhip_node_epilogue_*): the bits of torch's three operations; the bias
    gradient from the backward kernel's per-128-row column sums, summed in
    order."""

    @staticmethod
    def forward(ctx, x, row_scale, bias, relu):
        from ... import _ffi, kernel
        n, F = x.shape
        out = torch.empty_like(x)
        _ffi.check_call(_ffi.LIB.dglhip_node_epilogue_fwd_device(
            n, F, _ffi.ptr(x), _ffi.ptr(row_scale), _ffi.ptr(bias), 1 if relu else 0,
            _ffi.ptr(out), kernel._stream_of(x.device)))
        ctx.relu = relu
        ctx.has_bias = bias is not None
        ctx.save_for_backward(out if relu else None, row_scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ... import _ffi, kernel
        out, row_scale = ctx.saved_tensors
        dout = dout.contiguous()
        n, F = dout.shape
        dx = torch.empty_like(dout)
        parts = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            parts = torch.empty(max(int(_ffi.LIB.dglhip_node_epilogue_parts(n)), 1), F,
                                dtype=torch.float32, device=dout.device)
        _ffi.check_call(_ffi.LIB.dglhip_node_epilogue_bwd_device(
            n, F, _ffi.ptr(dout), _ffi.ptr(out), _ffi.ptr(row_scale), 1 if ctx.relu else 0,
            _ffi.ptr(dx), _ffi.ptr(parts), kernel._stream_of(dout.device)))
        db = parts.sum(0) if parts is not None else None
        return dx, None, db, None


def node_epilogue(x, row_scale=None, bias=None, activation=None):
    """``activation(x * row_scale + bias)`` over node rows (the GCN layer's
    destination normalisation, bias and ReLU after its aggregation):
    ``row_scale`` (n,) or (n, 1), not differentiated; ``bias`` (F,);
    ``activation`` None or ReLU. On a ROCm device one kernel forward and one
    backward with the same forward bits and input gradient as the three torch
    operations (the bias gradient within fp32 summation tolerance); otherwise
    those operations."""
    relu = activation in (torch.relu, torch.nn.functional.relu)
    fused = (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and
             (activation is None or relu) and x.shape[1] <= 1024 and
             (row_scale is None or (row_scale.numel() == x.shape[0] and
                                    row_scale.dtype == torch.float32)) and
             (bias is None or (bias.dim() == 1 and bias.numel() == x.shape[1] and
                               bias.dtype == torch.float32)))
    if not fused:
        h = x if row_scale is None else x * row_scale.reshape(-1, 1)
        if bias is not None:
            h = bias_add(h, bias)
        return activation(h) if activation else h
    rs = None if row_scale is None else row_scale.detach().reshape(-1).contiguous()
    return _NodeEpilogueFn.apply(x.contiguous(), rs, bias, relu)


def dense_mm(x, w):
    """``torch.mm(x, w)`` for node-row inputs, with the weight gradient over
    the node dimension split into row chunks (summed in chunk order; fp32
    summation tolerance against torch's)."""
    if x.dim() != 2 or w.dim() != 2 or not (x.requires_grad or w.requires_grad):
        return torch.mm(x, w)
    return _DenseMMFn.apply(x, w)


class _BiasAddFn(torch.autograd.Function):
    """h + bias over node rows, whose bias gradient is the chunked column sum
    (_colsum) instead of torch's reduction over the node dimension (r06: the
    2-layer GCN's bias gradient over 232,965 x 128 took 1.16 ms of a 15.8 ms
    epoch in torch's reduce kernel)."""

    @staticmethod
    def forward(ctx, h, bias):
        ctx.bias_shape = bias.shape
        return h + bias

    @staticmethod
    def backward(ctx, dy):
        db = None
        if ctx.needs_input_grad[1]:
            d2 = dy.reshape(-1, dy.shape[-1]) if dy.dim() != 2 else dy
            db = _colsum(d2.contiguous()).reshape(ctx.bias_shape)
        return (dy if ctx.needs_input_grad[0] else None), db


def bias_add(h, bias):
    """``h + bias`` for a bias broadcast over the rows of a node tensor
    (bias of h's trailing width); the same values, and a bias gradient summed
    in row chunks (fp32 summation tolerance against torch's reduction, whose
    association is implementation-defined too)."""
    if bias is None:
        return h
    if not (h.is_cuda and h.dim() >= 2 and bias.dim() == 1 and bias.shape[0] == h.shape[-1]):
        return h + bias
    return _BiasAddFn.apply(h, bias)


def _mm_t(x, w):
    return x.matmul(w.t())


# -- MFMA node Linear (csrc/node_linear.hip) ----------------------------------
# The narrow products of a GraphSAGE output layer (in 64/128/256, out <= 64)
# run on the library's f32 MFMA kernels: both products of the input rows in one
# pass, and the input gradient of both in one pass. Other shapes (and CPU
# tensors) take torch's GEMMs, which run them at their rate already.

def _mfma_fwd_ok(x, *ms):
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1 and
            x.stride(0) % 4 == 0 and x.shape[1] in (64, 128, 256) and x.data_ptr() % 16 == 0 and
            all(1 <= m <= 64 for m in ms))


def _mfma_dgrad_ok(k, *dys):
    return k in (64, 128) and all(
        d.is_cuda and d.dtype == torch.float32 and d.dim() == 2 and d.stride(1) == 1 and
        1 <= d.shape[1] <= 64 for d in dys)


def _w(t):
    return None if t is None else t.detach().contiguous()


def _node_linear2(x, w1, ld1, w2, b2):
    """(y1 (n, m1) viewed out of rows padded to ld1, y2 = x W2^T + b2), one pass."""
    from ... import _ffi, kernel
    n, k = x.shape
    m1, m2 = w1.shape[0], w2.shape[0]
    w1, w2, b2 = _w(w1), _w(w2), _w(b2)
    y1 = torch.empty(n, ld1, dtype=torch.float32, device=x.device)
    y2 = torch.empty(n, m2, dtype=torch.float32, device=x.device)
    _ffi.check_call(_ffi.LIB.dglhip_node_linear_device(
        n, k, _ffi.ptr(x), x.stride(0), m1, _ffi.ptr(w1), None, _ffi.ptr(y1), ld1, m2,
        _ffi.ptr(w2), _ffi.ptr(b2), _ffi.ptr(y2), m2, kernel._stream_of(x.device)))
    return y1[:, :m1], y2


def _mfma_cat_ok(x1, x2, m, relu=False):
    # up to 64 outputs, or 128 from 128-column inputs (one pass over the
    # inputs: 38.4 ms at 67M rows vs 43 for hipBLASLt's two products,
    # tools/node_linear_bench.py), or 128 from 64-column inputs with the ReLU
    # fused into the store (two passes)
    k = x1.shape[1] if x1.dim() == 2 else 0
    return (1 <= m <= (128 if (relu or k == 128) else 64) and x1.shape == x2.shape and all(
        t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 and
        t.stride(0) % 4 == 0 and t.shape[1] in (64, 128) and t.data_ptr() % 16 == 0
        for t in (x1, x2)))


def _node_linear_cat(x1, w1, x2, w2, b, relu=False):
    """x1 W1^T + x2 W2^T + b (relu: max(., 0) fused into the store) in one
    pass per 64 outputs."""
    from ... import _ffi, kernel
    n, k = x1.shape
    m = w1.shape[0]
    w1, w2, b = _w(w1), _w(w2), _w(b)
    y = torch.empty(n, m, dtype=torch.float32, device=x1.device)
    _ffi.check_call(_ffi.LIB.dglhip_node_linear_cat_device(
        n, k, _ffi.ptr(x1), x1.stride(0), _ffi.ptr(x2), x2.stride(0), m, _ffi.ptr(w1),
        _ffi.ptr(w2), _ffi.ptr(b), _ffi.ptr(y), m, int(relu), kernel._stream_of(x1.device)))
    return y


def _node_dgrad2(k, dy1, w1, dy2, w2, gate=None, colsum=False):
    """dy1 W1 + dy2 W2 in one pass (n, k); ``gate`` (n, k, unit column
    stride): 0 where gate <= 0 (ReLU's backward applied in the store).
    ``colsum``: also return dx's column sums, summed as the kernel stores."""
    from ... import _ffi, kernel
    n = dy1.shape[0]
    w1, w2 = _w(w1), _w(w2)
    dev = dy1.device
    dx = torch.empty(n, k, dtype=torch.float32, device=dev)
    cs = ws = None
    if colsum:
        cs = torch.empty(k, dtype=torch.float32, device=dev)
        ws = torch.empty(_ffi.LIB.dglhip_node_linear_dgrad_workspace_floats(k),
                         dtype=torch.float32, device=dev)
    _ffi.check_call(_ffi.LIB.dglhip_node_linear_dgrad_device(
        n, k, dy1.shape[1], _ffi.ptr(dy1), dy1.stride(0), _ffi.ptr(w1), dy2.shape[1],
        _ffi.ptr(dy2), dy2.stride(0), _ffi.ptr(w2), _ffi.ptr(dx), k,
        _ffi.ptr(gate), 0 if gate is None else gate.stride(0), _ffi.ptr(cs), _ffi.ptr(ws),
        kernel._stream_of(dev)))
    return (dx, cs) if colsum else dx


class _DualLinearFn(torch.autograd.Function):
    """out = x @ Ws^T + b + agg @ Wn^T (relu: max(., 0)) as one product over
    the concatenated inputs (the MFMA kernel: one pass over x and agg, the
    ReLU in its store), or one GEMM and one accumulating GEMM (beta = 1): no
    separate sum pass, and neither product is materialised. With relu the
    output is saved and the backward masks dy by out > 0 (ReLU's own rule)."""

    @staticmethod
    def forward(ctx, x, w_self, bias, agg, w_neigh, relu):
        ctx.has_bias = bias is not None
        ctx.relu = bool(relu)
        if _mfma_cat_ok(x, agg, w_self.shape[0], relu):
            out = _node_linear_cat(x, w_self, agg, w_neigh, bias, relu)
        else:
            out = torch.addmm(bias, x, w_self.t()) if bias is not None else _mm_t(x, w_self)
            out.addmm_(agg, w_neigh.t())
            if relu:
                out.relu_()
        ctx.save_for_backward(x, w_self, agg, w_neigh, out if relu else None)
        ctx.out_ref = output_ref(out)
        ctx.premasked = None
        return out

    @staticmethod
    def backward(ctx, dy):
        x, w_self, agg, w_neigh, out = ctx.saved_tensors
        premasked, ctx.premasked = ctx.premasked, None
        colsum = None
        got = take(premasked, dy)  # (dy's column sums or None,): dy already masked
        if got is not None:
            colsum = got[0]  # taken as dy was stored
        elif ctx.relu:
            dy = torch.ops.aten.threshold_backward(dy, out, 0)  # ReLU's own backward, one pass
        dy = dy.contiguous()
        need = ctx.needs_input_grad
        dx = dy.matmul(w_self) if need[0] else None
        dws = _splitk_tn(dy, x.contiguous()) if need[1] else None
        db = None
        if ctx.has_bias and need[2]:
            db = colsum if colsum is not None else _colsum(dy)
        dagg = dy.matmul(w_neigh) if need[3] else None
        dwn = _splitk_tn(dy, agg.contiguous()) if need[4] else None
        return dx, dws, db, dagg, dwn, None


class _PreAggregateFn(torch.autograd.Function):
    """out = x @ Ws^T + b + A(x @ Wn^T) for a neighbour Linear that narrows
    the features (aggregate the narrow side). The aggregation runs through
    its own autograd (DGLGraph or a partitioned graph's pipelined halo); its
    transpose is taken inside this backward so that dx = dy Ws + (A^T dy) Wn
    is one GEMM and one accumulating GEMM, not two products and a sum."""

    @staticmethod
    def forward(ctx, x, w_self, bias, w_neigh, aggregate):
        self_out = None
        if _mfma_fwd_ok(x, w_neigh.shape[0], w_self.shape[0]):
            # both products in one pass over x; the aggregated one at a
            # line-aligned row stride, gathered by the g-SpMM without a copy
            from ... import kernel
            pre, self_out = _node_linear2(x, w_neigh, kernel.padded_width(w_neigh.shape[0]),
                                          w_self, bias)
        else:
            pre = _mm_t(x, w_neigh)
        # an aggregation that can add its result into a tensor in its own
        # store (``aggregate.add_into(h, out)``, e.g. kernel.gspmm_mean_add)
        # takes self_out as that tensor: out = self_out + A(pre), no sum pass
        add_into = getattr(aggregate, "add_into", None) if self_out is not None else None
        agg = aggregate if add_into is None else (lambda t: add_into(t, self_out))
        if any(ctx.needs_input_grad):
            with torch.enable_grad():
                pre_leaf = pre.detach().requires_grad_(True)
                neigh = agg(pre_leaf)
        else:  # inference: no graph to keep
            pre_leaf, neigh = None, agg(pre)
        del pre
        # accumulate into the aggregate's own buffer (its backward does not
        # read it): no copy of an (N, out) tensor. Not into a view: autograd
        # would rebase the view's graph on the in-place update (a zero fill
        # and a copy of the gradient); then into self_out (a + b == b + a)
        if add_into is not None:
            out = neigh.detach()
            del self_out
        elif self_out is not None and neigh._base is not None:
            out = self_out.add_(neigh.detach())
            del self_out
        elif self_out is not None:
            out = neigh.detach()
            out.add_(self_out)
            del self_out
        else:
            out = neigh.detach() if neigh._base is None else neigh.detach().clone()
            out.addmm_(x, w_self.t())
            if bias is not None:
                out.add_(bias)
        ctx.save_for_backward(x, w_self, w_neigh)
        ctx.graph = (pre_leaf, neigh) if pre_leaf is not None else None
        ctx.has_bias = bias is not None
        ctx.out_ref = output_ref(out)
        ctx.wants_dy_colsum = ctx.has_bias and ctx.needs_input_grad[2]
        ctx.dy_colsum = None
        # the in-store mean-add's backward operand dy / deg can come from dy's
        # producer (the loss kernel) as it stores dy
        inner = neigh.grad_fn if (add_into is not None and pre_leaf is not None) else None
        ctx.inner = inner if getattr(inner, "scale_spec", None) is not None else None
        ctx.dy_scaled_spec = ctx.inner.scale_spec if ctx.inner is not None else None
        ctx.dy_scaled = None
        ctx.relu_node = _relu_producer(x)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, w_self, w_neigh = ctx.saved_tensors
        pre_leaf, neigh = ctx.graph
        ctx.graph = None
        dy = dy.contiguous()
        need = ctx.needs_input_grad
        dws = None
        side = _side_stream(dy.device) if (_OVERLAP and dy.is_cuda and need[1]) else None
        if side is not None:
            # the self weight's gradient needs only dy: its MFMA product runs on
            # a side stream while the transposed aggregation (a byte-bound
            # gather) runs on this one (the byte-bound bias column sums stay
            # here: beside the gather they only slow both)
            main = torch.cuda.current_stream(dy.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                dws = _splitk_tn(dy, x.contiguous())
            for t in (dy, x):
                t.record_stream(side)
        scaled, ctx.dy_scaled = ctx.dy_scaled, None
        inner, ctx.inner = ctx.inner, None
        scaled = take(scaled, dy)
        if inner is not None and scaled is not None:
            # the mean-add's backward receives this same dy as its dout
            inner.prescaled = GradHandoff(dy, scaled)
        (dpre,) = torch.autograd.grad(neigh, pre_leaf, dy)
        dpre = dpre.contiguous()
        dx = None
        node, ctx.relu_node = ctx.relu_node, None
        if need[0]:
            if _mfma_dgrad_ok(x.shape[1], dy, dpre):
                # x is a fused-ReLU layer's output: its backward mask (out > 0
                # is x > 0) is applied in this product's store, and that
                # layer skips its own pass over the gradient when it receives
                # this very tensor unmodified (same storage, same version:
                # a gradient summed with another consumer's is masked there)
                # (and, for that layer's bias gradient, dx's column sums are
                # taken as the store writes them)
                gate = x if node is not None else None
                if gate is not None:
                    dx, cs = _node_dgrad2(x.shape[1], dy, w_self, dpre, w_neigh, gate=gate,
                                          colsum=node.has_bias)
                    node.premasked = GradHandoff(dx, (cs,))
                else:
                    dx = _node_dgrad2(x.shape[1], dy, w_self, dpre, w_neigh)
            else:
                dx = dy.matmul(w_self)
                dx.addmm_(dpre, w_neigh)
        if side is None:
            dws = _splitk_tn(dy, x.contiguous()) if need[1] else None
        db = _given_colsum(ctx, dy) if ctx.has_bias and need[2] else None
        dwn = _splitk_tn(dpre, x.contiguous()) if need[3] else None
        if side is not None:
            main.wait_stream(side)
            dws.record_stream(main)
        return dx, dws, db, dwn, None


_OVERLAP = True
_SIDE = {}


def _side_stream(device):
    """One side stream per device for gradients that can run beside the
    aggregation's backward."""
    key = torch.device(device).index
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


def _relu_producer(x):
    """The _DualLinearFn node whose fused-ReLU output ``x`` is (the tensor
    itself, not a view or an in-place update of it), else None."""
    node = x.grad_fn
    if (isinstance(node, _DualLinearFn._backward_cls) and getattr(node, "relu", False) and
            is_output(node, x) and x.is_contiguous()):
        return node
    return None


def _is_relu(act):
    return act in (torch.relu, torch.nn.functional.relu) or isinstance(act, torch.nn.ReLU)


def sage_dense(h, aggregate, fc_self, fc_neigh, activation=None):
    """GraphSAGE's dense step fc_self(h) + fc_neigh(aggregate(h)) on
    NodeLinear weights (fc_neigh without bias), shaped for full-graph node
    counts. fc_neigh commutes with the (linear) aggregation, so the narrower
    side is aggregated; the two products and their sum are one GEMM plus one
    accumulating GEMM in both directions, which at 10^7-10^8 nodes saves a
    pass over an (N, out) tensor per direction and two (N, out) buffers of
    peak memory (RMAT-26: 34 GB each). ``activation`` is applied to the sum;
    a ReLU on the widening / square layer is fused into the product's store
    (its backward mask into the fused backward). An ``aggregate`` carrying
    ``add_into(h, out)`` (out <- out + aggregate(h) in place, differentiable in
    h; kernel.gspmm_mean_add for the mean) lets the narrowing layer add
    fc_self(h) in the aggregation's own store."""
    def act(t):
        return activation(t) if activation is not None else t
    if h.dim() != 2 or fc_neigh.bias is not None:
        # (a bias on fc_neigh would not commute with the mean's empty rows)
        return act(fc_self(h) + fc_neigh(aggregate(h)))
    if fc_neigh.in_features > fc_neigh.out_features:
        return act(_PreAggregateFn.apply(h, fc_self.weight, fc_self.bias, fc_neigh.weight,
                                         aggregate))
    relu = _is_relu(activation)
    out = _DualLinearFn.apply(h, fc_self.weight, fc_self.bias, aggregate(h), fc_neigh.weight,
                              relu)
    return out if relu else act(out)


class NodeLinear(nn.Module):
    """Drop-in for nn.Linear on (num_nodes, in_features) inputs (same
    parameters, initialisation and forward arithmetic)."""

    def __init__(self, in_features, out_features, bias=True):
        super(NodeLinear, self).__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        # nn.Linear's initialisation
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(self.in_features) if self.in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        if x.dim() != 2:
            return nn.functional.linear(x, self.weight, self.bias)
        return _NodeLinearFn.apply(x, self.weight, self.bias)
