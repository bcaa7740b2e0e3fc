"""Weighted softmax cross-entropy over node rows, the loss of a full-graph
node classifier (csrc/node_loss.hip).

``weighted_cross_entropy(z, y, w)`` is the value of

    (F.cross_entropy(z, y, reduction="none") * w).sum()

(the masked training loss of the examples when ``w`` is the float training
mask; the reference's examples reduce ``F.cross_entropy`` / ``nll_loss`` over
``logits[train_mask]``, examples/pytorch/gcn/gcn_spmv.py:113-118). At 10^7-10^8
rows PyTorch runs it as five passes over the logits (log-softmax, the nll
gather, a zero fill, the nll scatter, the log-softmax backward); on a ROCm
device with 1..64 classes it is one kernel forward (one read) and one
backward (one read, one write), the upstream gradient read on the device.
When the logits are the output of a NodeLinear / sage_dense with a bias, the
backward also returns that bias's gradient (dz's column sums) from the same
kernel, read back from the tile it stores (no separate column reduce over
the rows); when they are a sage_dense output whose mean aggregation added into
them (kernel.gspmm_mean_add), also dz / deg in the padded rows that
aggregation's backward gathers (no division pass). Other devices and shapes
compute the expression above with PyTorch's own operators. Results agree with
it to fp32 rounding (the sums associate differently). Rows labelled -100
(PyTorch's ignore_index) contribute nothing; any other label outside [0, C)
is an error in PyTorch, and makes the fused loss (and that row's gradient)
NaN: never a silently different value.
"""
import torch
import torch.nn.functional as F

from ..._handoff import GradHandoff, is_output

__all__ = ["weighted_cross_entropy"]

_MAX_CLASSES = 64


def _fused_ok(z, y, w):
    return (z.is_cuda and z.dtype == torch.float32 and z.dim() == 2 and z.stride(1) == 1 and
            1 <= z.shape[1] <= _MAX_CLASSES and z.stride(0) >= z.shape[1] and y.dim() == 1 and y.shape[0] == z.shape[0] and
            y.dtype == torch.int64 and y.device == z.device and
            (w is None or (w.dim() == 1 and w.shape[0] == z.shape[0] and
                           w.dtype == torch.float32 and w.device == z.device)))


def _bias_producer(z):
    """The NodeLinear / sage_dense autograd node whose output ``z`` is (the
    tensor itself) and that will want dz's column sums for its bias, or dz
    divided by its mean aggregation's degrees (``dy_scaled_spec``: divisor,
    padded row stride), else None: the loss backward then takes them from its
    tile as it stores dz."""
    node = z.grad_fn
    if (node is not None and (getattr(node, "wants_dy_colsum", False) or
                              getattr(node, "dy_scaled_spec", None) is not None) and
            is_output(node, z) and z.is_contiguous()):
        return node
    return None


class _WeightedXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, y, w):
        from ... import _ffi, kernel
        y = y.contiguous()
        w = None if w is None else w.detach().contiguous()
        n, C = z.shape
        loss = torch.empty((), dtype=torch.float32, device=z.device)
        ws = torch.empty(_ffi.LIB.dglhip_xent_workspace_floats(), dtype=torch.float32,
                         device=z.device)
        _ffi.check_call(_ffi.LIB.dglhip_xent_fwd_device(
            n, C, _ffi.ptr(z), z.stride(0), _ffi.ptr(y), _ffi.ptr(w), _ffi.ptr(loss),
            _ffi.ptr(ws), kernel._stream_of(z.device)))
        ctx.save_for_backward(z, y, w)
        ctx.bias_node = _bias_producer(z)
        return loss

    @staticmethod
    def backward(ctx, g):
        from ... import _ffi, kernel
        z, y, w = ctx.saved_tensors
        n, C = z.shape
        g = g.detach().to(torch.float32).contiguous()
        dz = torch.empty(n, C, dtype=torch.float32, device=z.device)
        node, ctx.bias_node = ctx.bias_node, None
        cs = ws = div = scaled = None
        lds = 0
        if node is not None and getattr(node, "wants_dy_colsum", False):
            cs = torch.empty(C, dtype=torch.float32, device=z.device)
            ws = torch.empty(_ffi.LIB.dglhip_xent_colsum_workspace_floats(C),
                             dtype=torch.float32, device=z.device)
        spec = getattr(node, "dy_scaled_spec", None) if node is not None else None
        if spec is not None and spec[0].shape[0] == n:
            div, lds = spec
            scaled = torch.empty(n, lds, dtype=torch.float32, device=z.device)
        _ffi.check_call(_ffi.LIB.dglhip_xent_bwd_ex_device(
            n, C, _ffi.ptr(z), z.stride(0), _ffi.ptr(y), _ffi.ptr(w), _ffi.ptr(g), _ffi.ptr(dz),
            C, _ffi.ptr(cs), _ffi.ptr(ws), _ffi.ptr(div), _ffi.ptr(scaled), lds,
            kernel._stream_of(z.device)))
        if cs is not None:
            # the producing Linear's bias gradient, summed as dz was stored
            node.dy_colsum = GradHandoff(dz, cs)
        if scaled is not None:
            # dz / deg in the padded rows of the producer's mean aggregation
            node.dy_scaled = GradHandoff(dz, scaled[:, :C])
        return dz, None, None


def weighted_cross_entropy(logits, labels, weight=None):
    """sum_i weight_i * cross_entropy(logits_i, labels_i) (weight None: all
    ones), differentiable in ``logits``; see the module docstring."""
    if _fused_ok(logits, labels, weight) and (weight is None or not weight.requires_grad):
        return _WeightedXentFn.apply(logits, labels, weight)
    ce = F.cross_entropy(logits, labels, reduction="none")
    return (ce * weight).sum() if weight is not None else ce.sum()
