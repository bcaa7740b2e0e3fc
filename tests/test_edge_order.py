"""Edge values in the forward CSR's slot order (``edge_order="slot"``).

GAT's attention is produced by one kernel and consumed by the next two, so
its layout is internal to the layer: with ``edge_order="slot"`` the
attention kernel stores value k at row k (sequential stores along the walk)
and the u_mul_e / copy_e g-SpMMs read row k for slot k, without the per-edge
eid gather (DESIGN.md §6 "Edge-value order"). Every element is computed by
the same arithmetic in the same order as in edge-id layout, so everything
here is compared bit for bit with the edge-id path permuted by
``slot_permutation`` (forward, both gradients, every reducer), on graphs
whose edges were added source-major (eid != slot order) and destination-major.
"""
import numpy as np
import pytest
import torch

from dgl import kernel

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device(device)


def _graph(seed, n, nnz, order):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, nnz)
    dst = rng.integers(0, n, nnz)
    key = src * n + dst if order == "src" else dst * n + src
    o = np.argsort(key, kind="stable")
    return src[o].astype(np.int64), dst[o].astype(np.int64)


def _rand(rng, shape, dev):
    return torch.from_numpy(rng.standard_normal(shape).astype(np.float32)).to(dev)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("order", ["src", "dst"])
def test_attention_slot_order_bits(device, order):
    dev = _dev(device)
    n, m, H = 600, 25000, 8
    src, dst = _graph(11, n, m, order)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    rng = np.random.default_rng(1)
    a1 = _rand(rng, (n, H), dev).requires_grad_(True)
    a2 = _rand(rng, (n, H), dev).requires_grad_(True)
    b1 = a1.detach().clone().requires_grad_(True)
    b2 = a2.detach().clone().requires_grad_(True)
    perm = kernel.slot_permutation(adj)
    by_eid = kernel.edge_attention(adj, a1, a2, m)
    by_slot = kernel.edge_attention(adj, b1, b2, m, edge_order="slot")
    assert torch.equal(by_slot, by_eid[perm])
    G = _rand(rng, (m, H), dev)
    by_eid.backward(G)
    by_slot.backward(G[perm])
    assert torch.equal(a1.grad, b1.grad)
    assert torch.equal(a2.grad, b2.grad)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("order", ["src", "dst"])
@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
@pytest.mark.parametrize("F,H", [(64, 8), (128, 8), (48, 1), (32, 32)])
def test_u_mul_e_slot_order_bits(device, order, reduce, F, H):
    """Per-head (or scalar, or full-width) edge weights in slot order: the
    forward, dU and the dE g-SDDMM (forward walk, stores by slot) equal the
    edge-id layout's bits."""
    dev = _dev(device)
    n, m = 500, 20000
    src, dst = _graph(F + H, n, m, order)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    rng = np.random.default_rng(F * H)
    D = F // H
    u = _rand(rng, (n, H, D), dev).requires_grad_(True)
    w = _rand(rng, (m, H, 1), dev).requires_grad_(True)
    u2 = u.detach().clone().requires_grad_(True)
    perm = kernel.slot_permutation(adj)
    w2 = w.detach()[perm].clone().requires_grad_(True)
    out = kernel.gspmm(adj, "u_mul_e", reduce, u, w)
    out2 = kernel.gspmm(adj, "u_mul_e", reduce, u2, w2, edge_order="slot")
    assert torch.equal(out, out2)
    G = _rand(rng, tuple(out.shape), dev)
    out.backward(G)
    out2.backward(G)
    if reduce == "max":
        # argmax routing scatters with index_put_(accumulate=True), whose add
        # order is not fixed: the same terms, summed in either order
        torch.testing.assert_close(u.grad, u2.grad, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(w.grad[perm], w2.grad, rtol=1e-6, atol=1e-6)
    else:
        assert torch.equal(u.grad, u2.grad)
        assert torch.equal(w.grad[perm], w2.grad)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("order", ["src", "dst"])
def test_copy_e_and_full_width_slot_order_bits(device, order):
    dev = _dev(device)
    n, m, F = 400, 15000, 24
    src, dst = _graph(5, n, m, order)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    rng = np.random.default_rng(2)
    perm = kernel.slot_permutation(adj)
    e = _rand(rng, (m, F), dev).requires_grad_(True)
    e2 = e.detach()[perm].clone().requires_grad_(True)
    out = kernel.gspmm(adj, "copy_e", "sum", None, e)
    out2 = kernel.gspmm(adj, "copy_e", "sum", None, e2, edge_order="slot")
    assert torch.equal(out, out2)
    G = _rand(rng, tuple(out.shape), dev)
    out.backward(G)
    out2.backward(G)
    assert torch.equal(e.grad[perm], e2.grad)
    # u_mul_e with a full-width edge feature (EM_FULL)
    u = _rand(rng, (n, F), dev).requires_grad_(True)
    u2 = u.detach().clone().requires_grad_(True)
    we = _rand(rng, (m, F), dev).requires_grad_(True)
    we2 = we.detach()[perm].clone().requires_grad_(True)
    o = kernel.gspmm(adj, "u_mul_e", "sum", u, we)
    o2 = kernel.gspmm(adj, "u_mul_e", "sum", u2, we2, edge_order="slot")
    assert torch.equal(o, o2)
    o.backward(G)
    o2.backward(G)
    assert torch.equal(u.grad, u2.grad)
    assert torch.equal(we.grad[perm], we2.grad)


@pytest.mark.parametrize("device", DEVICES)
def test_gsddmm_dot_slot_order(device):
    dev = _dev(device)
    n, m = 300, 9000
    src, dst = _graph(9, n, m, "src")
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    rng = np.random.default_rng(4)
    A, B = _rand(rng, (n, 128), dev), _rand(rng, (n, 128), dev)
    for H in (1, 4, 8, 16, 32):
        by_eid = kernel.gsddmm_dot(adj, A, B, m, H)
        by_slot = kernel.gsddmm_dot(adj, A, B, m, H, edge_order="slot")
        assert torch.equal(by_slot, by_eid[kernel.slot_permutation(adj)])


def test_bad_edge_order():
    from dgl.base import DGLError
    adj = kernel.from_coo(3, 3, [0, 1], [1, 2], kernel.ORDER_EID, "cpu")
    with pytest.raises(DGLError):
        kernel.gspmm(adj, "copy_e", "sum", None, torch.ones(2, 1), edge_order="csr")
