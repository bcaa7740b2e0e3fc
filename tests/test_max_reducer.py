"""``max`` reducer: the segmented-max kernels against a
numpy restatement of the reference's degree-bucketing ``F.max(mailbox, 1)``
(python/dgl/runtime/degree_bucketing.py:13-190 with the reducer of
function/reducer.py): per destination the messages in edge order, the first
of equal maxima wins, rows without messages read 0. Values are integers so
ties are frequent. Forward bit-exact; gradients (routed to the argmax slot)
within 1e-5. Sweeps the kernel's (VEC, GROUP) shapes and every message /
edge-feature layout (copy_u, copy_e, u_mul_e with scalar, per-head and full
edge features), on the host path and, under the gpu marker, the MI355X.
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


def _graph(rng, n, nnz):
    p = 1.0 / np.arange(1, n + 1) ** 1.1  # a few long rows, some empty ones
    row = rng.choice(n, size=nnz, p=p / p.sum()).astype(np.int64)
    col = rng.integers(0, n, nnz).astype(np.int64)
    return row, col


def _reference(n, row, col, msgs, G, U, E, msg, dpe):
    """Forward max + gradients of sum(out * G) w.r.t. U and E (float64 grads)."""
    E_ = msgs.shape[0]
    F = msgs.shape[1]
    out = np.zeros((n, F), np.float32)
    arg = np.full((n, F), -1, np.int64)
    order = np.argsort(row, kind="stable")  # edge-id order within each row
    bounds = np.searchsorted(row[order], np.arange(n + 1))
    for v in range(n):
        es = order[bounds[v]:bounds[v + 1]]
        if len(es):
            m = msgs[es]                       # (deg, F) in edge order
            first = np.argmax(m, axis=0)       # first occurrence of the maximum
            arg[v] = es[first]
            out[v] = m[first, np.arange(F)]
    dU = None if U is None else np.zeros(U.shape, np.float64)
    dE = None if E is None else np.zeros(E.shape, np.float64)
    vs, fs = np.nonzero(arg >= 0)
    es = arg[vs, fs]
    g = G[vs, fs].astype(np.float64)
    if dU is not None:
        w = E[es, fs // dpe].astype(np.float64) if msg == "u_mul_e" else 1.0
        np.add.at(dU, (col[es], fs), g * w)
    if dE is not None:
        w = U[col[es], fs].astype(np.float64) if msg == "u_mul_e" else 1.0
        np.add.at(dE, (es, fs // dpe), g * w)
    assert E_ == len(row)
    return out, dU, dE


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("F", [1, 3, 16, 41, 64, 128, 256, 602])
def test_max_copy_u(device, F):
    dev = _dev(device)
    rng = np.random.default_rng(F)
    n = 400
    row, col = _graph(rng, n, 6000)
    U = rng.integers(-4, 5, (n, F)).astype(np.float32)
    G = rng.standard_normal((n, F)).astype(np.float32)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, dev)
    u = torch.from_numpy(U).to(dev).requires_grad_(True)
    out = kernel.gspmm(adj, "copy_u", "max", u)
    ref, dU, _ = _reference(n, row, col, U[col], G, U, None, "copy_u", 1)
    assert np.array_equal(out.detach().cpu().numpy(), ref)
    out.backward(torch.from_numpy(G).to(dev))
    np.testing.assert_allclose(u.grad.cpu().numpy(), dU, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("msg,layout", [("copy_e", "full"), ("copy_e", "scalar"),
                                        ("u_mul_e", "full"), ("u_mul_e", "scalar"),
                                        ("u_mul_e", "head")])
def test_max_edge_messages(device, msg, layout):
    dev = _dev(device)
    rng = np.random.default_rng(len(msg) * 7 + len(layout))
    n, H, D = 300, 4, 8
    F = H * D
    row, col = _graph(rng, n, 5000)
    nnz = len(row)
    U = rng.integers(-3, 4, (n, F)).astype(np.float32)
    elen = {"full": F, "scalar": 1, "head": H}[layout]
    E = rng.integers(-2, 3, (nnz, elen)).astype(np.float32)
    dpe = F // elen
    G = rng.standard_normal((n, F)).astype(np.float32)
    if msg == "copy_e":
        msgs = np.repeat(E, dpe, axis=1)
        uref = None
    else:
        msgs = U[col] * np.repeat(E, dpe, axis=1)
        uref = U
    ref, dU, dE = _reference(n, row, col, msgs.astype(np.float32), G, uref, E, msg, dpe)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID, dev)
    e = torch.from_numpy(E).to(dev)
    if layout == "head":
        e = e.reshape(nnz, H, 1)
    e.requires_grad_(True)
    if msg == "copy_e":
        ein = e if layout == "full" else e.expand(nnz, F) if layout == "scalar" else None
        out = kernel.gspmm(adj, "copy_e", "max", None, ein)
        u = None
    else:
        u = torch.from_numpy(U).to(dev)
        u = (u.reshape(n, H, D) if layout == "head" else u).requires_grad_(True)
        out = kernel.gspmm(adj, "u_mul_e", "max", u, e)
    assert np.array_equal(out.detach().cpu().numpy().reshape(n, F), ref)
    out.backward(torch.from_numpy(G).to(dev).reshape(out.shape))
    np.testing.assert_allclose(e.grad.cpu().numpy().reshape(nnz, elen), dE, rtol=1e-5, atol=1e-5)
    if u is not None:
        np.testing.assert_allclose(u.grad.cpu().numpy().reshape(n, F), dU, rtol=1e-5, atol=1e-5)
