"""Per-edge kernels (g-SDDMM dot, GAT edge attention) walk whichever CSR of
the adjacency visits the edge ids most nearly in order (kernel._eid_major),
so their out[eid] stores are sequential. Each per-edge value is symmetric in
its two endpoint operands, so walking the transpose must give the same bits
as walking the destination-major CSR: checked here against a direct call on
the forward CSR, on a graph whose edges were added source-major (the
(src, dst)-sorted loaders' order, where the transpose is taken) and on one
in destination order (where the forward CSR is kept)."""
import numpy as np
import pytest
import torch

from dgl import kernel
from dgl._ffi import LIB, check_call

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


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("order", ["src", "dst"])
@pytest.mark.parametrize("F,H", [(128, 1), (64, 8), (48, 3), (32, 1)])
def test_sddmm_dot_walk_bits(device, order, F, H):
    dev = _dev(device)
    n, m = 700, 30000
    src, dst = _graph(F + H, n, m, order)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    rng = np.random.default_rng(5)
    A = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(dev)
    B = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(dev)
    _, tr = kernel._eid_major(adj)
    assert tr == (order == "src")
    got = kernel.gsddmm_dot(adj, A, B, m, H)
    ref = kernel._run_sddmm_dot(adj.fwd, A, B, m, H)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("order", ["src", "dst"])
def test_edge_attention_walk_bits(device, order):
    dev = _dev(device)
    n, m, H = 500, 20000, 8
    src, dst = _graph(3, n, m, order)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    rng = np.random.default_rng(6)
    a1 = torch.from_numpy(rng.standard_normal((n, H)).astype(np.float32)).to(dev)
    a2 = torch.from_numpy(rng.standard_normal((n, H)).astype(np.float32)).to(dev)
    got = kernel.edge_attention(adj, a1, a2, m)
    # the reference's edge UDF (gat/train.py:90-96) on the same values
    s, d = torch.from_numpy(src).to(dev), torch.from_numpy(dst).to(dev)
    x = a1[s] + a2[d]
    x = torch.where(x > 0, x, 0.2 * x)
    ref = torch.exp(x).clamp(-10, 10)
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=0)
    # the same bits as the kernel over the forward CSR
    fwd = adj.fwd
    out = torch.empty(m, H, device=dev)
    p = kernel.ptr
    args = (fwd.num_rows, H, p(fwd.indptr), p(fwd.indices), p(fwd.eid), p(a1), p(a2),
            0.2, -10.0, 10.0, 1, p(out))
    if dev.type == "cuda":
        check_call(LIB.dglhip_gsddmm_attention_device(*(args + (kernel._stream_of(dev),))))
    else:
        check_call(LIB.dglhip_gsddmm_attention_host(*(args + (0,))))
    assert torch.equal(got, out)


@pytest.mark.parametrize("device", DEVICES)
def test_u_mul_e_weight_grad_walk_bits(device):
    """The u_mul_e weight gradient (g-SDDMM in _GSpMM.backward) over the
    transpose equals the forward-CSR walk."""
    dev = _dev(device)
    n, m, F = 600, 25000, 64
    src, dst = _graph(11, n, m, "src")
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    rng = np.random.default_rng(7)
    H = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(dev)
    W = torch.from_numpy(rng.standard_normal(m).astype(np.float32)).to(dev).requires_grad_(True)
    G = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(dev)
    kernel.gspmm(adj, "u_mul_e", "sum", H, W).backward(G)
    ref = kernel._run_sddmm_dot(adj.fwd, G, H, m, 1).reshape(-1)
    assert torch.equal(W.grad.reshape(-1), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("H", [1, 2, 4, 8, 16])
def test_edge_attention_vector_kernel_bits(H):
    """The per-slot vector kernel (H in 1, 2, 4, 8, 16; aligned rows) gives the
    bits of the generic (slot, head)-lane kernel, which runs when the rows are
    not vector-aligned: same inputs at an odd float offset."""
    dev = _dev("cuda")
    n, m = 400, 30000
    src, dst = _graph(H, n, m, "dst")
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    rng = np.random.default_rng(H)
    a1 = torch.from_numpy(rng.standard_normal((n, H)).astype(np.float32)).to(dev)
    a2 = torch.from_numpy(rng.standard_normal((n, H)).astype(np.float32)).to(dev)
    vec = kernel.edge_attention(adj, a1, a2, m)
    buf = torch.empty(n * H + 1, device=dev)
    a1_odd = buf[1:].view(n, H)
    a1_odd.copy_(a1)
    gen = kernel.edge_attention(adj, a1_odd, a2, m)
    assert torch.equal(vec, gen)
