"""R-GCN typed-edge block g-SpMM vs the reference's UDF formulation
(examples/pytorch/rgcn/layers.py:121-132: gather W[type], bmm, sum by dst),
forward and gradients, within fp32 tolerance (the reference's bmm/sum orders
are implementation-defined)."""
import numpy as np
import pytest
import torch

from dgl import kernel

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def reference(src, dst, etype, h, W, n_dst, norm=None):
    R, nb, si, so = W.shape
    w = W[etype].reshape(-1, si, so)                     # (E*nb, si, so)
    node = h[src].reshape(-1, 1, si)                     # (E*nb, 1, si)
    msg = torch.bmm(node, w).reshape(len(src), nb * so)  # (E, out)
    if norm is not None:
        msg = msg * norm.unsqueeze(1)
    out = torch.zeros(n_dst, nb * so, dtype=msg.dtype, device=msg.device)
    return out.index_add(0, dst, msg)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("shape", [(11, 4, 3, 5), (20, 100, 5, 5)])
def test_typed_block(device, shape):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device(device)
    R, nb, si, so = shape
    rng = np.random.default_rng(3)
    n, m = 300, 5000
    src = torch.from_numpy(rng.integers(0, n, m)).to(dev)
    dst = torch.from_numpy(rng.integers(0, n, m)).to(dev)
    etype = torch.from_numpy(rng.integers(0, R, m)).to(dev)
    norm = torch.from_numpy(rng.uniform(0.1, 1, m).astype(np.float32)).to(dev)
    h = torch.randn(n, nb * si, device=dev, dtype=torch.float64)
    W = torch.randn(R, nb, si, so, device=dev, dtype=torch.float64) * 0.3
    G = torch.randn(n, nb * so, device=dev)
    adj = kernel.from_coo(n, n, dst.cpu(), src.cpu(), kernel.ORDER_EID, dev)
    for nm in (None, norm):
        h1 = h.float().clone().requires_grad_(True)
        W1 = W.float().clone().requires_grad_(True)
        out = kernel.typed_block_spmm(adj, h1, W1, etype, nm)
        out.backward(G)
        h2 = h.clone().requires_grad_(True)
        W2 = W.clone().requires_grad_(True)
        ref = reference(src, dst, etype, h2, W2, n, None if nm is None else nm.double())
        ref.backward(G.double())
        torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(h1.grad.double(), h2.grad, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(W1.grad.double(), W2.grad, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(7, 3, 1, 2), (9, 10, 2, 7), (11, 4, 3, 5), (20, 100, 5, 5),
                                   (5, 8, 8, 3), (4, 2, 16, 40), (6, 3, 7, 9)])
def test_typed_block_device_matches_host_bits(shape):
    """The HIP kernel (templated block widths 1/2/4/5/8/16, runtime width
    otherwise; slices of 64 outputs per wave, 4 edges in flight) runs the same
    per-element fma chains as the host kernel: identical bits, forward and
    the transposed-block backward. A power-law destination set gives rows far
    longer than the edge group."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    R, nb, si, so = shape
    rng = np.random.default_rng(sum(shape))
    n, m = 400, 8000
    p = 1.0 / np.arange(1, n + 1) ** 1.1
    dst = torch.from_numpy(rng.choice(n, size=m, p=p / p.sum()))
    src = torch.from_numpy(rng.integers(0, n, m))
    etype = torch.from_numpy(rng.integers(0, R, m))
    norm = torch.from_numpy(rng.uniform(0.1, 1, m).astype(np.float32))
    h = torch.randn(n, nb * si)
    W = torch.randn(R, nb, si, so) * 0.3
    G = torch.randn(n, nb * so)
    outs, grads = [], []
    for dev in ("cpu", "cuda"):
        adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
        h1 = h.detach().to(dev).clone().requires_grad_(True)
        out = kernel.typed_block_spmm(adj, h1, W.to(dev), etype.to(dev), norm.to(dev))
        out.backward(G.to(dev))
        outs.append(out.detach().cpu())
        grads.append(h1.grad.cpu())
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(grads[0], grads[1])
