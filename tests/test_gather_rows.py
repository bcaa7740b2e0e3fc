"""kernel.gather_rows: x[idx] whose backward is the g-SpMM over the
transposed selection (used by the R-GCN example's DistMult decoder). The
gradient of every row is the chain of its duplicates' upstream rows in
increasing position — the oracle's nnz-order chain over COO (idx, i) — bit
for bit, host and device; forward equals index_select."""
import numpy as np
import pytest
import torch

from dgl import kernel
from oracle import oracle as O

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("shape", [(500,), (7,), (4, 3)])
def test_gather_rows_grad_is_the_ordered_chain(device, shape):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device(device)
    gen = torch.Generator().manual_seed(3)
    n, m = 300, 6000
    idx = torch.randint(0, n, (m,), generator=gen)
    idx[::3] = 5  # a hub row: 2,000 duplicates
    x = torch.randn((n,) + shape, generator=gen)
    dy = torch.randn((m,) + shape, generator=gen)
    xd = x.to(dev).requires_grad_(True)
    y = kernel.gather_rows(xd, idx.to(dev))
    assert torch.equal(y.detach().cpu(), x[idx])
    y.backward(dy.to(dev))
    F = int(np.prod(shape))
    ref = O.spmm_coo(n, idx.numpy(), np.arange(m), dy.reshape(m, F).numpy())
    assert np.array_equal(xd.grad.cpu().reshape(n, F).numpy(), ref)


def test_gather_rows_empty():
    x = torch.randn(10, 4, requires_grad=True)
    y = kernel.gather_rows(x, torch.zeros(0, dtype=torch.int64))
    assert y.shape == (0, 4)
    y.sum().backward()
    assert torch.equal(x.grad, torch.zeros(10, 4))
