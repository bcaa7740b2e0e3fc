"""kernel.gather_rows: x[idx] whose backward sums each row's duplicates
deterministically (used by the R-GCN example's DistMult decoder): chains of
kernel.TYPED_CHUNK positions in increasing order, a long row's chunk sums
added in order — restated here in numpy float32, bit for bit, host and
device; rows of at most one chunk equal the oracle's nnz-order chain; the
whole gradient is within fp32 summation tolerance of a float64 sum; forward
equals index_select."""
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
    got = xd.grad.cpu().reshape(n, F).numpy()
    d2 = dy.reshape(m, F).numpy()
    ref = _chunked(n, idx.numpy(), d2)
    assert np.array_equal(got, ref)
    chain = O.spmm_coo(n, idx.numpy(), np.arange(m), d2)
    short = np.bincount(idx.numpy(), minlength=n) <= kernel.TYPED_CHUNK
    assert np.array_equal(got[short], chain[short])
    exact = np.zeros((n, F))
    np.add.at(exact, idx.numpy(), d2.astype(np.float64))
    assert np.allclose(got, exact, rtol=1e-5, atol=1e-4)


def _chunked(n, idx, dy):
    """The kernel's order: per row, its positions ascending in chunks of
    TYPED_CHUNK, each chunk's sum a float32 chain from zero, the chunk sums
    added in order."""
    C = kernel.TYPED_CHUNK
    out = np.zeros((n, dy.shape[1]), np.float32)
    for r in np.unique(idx):
        pos = np.nonzero(idx == r)[0]
        tot = None
        for c in range(0, len(pos), C):
            part = np.zeros(dy.shape[1], np.float32)
            for i in pos[c:c + C]:
                part = part + dy[i]
            tot = part if tot is None else tot + part
        out[r] = tot
    return out


def test_gather_rows_empty():
    x = torch.randn(10, 4, requires_grad=True)
    y = kernel.gather_rows(x, torch.zeros(0, dtype=torch.int64))
    assert y.shape == (0, 4)
    y.sum().backward()
    assert torch.equal(x.grad, torch.zeros(10, 4))
