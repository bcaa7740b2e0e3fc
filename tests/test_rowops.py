"""Row passes of the g-SpMM autograd (csrc/rowops.hip): the mean reducer's
backward division written into the padded rows of the transposed product."""
import numpy as np
import pytest
import torch

from dgl import _ffi, kernel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("n,F,ld", [(1, 1, 1), (255, 41, 48), (257, 41, 41), (1000, 7, 9),
                                    (3000, 64, 64), (100, 600, 608)])
def test_div_rows_equals_torch_div(cuda, n, F, ld):
    rng = np.random.default_rng(n + F)
    x = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(cuda)
    x[::5] *= 1e-38  # subnormal quotients too
    d = torch.from_numpy(rng.integers(1, 5000, (n, 1)).astype(np.float32)).to(cuda)
    buf = torch.full((n, ld), 7.0, device=cuda)
    _ffi.check_call(_ffi.LIB.dglhip_div_rows_device(n, F, _ffi.ptr(x), F, _ffi.ptr(d),
                                                    _ffi.ptr(buf), ld, kernel._stream_of(cuda)))
    assert torch.equal(buf[:, :F], x / d)
    assert bool(((buf[:, F:] == 7.0) | (buf[:, F:] == 0.0)).all())  # pad: untouched or zeros


def test_mean_backward_padded_equals_unpadded(cuda):
    """dH of copy_u + mean at F = 41: the quotient written into the padded
    rows gives the bits of the plain division + contiguous gather."""
    rng = np.random.default_rng(2)
    n, m, F = 300_000, 2_000_000, 41
    src = torch.from_numpy(rng.integers(0, n, m))
    dst = torch.from_numpy((rng.pareto(1.2, m) * 50).astype(np.int64) % n)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, cuda)
    h = torch.from_numpy(rng.uniform(-1, 1, (n, F)).astype(np.float32)).to(cuda)
    g = torch.from_numpy(rng.uniform(-1, 1, (n, F)).astype(np.float32)).to(cuda)
    grads = []
    for policy in ("auto", "off"):
        old = kernel.set_pad_rows(policy)
        try:
            hh = h.clone().requires_grad_(True)
            kernel.gspmm(adj, "copy_u", "mean", hh).backward(g)
            grads.append(hh.grad)
        finally:
            kernel.set_pad_rows(old)
    assert torch.equal(grads[0], grads[1])
