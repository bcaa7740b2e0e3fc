"""DGLHIP_REDUCE_SUM_ACCUM (kernel.gspmm_into(..., accumulate=True)): one
product evaluated segment by segment, the way dgl.distributed's pipelined
forward reduces its own-source and halo segments. Splitting a row's edges
into segments S0, S1, ... and reducing them in turn must equal the single
sequential chain over the edges ordered (segment, edge id) — bit for bit,
against the oracle's restatement of the reference's product. Under a forced
heavy-row split the chunk partials are added in order: deterministic, and
within 1e-5 x sum|terms| of the exact sum (as the sequential chain is).
"""
import numpy as np
import pytest
import torch

from dgl import kernel
from oracle import oracle as O

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device(device)


def _case(seed, n=500, nnz=40000, F=64, segs=3):
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, n + 1) ** 1.2
    row = rng.choice(n, size=nnz, p=p / p.sum()).astype(np.int64)
    col = rng.integers(0, n, nnz).astype(np.int64)
    seg = rng.integers(0, segs, nnz)
    H = rng.standard_normal((n, F)).astype(np.float32)
    return n, row, col, seg, H


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("F", [1, 41, 128])
def test_segments_equal_one_chain(device, F):
    dev = _dev(device)
    n, row, col, seg, H = _case(F, F=F)
    Hd = torch.from_numpy(H).to(dev)
    out = torch.full((n, F), float("nan"), device=dev)
    for s in range(seg.max() + 1):
        m = seg == s
        csr = kernel.build_csr(n, n, row[m], col[m], kernel.ORDER_EID, dev)
        kernel.gspmm_into(csr, out, Hd, accumulate=s > 0)
    order = np.lexsort((np.arange(len(row)), seg))  # (segment, edge id)
    ref = O.spmm_coo(n, row[order], col[order], H)
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
def test_segments_with_heavy_row_chunks():
    dev = _dev("cuda")
    n, row, col, seg, H = _case(5, nnz=200000, F=128)
    Hd = torch.from_numpy(H).to(dev)
    csrs = []
    for s in range(seg.max() + 1):
        m = seg == s
        csrs.append(kernel.build_csr(n, n, row[m], col[m], kernel.ORDER_EID, dev))
    order = np.lexsort((np.arange(len(row)), seg))
    ref = O.spmm_coo(n, row[order], col[order], H)
    outs = []
    old = kernel.set_row_split(256)
    try:  # the longest rows hold thousands of slots
        assert max(c.max_degree for c in csrs) > 4 * 256
        for _ in range(2):
            out = torch.empty(n, 128, device=dev)
            for s, csr in enumerate(csrs):
                kernel.gspmm_into(csr, out, Hd, accumulate=s > 0)
            outs.append(out.cpu().numpy())
    finally:
        kernel.set_row_split(old)
    assert np.array_equal(outs[0], outs[1])
    # reassociated sums: judge both orders against the exact (float64) sum, with
    # the fp32 summation bound scaled by sum |terms| (the reference chain itself
    # is 4e-6 * sum|x| off at these degrees)
    exact = np.zeros((n, 128))
    np.add.at(exact, row, H[col].astype(np.float64))
    mag = np.zeros((n, 128))
    np.add.at(mag, row, np.abs(H[col]).astype(np.float64))
    assert np.all(np.abs(outs[0] - exact) <= 1e-5 * mag + 1e-6)
    assert np.all(np.abs(ref - exact) <= 1e-5 * mag + 1e-6)


def test_gspmm_into_checks_shapes():
    n, row, col, seg, H = _case(1, n=50, nnz=300, F=8)
    csr = kernel.build_csr(n, n, row, col, kernel.ORDER_EID, "cpu")
    with pytest.raises(Exception):
        kernel.gspmm_into(csr, torch.empty(n - 1, 8), torch.from_numpy(H))
    with pytest.raises(Exception):
        kernel.gspmm_into(csr, torch.empty(n, 8), torch.from_numpy(H[:10]))


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("F", [1, 2, 41, 128, 256])
def test_bf16_rows_equal_widened_fp32(device, F):
    """DGLHIP_MSG_COPY_U_BF16 (gspmm_into on bfloat16 rows, the bf16 halo's
    segments): segment 0 reads fp32 rows, the others bf16 rows; the result is
    the oracle's chain in (segment, edge id) order over the bf16 rows widened
    to fp32, bit for bit. F = 1 / 41 take the scalar lanes, 2 / 128 / 256 the
    two-value loads."""
    dev = _dev(device)
    n, row, col, seg, H = _case(11 + F, F=F)
    Hd = torch.from_numpy(H).to(dev)
    Hb = Hd.to(torch.bfloat16)
    Hw = Hb.float().cpu().numpy()  # the widened rows the bf16 segments see
    out = torch.full((n, F), float("nan"), device=dev)
    for s in range(seg.max() + 1):
        m = seg == s
        csr = kernel.build_csr(n, n, row[m], col[m], kernel.ORDER_EID, dev)
        kernel.gspmm_into(csr, out, Hd if s == 0 else Hb, accumulate=s > 0)
    order = np.lexsort((np.arange(len(row)), seg))
    # the chain over rows that are fp32 in segment 0 and widened bf16 after
    X = np.concatenate([H, Hw], 0)
    src = np.where(seg[order] == 0, col[order], col[order] + n)
    ref = O.spmm_coo(n, row[order], src, X)
    assert np.array_equal(out.cpu().numpy(), ref)
    # one bf16 product on its own equals the fp32 product on the widened rows
    csr = kernel.build_csr(n, n, row, col, kernel.ORDER_EID, dev)
    one = kernel.gspmm_into(csr, torch.empty(n, F, device=dev), Hb)
    assert np.array_equal(one.cpu().numpy(), O.spmm_coo(n, row, col, Hw))


@pytest.mark.gpu
def test_bf16_rows_heavy_row_chunks():
    """bf16 rows through the heavy-row split (chunk partials + combine)."""
    dev = _dev("cuda")
    n, row, col, seg, H = _case(6, nnz=200000, F=128)
    Hb = torch.from_numpy(H).to(dev).to(torch.bfloat16)
    Hw = torch.from_numpy(H).to(dev).to(torch.bfloat16).float()
    csr = kernel.build_csr(n, n, row, col, kernel.ORDER_EID, dev)
    old = kernel.set_row_split(256)
    try:
        assert csr.max_degree > 4 * 256
        a = kernel.gspmm_into(csr, torch.empty(n, 128, device=dev), Hb)
        b = kernel.gspmm_into(csr, torch.empty(n, 128, device=dev), Hw)
    finally:
        kernel.set_row_split(old)
    assert torch.equal(a, b)
