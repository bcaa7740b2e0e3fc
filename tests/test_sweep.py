"""The source-swept schedule of copy_u + sum / mean / sum_accum
(kernel.set_sweep, dglhip_gspmm_sweep_device): one launch in
which every wave holds its rows' partial sums in registers and walks the
source columns slice by slice, each row taking its next slots in slot order
while their column is below the slice's end. A slot is taken only after every
earlier slot of its row, so the chains are the one-launch kernel's for any
slot order: the results must equal it (and the oracle) bit for bit, on
source-major graphs and on graphs in random edge order alike.
"""
import numpy as np
import pytest
import torch

from dgl import kernel
from oracle import oracle as O


def _graph(n, m, seed, sorted_src=False, hub=0):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    if hub:  # one destination with `hub` extra in-edges (a heavy row)
        src = np.concatenate([src, rng.integers(0, n, hub)])
        dst = np.concatenate([dst, np.full(hub, 7)])
    if sorted_src:
        o = np.lexsort((dst, src))
        src, dst = src[o], dst[o]
    return src, dst


@pytest.fixture
def sweep_on():
    old = kernel.set_sweep("on", slice_bytes=1 << 16, rows=8, heavy=256)
    old_b = kernel.set_blocked("off")
    yield
    kernel.set_sweep(*old)
    kernel.set_blocked(old_b)


def test_set_sweep_validates_and_restores():
    old = kernel.set_sweep("off")
    with pytest.raises(Exception):
        kernel.set_sweep("on", rows=5)
    assert kernel.set_sweep(*old)[0] == "off"


@pytest.mark.parametrize("rows", [4, 8, 16])
@pytest.mark.parametrize("skip", [False, True])
def test_plan_covers_every_row_once(rows, skip):
    n, m = 3000, 60_000
    src, dst = _graph(n, m, 3, hub=2000)
    dst[:50] = 0  # keep some rows empty below
    csr = kernel.build_csr(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                           kernel.ORDER_EID, "cpu")
    old = kernel.set_sweep("on", heavy=500)
    try:
        heavy, wr, W = kernel._sweep_plan(csr, rows, skip)
    finally:
        kernel.set_sweep(*old)
    deg = csr.degrees()
    assert wr.numel() == W * rows
    listed = torch.cat([heavy.long(), wr[wr >= 0].long()])
    want = torch.nonzero(deg > 0).squeeze(1) if skip else torch.arange(n)
    assert torch.equal(torch.sort(listed)[0], want)
    assert bool((deg[heavy.long()] >= 500).all())
    assert int((deg[wr[wr >= 0].long()] >= 500).sum()) == 0
    # snake dealing: wave totals within one longest row of each other
    w = wr.view(W, rows).long()
    tot = torch.where(w >= 0, deg[w.clamp(min=0)], torch.zeros_like(w)).sum(1)
    light = deg[wr[wr >= 0].long()]
    assert int(tot.max() - tot.min()) <= int(light.max())


def test_slices_gate():
    csr = kernel.build_csr(4, 4, torch.tensor([0, 1]), torch.tensor([1, 2]), kernel.ORDER_EID,
                           "cpu")
    old = kernel.set_sweep("on", slice_bytes=8)
    try:
        assert kernel._sweep_slices(csr, torch.zeros(4, 3), 3) is None       # odd F
        # columns 1..2 of 16-B rows in 8-B slices: 4 slices of one column
        assert kernel._sweep_slices(csr, torch.zeros(4, 4), 4) == (1, 1, 4)
        kernel.set_sweep("off")
        assert kernel._sweep_slices(csr, torch.zeros(4, 4), 4) is None
    finally:
        kernel.set_sweep(*old)


def _dev():
    return torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("sorted_src", [True, False])
@pytest.mark.parametrize("F", [2, 16, 128, 130, 256])
@pytest.mark.parametrize("rows", [4, 8, 16])
def test_sweep_sum_bits(sweep_on, sorted_src, F, rows):
    n, m = 3000, 60_000
    src, dst = _graph(n, m, F + rows, sorted_src, hub=3000)
    H = np.random.default_rng(1).standard_normal((n, F)).astype(np.float32)
    dev = _dev()
    adj = kernel.from_coo(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                          kernel.ORDER_EID, dev)
    h = torch.from_numpy(H).to(dev)
    kernel.set_sweep("on", slice_bytes=1 << 16, rows=rows, heavy=256)
    assert kernel._sweep_slices(adj.fwd, h, F)[2] >= 2 or F < 16
    out = kernel.gspmm(adj, "copy_u", "sum", h)
    kernel.set_sweep("off")
    ref = kernel.gspmm(adj, "copy_u", "sum", h)
    assert torch.equal(out, ref)
    assert np.array_equal(out.cpu().numpy(), O.spmm_coo(n, dst, src, H))


@pytest.mark.gpu
@pytest.mark.parametrize("sorted_src", [True, False])
def test_sweep_mean_accum_bf16_strided_bits(sweep_on, sorted_src):
    n, m, F = 4000, 80_000, 128
    src, dst = _graph(n, m, 11, sorted_src, hub=5000)
    dst[:100] = 1  # rows 0.. left empty except row 1
    dev = _dev()
    adj = kernel.from_coo(n, n, torch.from_numpy(dst), torch.from_numpy(src),
                          kernel.ORDER_EID, dev)
    csr = adj.fwd
    h = torch.randn(n, F, device=dev)
    hp = torch.randn(n, 144, device=dev)[:, :F]  # padded row stride
    hb = torch.randn(n, F, device=dev).to(torch.bfloat16)
    base = torch.randn(n, F, device=dev)

    def run():
        mean = kernel.gspmm(adj, "copy_u", "mean", h)
        strided = torch.empty(n, F, device=dev)
        kernel.gspmm_into(csr, strided, hp)
        acc = base.clone()
        kernel.gspmm_into(csr, acc, h, accumulate=True)
        b = torch.empty(n, F, device=dev)
        kernel.gspmm_into(csr, b, hb)
        accb = base.clone()
        kernel.gspmm_into(csr, accb, hb, accumulate=True)
        return mean, strided, acc, b, accb

    got = run()
    kernel.set_sweep("off")
    want = run()
    for g, w in zip(got, want):
        assert torch.equal(g, w)


@pytest.mark.gpu
def test_sweep_through_update_all_and_backward(sweep_on):
    import dgl
    import dgl.function as fn
    n, m, F = 2500, 50_000, 64
    src, dst = _graph(n, m, 5, True, hub=1500)
    H = np.random.default_rng(2).standard_normal((n, F)).astype(np.float32)
    G = np.random.default_rng(3).standard_normal((n, F)).astype(np.float32)
    dev = _dev()
    g = dgl.DGLGraph(multigraph=True)
    g.add_nodes(n)
    g.add_edges(src, dst)
    h = torch.from_numpy(H).to(dev).requires_grad_(True)
    g.ndata["h"] = h
    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "o"))
    g.ndata["o"].backward(torch.from_numpy(G).to(dev))
    assert np.array_equal(g.ndata["o"].detach().cpu().numpy(), O.spmm_coo(n, dst, src, H))
    assert np.array_equal(h.grad.cpu().numpy(), O.spmm_coo(n, src, dst, G))
