"""kernel.gspmm_mean_add (DGLHIP_REDUCE_MEAN_ACCUM): out <- out + mean over
in-edges, the addition done in the aggregation's own store. The reference
arithmetic is fc_self(h) + mean(...) as two tensors and one sum
(examples/pytorch/graphsage, SURVEY §3: the mean replaces
runtime/degree_bucketing.py:13-84); every check here is against
``out + gspmm(adj, "copy_u", "mean", h)`` on the same engine, bit for bit
(a sum of two terms is the same either way round), forward and backward, on
every schedule the mean takes: one wave per row, the heavy-row split, the
short-row tiers and the padded-stride gather, and on the host path."""
import numpy as np
import pytest
import torch

from dgl import kernel
from dgl.nn.pytorch import NodeLinear, sage_dense


def _graph(rng, n, nnz, skew):
    if skew:  # power-law destinations: a few very long rows, many empty ones
        p = 1.0 / np.arange(1, n + 1) ** 1.1
        row = rng.choice(n, size=nnz, p=p / p.sum())
    else:
        row = rng.integers(0, n, nnz)
    col = rng.integers(0, n, nnz)
    return torch.from_numpy(row.astype(np.int64)), torch.from_numpy(col.astype(np.int64))


def _check(adj, h, base, dev):
    """Fused vs unfused: values and both gradients, bit for bit."""
    h1 = h.detach().clone().requires_grad_(True)
    ref = base + kernel.gspmm(adj, "copy_u", "mean", h1)
    g = torch.randn(ref.shape, generator=torch.Generator().manual_seed(3)).to(dev)
    ref.backward(g)
    h2 = h.detach().clone().requires_grad_(True)
    b2 = base.detach().clone().requires_grad_(True)
    out = kernel.gspmm_mean_add(adj, h2, b2.clone())
    out.backward(g)
    assert torch.equal(out.detach(), ref.detach())
    assert torch.equal(h2.grad, h1.grad)
    assert torch.equal(b2.grad, g)


def test_mean_add_host():
    rng = np.random.default_rng(0)
    n = 2000
    row, col = _graph(rng, n, 12000, skew=True)
    adj = kernel.from_coo(n, n, row, col, kernel.ORDER_EID)
    for F in (1, 7, 41):
        h = torch.randn(n, F)
        base = torch.randn(n, F)
        _check(adj, h, base, torch.device("cpu"))


def test_mean_add_rejects_bad_out():
    adj = kernel.from_coo(4, 4, torch.tensor([0, 1]), torch.tensor([1, 2]), kernel.ORDER_EID)
    h = torch.randn(4, 3)
    with pytest.raises(Exception):
        kernel.gspmm_mean_add(adj, h, torch.zeros(4, 3, dtype=torch.float64))
    with pytest.raises(Exception):
        kernel.gspmm_mean_add(adj, h, torch.zeros(3, 3))
    with pytest.raises(Exception):
        kernel.gspmm_mean_add(adj, h, torch.zeros(4, 6)[:, :3])


@pytest.mark.gpu
@pytest.mark.parametrize("F", [41, 128, 3])
@pytest.mark.parametrize("split", ["off", 2000])
@pytest.mark.parametrize("tiered", [True, False])
def test_mean_add_device_schedules(F, split, tiered):
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(F)
    n = 300_000
    row, col = _graph(rng, n, 900_000, skew=True)
    adj = kernel.from_coo(n, n, row.to(dev), col.to(dev), kernel.ORDER_EID, dev)
    gen = torch.Generator().manual_seed(F)
    h = (torch.rand(n, F, generator=gen) * 2 - 1).to(dev)
    base = torch.randn(n, F, generator=gen).to(dev)
    old_s, old_t = kernel.set_row_split(split), kernel.set_short_rows(tiered)
    try:
        _check(adj, h, base, dev)
        if F == 41:  # rows of a padded-stride view gathered in place (sage_dense's layout)
            hp = torch.zeros(n, 48, device=dev)
            hp[:, :F] = h
            _check(adj, hp[:, :F], base, dev)
    finally:
        kernel.set_row_split(old_s)
        kernel.set_short_rows(old_t)


@pytest.mark.gpu
def test_sage_dense_add_into_equals_sum(monkeypatch):
    """The narrowing SAGE layer with the aggregation's add_into: the same
    output, parameter gradients and input gradient as with the separate sum
    (and the same loss-kernel bias gradient); with add_into, the mean
    backward's dC / deg comes from the loss kernel (no division pass)."""
    from dgl.nn.pytorch import weighted_cross_entropy
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    n, k, C = 200_000, 128, 41
    row, col = _graph(rng, n, 1_500_000, skew=True)
    adj = kernel.from_coo(n, n, row.to(dev), col.to(dev), kernel.ORDER_EID, dev)
    gen = torch.Generator().manual_seed(2)
    x = torch.randn(n, k, generator=gen).to(dev)
    y = torch.randint(0, C, (n,), generator=gen).to(dev)
    w = (torch.rand(n, generator=gen) < 0.5).float().to(dev)
    torch.manual_seed(0)
    fc_self, fc_neigh = NodeLinear(k, C).to(dev), NodeLinear(k, C, bias=False).to(dev)

    def aggregate(t):
        return kernel.gspmm(adj, "copy_u", "mean", t)

    def fused(t):
        return aggregate(t)
    fused.add_into = lambda t, out: kernel.gspmm_mean_add(adj, t, out)

    calls = []
    real = kernel._mean_scaled
    monkeypatch.setattr(kernel, "_mean_scaled",
                        lambda *a, **k: calls.append(1) or real(*a, **k))
    res = []
    for agg in (aggregate, fused):
        calls.clear()
        xx = x.detach().clone().requires_grad_(True)
        z = sage_dense(xx, agg, fc_self, fc_neigh)
        fc_self.zero_grad()
        fc_neigh.zero_grad()
        (weighted_cross_entropy(z, y, w) * 1e-3).backward()
        res.append((z.detach(), xx.grad, fc_self.weight.grad.clone(), fc_self.bias.grad.clone(),
                    fc_neigh.weight.grad.clone()))
        assert len(calls) == (1 if agg is aggregate else 0)
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("F,strided", [(41, False), (41, True), (128, False), (16, False)])
def test_mean_add_blocked_schedule(F, strided):
    """mean_add on the source-blocked schedule (r06: the chains in rows of
    their own, sum / deg added to out at the end): the plan takes the blocked
    path, and values and gradients equal the unfused out + mean bit for bit
    (padded F = 41 copies, a row-padded view read in place, empty rows)."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11 + F)
    n = 60_000
    # uniform rows (a hub row past the heavy-row threshold keeps the one-launch
    # schedule), some rows empty
    row, col = _graph(rng, n, 1_500_000, skew=False)
    keep = row % 17 != 0
    row, col = row[keep], col[keep]
    o = np.lexsort((row.numpy(), col.numpy()))  # source-major edge numbering
    row, col = row[o], col[o]
    from dgl._ffi import LIB
    old_knob = LIB.dglhip_set_blocked_mean_add(1)
    with kernel.scheduled(block_table_min=0, block_bytes=1 << 20, block_min_row_bytes=0,
                          block_min_slots=1):
        adj = kernel.from_coo(n, n, row.to(dev), col.to(dev), kernel.ORDER_EID, dev)
        gen = torch.Generator().manual_seed(F)
        h = (torch.rand(n, F, generator=gen) * 2 - 1).to(dev)
        base = torch.randn(n, F, generator=gen).to(dev)
        if strided:
            hp = torch.zeros(n, 48, device=dev)
            hp[:, :F] = h
            h = hp[:, :F]
        ldu = h.stride(0) if strided else 0
        path, launches = adj.fwd.plan.schedule(kernel.MSG_COPY_U, kernel.RED_MEAN_ACCUM, F, ldu, n)
        try:
            assert path == kernel.PLAN_PATH_BLOCKED and launches > 1
            _check(adj, h, base, dev)
        finally:
            LIB.dglhip_set_blocked_mean_add(old_knob)
