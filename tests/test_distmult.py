"""The fused DistMult decoder (kernel.distmult_score, csrc/typed_block.hip):
R-GCN link prediction's score (the reference's calc_score,
examples/pytorch/rgcn/link_predict.py:50-55, s = h[s] * w[r] * h[o],
score = s.sum(1)) in one kernel, and its gradients as ordered chains.

* gradients: the bits of the torch formulation the fused model used before
  (gather_rows(h, cat(s, o)) split, times gather_rows(w, r), its duplicates
  summed by gather_rows' chains) — every term and chain is the same;
* scores: within 1e-6 of that formulation's (the sum runs in the kernel's
  lane-chain + butterfly order, not torch's) and of float64;
* host = device bit for bit; out-of-range indices give NaN, not a fault.
"""
import numpy as np
import pytest
import torch

import dgl
from dgl import kernel

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device(device)


def _case(N=700, R=40, F=500, n=3000, seed=0, hub=True):
    gen = torch.Generator().manual_seed(seed)
    h = torch.randn(N, F, generator=gen)
    w = torch.randn(R, F, generator=gen)
    s = torch.randint(0, N, (n,), generator=gen)
    o = torch.randint(0, N, (n,), generator=gen)
    r = torch.randint(0, R, (n,), generator=gen)
    if hub:  # a hub entity and relation of > DGLHIP_TYPED_CHUNK positions
        s[::7] = 3
        r[::5] = 1
    return h, w, s, r, o


def _torch_form(h, w, s, r, o):
    n = s.numel()
    ho = kernel.gather_rows(h, torch.cat([s, o]))
    return (ho[:n] * kernel.gather_rows(w, r) * ho[n:]).sum(1)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("F", [500, 64, 37])
def test_distmult_grads_bits_of_the_torch_form(device, F):
    dev = _dev(device)
    h, w, s, r, o = (t.to(dev) for t in _case(F=F))
    h1, w1 = h.clone().requires_grad_(True), w.clone().requires_grad_(True)
    h2, w2 = h.clone().requires_grad_(True), w.clone().requires_grad_(True)
    sc = kernel.distmult_score(h1, w1, s, r, o)
    ref = _torch_form(h2, w2, s, r, o)
    exact = (h.double()[s] * w.double()[r] * h.double()[o]).sum(1)
    mag = (h.double()[s] * w.double()[r] * h.double()[o]).abs().sum(1)
    assert ((sc.double() - exact).abs() <= 1e-6 * mag + 1e-30).all()
    assert ((ref.double() - exact).abs() <= 1e-6 * mag + 1e-30).all()
    dsc = torch.randn(s.numel(), generator=torch.Generator().manual_seed(3)).to(dev)
    g1 = torch.autograd.grad(sc, (h1, w1), dsc)
    g2 = torch.autograd.grad(ref, (h2, w2), dsc)
    assert torch.equal(g1[0], g2[0]) and torch.equal(g1[1], g2[1])


@pytest.mark.parametrize("device", DEVICES)
def test_distmult_only_one_grad_and_empty(device):
    dev = _dev(device)
    h, w, s, r, o = (t.to(dev) for t in _case(n=500, hub=False))
    h1 = h.clone().requires_grad_(True)
    (dh,) = torch.autograd.grad(kernel.distmult_score(h1, w, s, r, o).sum(), (h1,))
    h2 = h.clone().requires_grad_(True)
    (dh2,) = torch.autograd.grad(_torch_form(h2, w, s, r, o).sum(), (h2,))
    assert torch.equal(dh, dh2)
    e = torch.empty(0, dtype=torch.int64, device=dev)
    h3 = h.clone().requires_grad_(True)
    sc = kernel.distmult_score(h3, w, e, e, e)
    assert sc.shape == (0,)
    (dh3,) = torch.autograd.grad(sc.sum(), (h3,), allow_unused=True)
    assert dh3 is None or not dh3.any()


@pytest.mark.parametrize("device", DEVICES)
def test_distmult_out_of_range_raises(device):
    """Out-of-range subject, relation or object ids raise IndexError at the
    call, as index_select in the torch formulation does, rather
    than surfacing later as a NaN loss; the kernel itself never reads past
    its tables (NaN for such a position)."""
    dev = _dev(device)
    old = kernel.set_validate_indices(True)  # device-resident ids: checked on request
    try:
        for which, bad in ((0, "s"), (1, "r"), (2, "o"), (1, "neg")):
            h, w, s, r, o = _case(n=10, hub=False)
            t = [s, r, o][which]
            t[4] = -1 if bad == "neg" else (w.shape[0] if which == 1 else h.shape[0])
            with pytest.raises(IndexError):
                kernel.distmult_score(h.to(dev), w.to(dev), s.to(dev), r.to(dev), o.to(dev))
            # host-resident ids are checked whatever the setting
            kernel.set_validate_indices(False)
            with pytest.raises(IndexError):
                kernel.distmult_score(h.to(dev), w.to(dev), s, r, o)
            kernel.set_validate_indices(True)
    finally:
        kernel.set_validate_indices(old)
    h, w, s, r, o = _case(n=10, hub=False)
    s[4] = h.shape[0]
    r[6] = -1
    sc = kernel._DistMult.apply(h, w, s, r, o)  # the kernel without the check
    assert torch.isnan(sc[4]) and torch.isnan(sc[6])
    assert torch.isfinite(sc[[0, 1, 2, 3, 5, 7, 8, 9]]).all()


@pytest.mark.gpu
def test_distmult_host_equals_device():
    dev = _dev("cuda")
    h, w, s, r, o = _case()
    dsc = torch.randn(s.numel(), generator=torch.Generator().manual_seed(4))
    res = []
    for d in (torch.device("cpu"), dev):
        hh, ww = h.to(d).requires_grad_(True), w.to(d).requires_grad_(True)
        sc = kernel.distmult_score(hh, ww, s.to(d), r.to(d), o.to(d))
        g = torch.autograd.grad(sc, (hh, ww), dsc.to(d))
        res.append([sc.detach().cpu(), g[0].cpu(), g[1].cpu()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("F", [500, 37])
def test_distmult_link_loss_matches_float64(device, F):
    """kernel.distmult_link_loss (the example's get_loss: BCE-with-logits of
    the scores, mean, + reg * (mean(h^2) + mean(w^2))) — fused on a device,
    the torch expression on the host — against float64: the loss within 1e-5
    of its terms' magnitudes, the scores with distmult_score's bits, every
    gradient element within 1e-5 of its Σ|terms| (hub rows of several chunks
    and rows no triple touches included)."""
    dev = _dev(device)
    h, w, s, r, o = _case(F=F, N=900)  # rows past 700 see no triple
    s, o = s % 700, o % 700
    labels = (torch.arange(s.numel()) % 2).float()
    reg = 0.01
    h1, w1 = h.clone().to(dev).requires_grad_(True), w.clone().to(dev).requires_grad_(True)
    loss = kernel.distmult_link_loss(h1, w1, s.to(dev), r.to(dev), o.to(dev), labels.to(dev), reg)
    loss.backward()
    h2, w2 = h.double().requires_grad_(True), w.double().requires_grad_(True)
    score = (h2[s] * w2[r] * h2[o]).sum(1)
    ref = (torch.nn.functional.binary_cross_entropy_with_logits(score, labels.double()) +
           reg * (h2.pow(2).mean() + w2.pow(2).mean()))
    ref.backward()
    with torch.no_grad():
        mag_s = (h2[s] * w2[r] * h2[o]).abs().sum(1)
        lmag = (mag_s + 1.0).mean() + reg * (h2.pow(2).mean() + w2.pow(2).mean())
    assert abs(float(loss) - float(ref)) <= 1e-5 * float(lmag)
    # gradient bounds: the same chains over magnitudes
    ha, wa = h.double().abs().requires_grad_(True), w.double().abs().requires_grad_(True)
    with torch.no_grad():
        # |sigmoid| + |label|: the Σ|terms| of the BCE gradient's subtraction
        # (saturated logits cancel it)
        ds = (torch.sigmoid(score) + labels.double()) / s.numel()
    lm = (ds * (ha[s] * wa[r] * ha[o]).sum(1)).sum() + reg * (ha.pow(2).mean() +
                                                             wa.pow(2).mean())
    lm.backward()
    for got, want, bound in ((h1.grad, h2.grad, ha.grad), (w1.grad, w2.grad, wa.grad)):
        err = (got.double().cpu() - want).abs()
        assert bool((err <= 1e-5 * bound + 1e-30).all()), float((err / (bound + 1e-30)).max())
