"""Backward hand-offs (dgl/_handoff.py) keyed on the gradient tensor itself.

The loss kernel hands the output layer dz's column sums (its bias gradient)
and dz / deg (its mean aggregation's backward operand); the second layer's
input-gradient kernel hands the first layer its ReLU-masked dx and that
tensor's column sums. Each is taken only by a backward that receives that
very tensor, unmodified. These tests defeat the old address-and-version
match (VERDICT r02 "Next" 6):

* ``autograd.grad(loss, z)`` stops at the logits (the output layer's
  backward never runs, its hand-offs stay attached), then ``z.backward`` with
  another upstream gradient, allocated where the first one lived, at
  version 0;
* the gradient altered in place between the loss and the Linear (a hook);

and check that the hand-offs are taken in a plain step, the gradients in
every case equal those of the same model with no hand-off offered.
"""
import gc

import numpy as np
import pytest
import torch

import dgl
import dgl.function as fn
from dgl import _handoff, kernel
from dgl.nn.pytorch import NodeLinear, sage_dense, weighted_cross_entropy
from dgl.nn.pytorch import linear as L
from dgl.nn.pytorch import loss as LS


# -- GradHandoff semantics (host) -------------------------------------------
def test_handoff_matches_only_the_same_unmodified_tensor():
    a = torch.ones(4)
    h = _handoff.GradHandoff(a, "v")
    assert h.take(a) == "v"
    assert h.take(a.clone()) is None            # equal values, other tensor
    assert h.take(a.view(4)) is None            # a view of it
    a.mul_(2)
    assert h.take(a) is None                    # modified in place


def test_handoff_dies_with_its_tensor():
    a = torch.ones(1 << 20)
    big = torch.zeros(1 << 20)
    h = _handoff.GradHandoff(a, big)
    del big
    del a
    gc.collect()
    b = torch.ones(1 << 20)  # may reuse a's storage: still no match
    assert h.take(b) is None
    assert not h._holder     # the value was dropped when a was freed
    assert _handoff.take(None, b) is None


def test_is_output():
    class Id(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            out = x * 1
            ctx.out_ref = _handoff.output_ref(out)
            return out

        @staticmethod
        def backward(ctx, g):
            return g
    x = torch.ones(3, requires_grad=True)
    y = Id.apply(x)
    assert _handoff.is_output(y.grad_fn, y)
    assert not _handoff.is_output(y.grad_fn, y.view(3))
    assert not _handoff.is_output(y.grad_fn, y.detach())


# -- the model's hand-offs on the device --------------------------------------
@pytest.fixture(scope="module")
def model_case():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    n, m, C = 60_000, 600_000, 41
    g = dgl.DGLGraph((torch.from_numpy(rng.integers(0, n, m)),
                      torch.from_numpy(rng.integers(0, n, m))))

    def aggregate(x):
        g.ndata["x"] = x
        g.update_all(fn.copy_src("x", "m"), fn.mean("m", "a"))
        g.ndata.pop("x")
        return g.ndata.pop("a")
    aggregate.add_into = lambda h, out: kernel.gspmm_mean_add(g.sparse_adjacency(h.device),
                                                              h, out)
    torch.manual_seed(0)
    mods = [NodeLinear(128, 128).to(dev), NodeLinear(128, 128, bias=False).to(dev),
            NodeLinear(128, C).to(dev), NodeLinear(128, C, bias=False).to(dev)]
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(n, 128, generator=gen).to(dev)
    y = torch.randint(0, C, (n,), generator=gen).to(dev)
    w = (torch.rand(n, generator=gen) < 0.5).float().to(dev)
    return dev, aggregate, mods, x, y, w


def _forward(case):
    dev, aggregate, mods, x, y, w = case
    for mm in mods:
        mm.zero_grad(set_to_none=True)
    h = sage_dense(x, aggregate, mods[0], mods[1], torch.relu)
    z = sage_dense(h, aggregate, mods[2], mods[3])
    return z, weighted_cross_entropy(z, y, w) * 1e-3


def _grads(case):
    return [p.grad.clone() for mm in case[2] for p in mm.parameters()]


def _no_handoffs(monkeypatch):
    monkeypatch.setattr(LS, "_bias_producer", lambda z: None)
    monkeypatch.setattr(L, "_relu_producer", lambda x: None)


def _close(a, b):
    for ga, gb in zip(a, b):
        torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-6 * float(gb.abs().max()) + 1e-9)


@pytest.mark.gpu
def test_plain_step_takes_every_handoff(model_case, monkeypatch):
    t0 = dict(_handoff.stats)
    z, loss = _forward(model_case)
    loss.backward()
    fused = _grads(model_case)
    taken = _handoff.stats["taken"] - t0["taken"]
    # dz's column sums; dz / deg (taken by the output layer, passed on to and
    # taken by its mean-add's backward); the masked dx with its column sums
    assert taken == 4, (taken, _handoff.stats)
    assert _handoff.stats["missed"] == t0["missed"]
    with monkeypatch.context() as mp:
        _no_handoffs(mp)
        z, loss = _forward(model_case)
        loss.backward()
        plain = _grads(model_case)
    _close(fused, plain)


@pytest.mark.gpu
def test_grad_stopped_at_logits_then_reused_storage(model_case, monkeypatch):
    """autograd.grad stops at z; the output layer's hand-offs stay attached.
    A new upstream gradient then lands in dz's freed storage at version 0:
    the old (address, version) match would have taken the stale column sums
    and dz / deg."""
    z, loss = _forward(model_case)
    (dz,) = torch.autograd.grad(loss, z, retain_graph=True)
    ptr = dz.data_ptr()
    shape = dz.shape
    del dz
    upstream = torch.full(shape, 0.25, device=z.device)  # version 0
    reused = upstream.data_ptr() == ptr
    t0 = dict(_handoff.stats)
    z.backward(upstream)
    got = _grads(model_case)
    assert _handoff.stats["missed"] > t0["missed"] or not reused
    with monkeypatch.context() as mp:
        _no_handoffs(mp)
        z, loss = _forward(model_case)
        z.backward(torch.full(shape, 0.25, device=z.device))
        want = _grads(model_case)
    _close(got, want)


@pytest.mark.gpu
def test_gradient_modified_in_place_is_not_taken(model_case, monkeypatch):
    def run(mp_ctx):
        z, loss = _forward(model_case)
        z.register_hook(lambda g: g.mul_(3.0))  # same tensor, new version
        loss.backward()
        return _grads(model_case)
    t0 = dict(_handoff.stats)
    got = run(None)
    assert _handoff.stats["missed"] - t0["missed"] >= 2  # column sums and dz / deg
    with monkeypatch.context() as mp:
        _no_handoffs(mp)
        want = run(mp)
    _close(got, want)
