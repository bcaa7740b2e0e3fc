"""weighted_cross_entropy (dgl.nn.pytorch.loss, csrc/node_loss.hip): the
fused node-row cross-entropy against PyTorch's own expression, in float64.

Tolerances: fp32 rounding of a sum of N per-row losses (relative 1e-5 on the
loss) and of one softmax per element (absolute 1e-6 scaled by the upstream
gradient on dz)."""
import pytest
import torch
import torch.nn.functional as F

from dgl.nn.pytorch import weighted_cross_entropy


def _ref(z, y, w, g=1.0):
    z64 = z.detach().double().requires_grad_(True)
    ce = F.cross_entropy(z64, y, reduction="none")
    loss = (ce * w.double()).sum() if w is not None else ce.sum()
    (loss * g).backward()
    return loss.detach(), z64.grad


def _case(n, C, dev, seed=0, ignore=0, ld=None):
    gen = torch.Generator().manual_seed(seed)
    base = torch.randn(n, ld or C, generator=gen) * 3.0
    z = base[:, :C]
    y = torch.randint(0, C, (n,), generator=gen)
    if ignore and n:
        y[torch.randperm(n, generator=gen)[:ignore]] = -100
    w = (torch.rand(n, generator=gen) < 0.6).float()
    return z.to(dev) if ld is None else base.to(dev)[:, :C], y.to(dev), w.to(dev)


def test_host_matches_expression():
    z, y, w = _case(500, 7, "cpu", ignore=5)
    z.requires_grad_(True)
    loss = weighted_cross_entropy(z, y, w)
    loss.backward()
    rl, rg = _ref(z, y, w)
    assert abs(loss.item() - rl.item()) <= 1e-5 * abs(rl.item())
    assert torch.allclose(z.grad.double(), rg, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("n,C,ld", [(0, 41, None), (1, 41, None), (255, 41, None),
                                    (257, 41, None), (1000, 1, None), (3001, 2, None),
                                    (4099, 40, None), (2048, 64, None), (1500, 41, 48),
                                    (777, 16, 20)])
def test_fused_matches_expression(n, C, ld):
    dev = torch.device("cuda", 0)
    z, y, w = _case(n, C, dev, seed=n + C, ignore=min(n, 3), ld=ld)
    for weight in (w, None):
        zz = z.detach().clone() if ld is None else z.detach()
        zz.requires_grad_(True)
        loss = weighted_cross_entropy(zz, y, weight)
        (loss * 2.5).backward()
        rl, rg = _ref(zz, y, weight, 2.5)
        assert loss.dtype == torch.float32 and loss.dim() == 0
        assert abs(loss.item() - rl.item()) <= 1e-5 * max(1.0, abs(rl.item())), (loss, rl)
        assert zz.grad.shape == (n, C)
        assert torch.allclose(zz.grad.double(), rg, atol=2.5e-6, rtol=1e-5)
        if n:
            assert bool((zz.grad[y < 0] == 0).all())


@pytest.mark.gpu
def test_fused_large_and_deterministic():
    """Many workgroups and tiles (1M rows, 41 classes); bit-identical reruns."""
    dev = torch.device("cuda", 0)
    z, y, w = _case(1 << 20, 41, dev, seed=3)
    z.requires_grad_(True)
    a = weighted_cross_entropy(z, y, w)
    a.backward()
    ga = z.grad.clone()
    z.grad = None
    b = weighted_cross_entropy(z, y, w)
    b.backward()
    assert a.item() == b.item() and torch.equal(ga, z.grad)
    rl, rg = _ref(z, y, w)
    assert abs(a.item() - rl.item()) <= 1e-5 * abs(rl.item())
    assert torch.allclose(ga.double(), rg, atol=1e-6, rtol=1e-5)


@pytest.mark.gpu
def test_fused_path_runs_native():
    from dgl.nn.pytorch import loss as L
    dev = torch.device("cuda", 0)
    z, y, w = _case(300, 41, dev)
    assert L._fused_ok(z, y, w)
    out = weighted_cross_entropy(z.requires_grad_(True), y, w)
    assert type(out.grad_fn).__name__ == "_WeightedXentFnBackward"
