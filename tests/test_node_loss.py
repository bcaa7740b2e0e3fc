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


@pytest.mark.gpu
@pytest.mark.parametrize("n,C", [(0, 41), (1, 41), (255, 41), (257, 7), (5000, 1), (70001, 41),
                                 (3001, 64), (1 << 20, 41)])
def test_bwd_column_sums(n, C):
    """dglhip_xent_bwd_ex_device: the same dz as the plain backward (bit
    for bit) and colsum = dz.sum(0) to fp32 summation tolerance, reruns
    bit-identical."""
    from dgl import _ffi, kernel
    dev = torch.device("cuda", 0)
    z, y, w = _case(n, C, dev, seed=7 + n, ignore=min(n, 11))
    g = torch.tensor(0.75, device=dev)
    ws = torch.empty(_ffi.LIB.dglhip_xent_colsum_workspace_floats(C), device=dev)
    div = torch.randint(1, 50, (n, 1), generator=torch.Generator().manual_seed(n)).float().to(dev)
    lds = (C + 7) // 8 * 8
    outs = []
    for with_cs, with_sc in ((False, False), (True, False), (True, True)):
        dz = torch.full((n, C), float("nan"), device=dev)
        cs = torch.full((C,), float("nan"), device=dev) if with_cs else None
        sc = torch.full((n, lds), float("nan"), device=dev) if with_sc else None
        _ffi.check_call(_ffi.LIB.dglhip_xent_bwd_ex_device(
            n, C, _ffi.ptr(z), C, _ffi.ptr(y), _ffi.ptr(w), _ffi.ptr(g), _ffi.ptr(dz), C,
            _ffi.ptr(cs), _ffi.ptr(ws), _ffi.ptr(div if with_sc else None), _ffi.ptr(sc),
            lds if with_sc else 0, kernel._stream_of(dev)))
        outs.append((dz, cs))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[1][0], outs[2][0])
    assert torch.equal(outs[1][1], outs[2][1])
    # dz / divisor at the padded stride (torch.div's bits), pad columns zero
    assert torch.equal(sc[:, :C], outs[0][0] / div)
    assert bool((sc[:, C:] == 0).all())
    ref = outs[0][0].double().sum(0)
    tol = 1e-6 * (outs[0][0].double().abs().sum(0) + 1.0)
    assert bool(((outs[1][1].double() - ref).abs() <= tol).all())


@pytest.mark.gpu
@pytest.mark.parametrize("narrow", [True, False])
def test_output_bias_grad_from_loss_kernel(narrow, monkeypatch):
    """The output layer's bias gradient comes from the loss kernel (no column
    reduce over the rows in the Linear's backward) and equals the float64
    expression's; weights and input gradients are unaffected."""
    from dgl.nn.pytorch import NodeLinear, sage_dense
    from dgl.nn.pytorch import linear as L
    dev = torch.device("cuda", 0)
    n, k, C = 70001, 128, 41
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(n, k, generator=gen).to(dev)
    y = torch.randint(0, C, (n,), generator=gen).to(dev)
    w = (torch.rand(n, generator=gen) < 0.5).float().to(dev)
    torch.manual_seed(0)
    fc_self = NodeLinear(k, C).to(dev)
    fc_neigh = NodeLinear(k, C, bias=False).to(dev)

    def agg(t):  # a linear stand-in for the mean aggregation
        return t * 0.5

    def run():
        xx = x.detach().clone().requires_grad_(True)
        z = sage_dense(xx, agg, fc_self, fc_neigh) if narrow else fc_self(xx)
        loss = weighted_cross_entropy(z, y, w) * 0.01
        fc_self.zero_grad()
        fc_neigh.zero_grad()
        loss.backward()
        return z.detach(), fc_self.bias.grad.clone(), fc_self.weight.grad.clone(), xx.grad

    calls = []
    real = L._colsum
    monkeypatch.setattr(L, "_colsum", lambda a: calls.append(a.shape) or real(a))
    z, db, dw, dx = run()
    assert calls == []  # the bias gradient did not run a column reduce
    # float64 reference from the same logits
    z64 = z.double().requires_grad_(True)
    (F.cross_entropy(z64, y, reduction="none") * w.double()).sum().mul(0.01).backward()
    ref = z64.grad.sum(0)
    assert torch.allclose(db.double(), ref, atol=1e-6, rtol=1e-5)
    assert torch.allclose(dw.double(), z64.grad.t().matmul(x.double()), atol=1e-4, rtol=1e-4)
    assert dx is not None and bool(torch.isfinite(dx).all())


@pytest.mark.gpu
def test_out_of_range_labels_are_loud():
    """-100 rows are ignored as PyTorch ignores them; any other label outside
    [0, C) (an error in PyTorch) makes the fused loss and that row's gradient
    NaN instead of contributing nothing."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda", 0)
    z, y, w = _case(1000, 7, dev, ignore=50)
    z = z.requires_grad_(True)
    loss = weighted_cross_entropy(z, y, w)
    ref, _ = _ref(z, y, w)
    assert torch.isfinite(loss) and abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref))
    for bad in (7, -1, 1 << 40):
        yb = y.clone()
        yb[123] = bad
        zb = z.detach().clone().requires_grad_(True)
        lb = weighted_cross_entropy(zb, yb, None)
        assert torch.isnan(lb)
        lb.backward()
        assert torch.isnan(zb.grad[123]).all() and torch.isfinite(zb.grad[:123]).all()


@pytest.mark.gpu
def test_overlapping_rows_take_the_torch_path():
    """A view whose rows overlap (row stride below the class count) is not
    handed to the kernel; the result is PyTorch's."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda", 0)
    base = torch.randn(4000, device=dev)
    z = base.as_strided((1000, 8), (3, 1))
    y = torch.randint(0, 8, (1000,), device=dev)
    loss = weighted_cross_entropy(z, y)
    ref = F.cross_entropy(z, y, reduction="none").sum()
    assert torch.allclose(loss, ref, rtol=1e-6)
