"""The f32 MFMA node Linear (csrc/node_linear.hip) and its use by sage_dense.

* layout: integer-valued operands keep every f32 fma exact, so the kernels
  must equal a float64 product bit for bit (any lane/register mix-up of the
  v_mfma_f32_16x16x4_f32 operand maps, an asymmetric weight included, shows);
* accuracy: random operands within the f32 summation bound of a float64
  product (|err| <= 1e-6 * sum |x w| per element);
* a row-padded g-SpMM input is gathered in place with the same bits as the
  contiguous copy;
* sage_dense on the device (MFMA path) equals the unfused layer.
"""
import numpy as np
import pytest
import torch

import dgl
import dgl.function as fn
from dgl import kernel
from dgl.nn.pytorch import NodeLinear, sage_dense
from dgl.nn.pytorch import linear as L

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda", 0)


def _ints(rng, shape, lo=-3, hi=4):
    return torch.from_numpy(rng.integers(lo, hi, shape).astype(np.float32))


@pytest.mark.parametrize("k", [64, 128, 256])
@pytest.mark.parametrize("m1,m2", [(1, 0), (16, 0), (41, 41), (64, 41), (41, 64), (7, 3)])
def test_forward_exact_integers(cuda, k, m1, m2):
    rng = np.random.default_rng(k * 1000 + m1 * 10 + m2)
    n = 1000 + 13  # not a multiple of 16: the last block is partial
    x = _ints(rng, (n, k)).to(cuda)
    w1 = _ints(rng, (m1, k), -2, 3).to(cuda)
    w2 = _ints(rng, (max(m2, 1), k), -2, 3).to(cuda)
    b2 = _ints(rng, (max(m2, 1),)).to(cuda)
    ld1 = kernel.padded_width(m1) if m1 > 1 else m1
    if m2 == 0:
        y1 = torch.empty(n, ld1, device=cuda)
        from dgl import _ffi
        _ffi.check_call(_ffi.LIB.dglhip_node_linear_device(
            n, k, _ffi.ptr(x), k, m1, _ffi.ptr(w1), None, _ffi.ptr(y1), ld1, 0, None, None,
            None, 0, kernel._stream_of(cuda)))
        y1 = y1[:, :m1]
    else:
        y1, y2 = L._node_linear2(x, w1, ld1, w2, b2)
        ref2 = x.double() @ w2.double().t() + b2.double()
        assert torch.equal(y2.double(), ref2)
    ref1 = x.double() @ w1.double().t()
    assert torch.equal(y1.double(), ref1)


@pytest.mark.parametrize("k", [64, 128])
@pytest.mark.parametrize("m1,m2", [(41, 41), (41, 0), (64, 64), (3, 41), (16, 8)])
def test_dgrad_exact_integers(cuda, k, m1, m2):
    rng = np.random.default_rng(k + m1 * 7 + m2)
    n = 777
    dy1 = _ints(rng, (n, m1)).to(cuda)
    w1 = _ints(rng, (m1, k), -2, 3).to(cuda)
    if m2:
        # the second gradient as a row-padded view, as sage_dense passes it
        buf = _ints(rng, (n, m2 + 6)).to(cuda)
        dy2 = buf[:, :m2]
        w2 = _ints(rng, (m2, k), -2, 3).to(cuda)
        dx = L._node_dgrad2(k, dy1, w1, dy2, w2)
        ref = dy1.double() @ w1.double() + dy2.double() @ w2.double()
    else:
        from dgl import _ffi
        dx = torch.empty(n, k, device=cuda)
        _ffi.check_call(_ffi.LIB.dglhip_node_linear_dgrad_device(
            n, k, m1, _ffi.ptr(dy1), m1, _ffi.ptr(w1), 0, None, 0, None, _ffi.ptr(dx), k,
            None, 0, None, None, kernel._stream_of(cuda)))
        ref = dy1.double() @ w1.double()
    assert torch.equal(dx.double(), ref)


def test_forward_random_within_summation_bound(cuda):
    rng = np.random.default_rng(5)
    n, k, m1, m2 = 50_000, 128, 41, 41
    x = torch.from_numpy(rng.standard_normal((n, k)).astype(np.float32)).to(cuda)
    w1 = torch.from_numpy(rng.standard_normal((m1, k)).astype(np.float32)).to(cuda)
    w2 = torch.from_numpy(rng.standard_normal((m2, k)).astype(np.float32)).to(cuda)
    b2 = torch.from_numpy(rng.standard_normal(m2).astype(np.float32)).to(cuda)
    y1, y2 = L._node_linear2(x, w1, 48, w2, b2)
    for y, w, b in ((y1, w1, None), (y2, w2, b2)):
        ref = x.double() @ w.double().t() + (0 if b is None else b.double())
        bound = x.double().abs() @ w.double().abs().t() + (0 if b is None else b.double().abs())
        assert ((y.double() - ref).abs() <= 1e-6 * bound + 1e-30).all()


@pytest.mark.parametrize("red", ["sum", "mean"])
def test_gspmm_gathers_row_padded_input_in_place(cuda, red):
    rng = np.random.default_rng(9)
    n, m, F = 200_000, 1_500_000, 41
    src = torch.from_numpy(rng.integers(0, n, m))
    dst = torch.from_numpy(rng.integers(0, n, m))
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, cuda)
    buf = torch.from_numpy(rng.uniform(-1, 1, (n, 48)).astype(np.float32)).to(cuda)
    view = buf[:, :F]
    assert kernel._row_strided(view, F)
    a = kernel.gspmm(adj, "copy_u", red, view)
    b = kernel.gspmm(adj, "copy_u", red, view.contiguous())
    assert torch.equal(a, b)
    # and through autograd: the gradient of the view is the transposed product
    v = view.detach().requires_grad_(True)
    g = torch.from_numpy(rng.uniform(-1, 1, (n, F)).astype(np.float32)).to(cuda)
    kernel.gspmm(adj, "copy_u", red, v).backward(g)
    c = view.contiguous().requires_grad_(True)
    kernel.gspmm(adj, "copy_u", red, c).backward(g)
    assert torch.equal(v.grad, c.grad)


def test_sage_dense_mfma_matches_unfused(cuda):
    import copy
    rng = np.random.default_rng(3)
    n, m, fin, fout = 100_000, 800_000, 128, 41
    g = dgl.DGLGraph((torch.from_numpy(rng.integers(0, n, m)),
                      torch.from_numpy(rng.integers(0, n, m))))

    def aggregate(x):
        g.ndata["x"] = x
        g.update_all(fn.copy_src("x", "m"), fn.mean("m", "a"))
        g.ndata.pop("x")
        return g.ndata.pop("a")

    torch.manual_seed(0)
    fs, fnb = NodeLinear(fin, fout).to(cuda), NodeLinear(fin, fout, bias=False).to(cuda)
    rs, rnb = copy.deepcopy(fs), copy.deepcopy(fnb)
    x = torch.randn(n, fin, device=cuda)
    dy = torch.randn(n, fout, device=cuda)
    assert L._mfma_fwd_ok(x, fout, fout)
    xa = x.clone().requires_grad_(True)
    ref = rs(xa) + rnb(aggregate(xa))
    ref.backward(dy)
    xb = x.clone().requires_grad_(True)
    out = sage_dense(xb, aggregate, fs, fnb)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    out.backward(dy)
    torch.testing.assert_close(xb.grad, xa.grad, rtol=1e-5, atol=1e-5)
    # weight gradients sum 10^5 rows, and dWn is (A^T dy)^T x here against
    # dy^T (A x) there: equal up to the summation bound of that many terms
    for a, b in ((fs.weight, rs.weight), (fs.bias, rs.bias), (fnb.weight, rnb.weight)):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-4,
                                   atol=1e-5 * float(b.grad.abs().max()))


@pytest.mark.parametrize("k,m", [(128, 128), (128, 100), (128, 65), (128, 41), (64, 100), (64, 16)])
def test_cat_exact_integers(cuda, k, m):
    """y = x1 W1^T + x2 W2^T + b (sage_dense's square / widening layer)."""
    rng = np.random.default_rng(k + m)
    n = 2000 + 5
    x1, x2 = _ints(rng, (n, k)).to(cuda), _ints(rng, (n, k)).to(cuda)
    w1, w2 = _ints(rng, (m, k), -2, 3).to(cuda), _ints(rng, (m, k), -2, 3).to(cuda)
    b = _ints(rng, (m,)).to(cuda)
    # sage_dense routes up to 64 outputs here, 128 from 128-column inputs
    # (one pass), or 128 with a fused ReLU
    assert L._mfma_cat_ok(x1, x2, m) == (m <= 64 or k == 128)
    assert L._mfma_cat_ok(x1, x2, m, relu=True)
    y = L._node_linear_cat(x1, w1, x2, w2, b)
    ref = x1.double() @ w1.double().t() + x2.double() @ w2.double().t() + b.double()
    assert torch.equal(y.double(), ref)
    yr = L._node_linear_cat(x1, w1, x2, w2, b, relu=True)
    assert torch.equal(yr.double(), ref.clamp(min=0))


@pytest.mark.parametrize("n", [0, 1, 15, 17])
def test_tiny_row_counts(cuda, n):
    """Empty inputs return without a launch; 1..17 rows (one partial block or
    a full one plus one row) match the float64 product exactly."""
    rng = np.random.default_rng(n)
    k, m = 128, 41
    x = _ints(rng, (n, k)).to(cuda)
    w1, w2 = _ints(rng, (m, k), -2, 3).to(cuda), _ints(rng, (m, k), -2, 3).to(cuda)
    b = _ints(rng, (m,)).to(cuda)
    y1, y2 = L._node_linear2(x, w1, 48, w2, b)
    assert y1.shape == (n, m) and y2.shape == (n, m)
    assert torch.equal(y1.double(), x.double() @ w1.double().t())
    assert torch.equal(y2.double(), x.double() @ w2.double().t() + b.double())
    dy1, dy2 = _ints(rng, (n, m)).to(cuda), _ints(rng, (n, m)).to(cuda)
    dx = L._node_dgrad2(k, dy1, w1, dy2, w2)
    assert torch.equal(dx.double(), dy1.double() @ w1.double() + dy2.double() @ w2.double())


@pytest.mark.parametrize("k", [64, 128])
def test_dgrad_gate_is_relu_backward(cuda, k):
    """A gated input gradient equals threshold_backward(dy1 W1 + dy2 W2, gate,
    0) bit for bit: zero where the gate is <= 0 (both zeros), NaN gates pass
    the gradient (torch's rule)."""
    rng = np.random.default_rng(k + 1)
    n, m = 1000 + 7, 41
    dy1, dy2 = _ints(rng, (n, m)).to(cuda), _ints(rng, (n, m)).to(cuda)
    w1, w2 = _ints(rng, (m, k), -2, 3).to(cuda), _ints(rng, (m, k), -2, 3).to(cuda)
    gbuf = _ints(rng, (n, k + 8), -2, 3).to(cuda)
    gbuf[::7, 5] = -0.0
    gbuf[::11, 9] = float("nan")
    gate = gbuf[:, :k]
    plain = L._node_dgrad2(k, dy1, w1, dy2, w2)
    gated, cs = L._node_dgrad2(k, dy1, w1, dy2, w2, gate=gate, colsum=True)
    ref = torch.ops.aten.threshold_backward(plain, gate, 0)
    assert torch.equal(gated, ref)
    # column sums as stored (integers: exact in any order)
    assert torch.equal(cs.double(), ref.double().sum(0))
    _, cs_plain = L._node_dgrad2(k, dy1, w1, dy2, w2, colsum=True)
    assert torch.equal(cs_plain.double(), plain.double().sum(0))
    # no rows: zero sums
    _, cs0 = L._node_dgrad2(k, dy1[:0], w1, dy2[:0], w2, colsum=True)
    assert torch.equal(cs0, torch.zeros(k, device=cuda))
    assert bool((gated[gate <= 0] == 0).all()) and bool((gated[gate > 0] == plain[gate > 0]).all())


@pytest.mark.parametrize("extra_consumer", [False, True])
def test_relu_mask_across_layers_equals_unfused(cuda, monkeypatch, extra_consumer):
    """Two sage_dense layers (128 -> 128 ReLU -> 41): the first layer's ReLU
    mask applied in the second layer's input-gradient store gives the same
    gradients, bit for bit, as the first layer's own threshold_backward pass
    (the first layer's bias gradient, summed by that store, within fp32
    summation tolerance); with a second consumer of the hidden rows the
    gradients are summed and the first layer masks and sums them itself."""
    import copy
    rng = np.random.default_rng(11)
    n, m = 60_000, 500_000
    g = dgl.DGLGraph((torch.from_numpy(rng.integers(0, n, m)),
                      torch.from_numpy(rng.integers(0, n, m))))

    def aggregate(x):
        g.ndata["x"] = x
        g.update_all(fn.copy_src("x", "m"), fn.mean("m", "a"))
        g.ndata.pop("x")
        return g.ndata.pop("a")

    torch.manual_seed(0)
    mods = [NodeLinear(128, 128), NodeLinear(128, 128, bias=False), NodeLinear(128, 41),
            NodeLinear(128, 41, bias=False)]
    mods = [mm.to(cuda) for mm in mods]
    x = torch.randn(n, 128, device=cuda)
    dy = torch.randn(n, 41, device=cuda)

    def run(ms):
        h = sage_dense(x, aggregate, ms[0], ms[1], torch.relu)
        out = sage_dense(h, aggregate, ms[2], ms[3])
        loss = (out * dy).sum()
        if extra_consumer:
            loss = loss + (h * h[:, :1]).sum()
        loss.backward()
        return [p.grad for mm in ms for p in mm.parameters()]

    calls = []
    orig = L._node_dgrad2

    def spy(*a, **kw):
        calls.append(kw.get("gate") is not None)
        return orig(*a, **kw)
    monkeypatch.setattr(L, "_node_dgrad2", spy)
    fused = run(mods)
    assert calls == [True]
    ref_mods = copy.deepcopy(mods)
    for p in (p for mm in ref_mods for p in mm.parameters()):
        p.grad = None
    monkeypatch.setattr(L, "_relu_producer", lambda t: None)
    calls.clear()
    plain = run(ref_mods)
    assert calls == [False]
    # every gradient bit for bit, except the first layer's bias: the fused
    # path sums its column as the input-gradient kernel stores it (another
    # association of the same 60,000 terms)
    bias1 = 1  # mods[0].parameters(): weight, bias
    for i, (a, b) in enumerate(zip(fused, plain)):
        if i == bias1 and not extra_consumer:
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * float(b.abs().max()))
        else:
            assert torch.equal(a, b)
