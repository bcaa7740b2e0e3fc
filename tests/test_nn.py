"""nn modules vs dense torch formulations of the same layer (CPU and GPU)."""
import numpy as np
import pytest
import torch

import dgl
from dgl import nn as dglnn

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def graph(device, n=60, m=400, seed=0):
    rng = np.random.default_rng(seed)
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    g = dgl.DGLGraph(multigraph=True)
    g.add_nodes(n)
    g.add_edges(src, dst)
    A = torch.zeros(n, n, dtype=torch.float64)
    A.index_put_((torch.as_tensor(dst), torch.as_tensor(src)),
                 torch.ones(m, dtype=torch.float64), accumulate=True)
    return g, A.to(device), torch.as_tensor(src).to(device), torch.as_tensor(dst).to(device)


def _dev(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device(device)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("fin,fout", [(8, 4), (4, 8)])
def test_graphconv(device, fin, fout):
    dev = _dev(device)
    g, A, _, _ = graph(dev)
    torch.manual_seed(0)
    conv = dglnn.GraphConv(fin, fout, norm="both", activation=torch.relu).to(dev)
    x = torch.randn(60, fin, device=dev)
    out = conv(g, x)
    dout = A.sum(0).clamp(min=1).pow(-0.5)  # out-degree of sources
    din = A.sum(1).clamp(min=1).pow(-0.5)
    ref = torch.relu((din[:, None] * (A @ (dout[:, None] * x.double())))
                     @ conv.weight.double() + conv.bias.double())
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_gatconv(device):
    dev = _dev(device)
    g, A, src, dst = graph(dev)
    torch.manual_seed(0)
    conv = dglnn.GATConv(8, 5, num_heads=3).to(dev)
    x = torch.randn(60, 8, device=dev)
    out = conv(g, x)
    ft = conv.fc(x).view(-1, 3, 5)
    el, er = (ft * conv.attn_l).sum(-1), (ft * conv.attn_r).sum(-1)
    e = torch.nn.functional.leaky_relu(el[src] + er[dst], 0.2).exp()  # E x H
    num = torch.zeros(60, 3, 5, device=dev).index_add(0, dst, e.unsqueeze(-1) * ft[src])
    den = torch.zeros(60, 3, device=dev).index_add(0, dst, e).clamp(min=1e-20)
    torch.testing.assert_close(out, num / den.unsqueeze(-1), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_sageconv(device):
    dev = _dev(device)
    g, A, _, _ = graph(dev)
    torch.manual_seed(0)
    for fin, fout in ((6, 4), (4, 6)):
        conv = dglnn.SAGEConv(fin, fout).to(dev)
        x = torch.randn(60, fin, device=dev)
        mean = (A @ x.double()) / A.sum(1, keepdim=True).clamp(min=1)
        ref = conv.fc_self(x).double() + mean @ conv.fc_neigh.weight.double().t()
        torch.testing.assert_close(conv(g, x).double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_relgraphconv(device):
    dev = _dev(device)
    g, A, src, dst = graph(dev)
    torch.manual_seed(0)
    conv = dglnn.RelGraphConv(8, 6, num_rels=4, num_bases=2).to(dev)
    x = torch.randn(60, 8, device=dev)
    et = torch.as_tensor(np.random.default_rng(1).integers(0, 4, 400)).to(dev)
    out = conv(g, x, et)
    W = conv.weight  # (R, nb, 4, 3)
    msg = torch.bmm(x[src].view(-1, 1, 4), W[et].reshape(-1, 4, 3)).view(400, 6)
    ref = torch.zeros(60, 6, device=dev).index_add(0, dst, msg) + x @ conv.loop_weight + conv.bias
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-5)


def test_node_linear_matches_linear():
    """NodeLinear == nn.Linear: same forward bits, gradients within fp32
    summation tolerance (split-K weight gradient, chunked bias gradient), on a
    row count that exercises several chunks plus a remainder."""
    import torch.nn as nn
    from dgl.nn.pytorch import NodeLinear
    from dgl.nn.pytorch import linear as L
    old = L._ROWS_PER_CHUNK
    L._ROWS_PER_CHUNK = 1000
    try:
        torch.manual_seed(0)
        ref = nn.Linear(24, 10)
        mine = NodeLinear(24, 10)
        mine.load_state_dict(ref.state_dict())
        x = torch.randn(5321, 24)
        g = torch.randn(5321, 10)
        xa = x.clone().requires_grad_(True)
        xb = x.clone().requires_grad_(True)
        ya, yb = ref(xa), mine(xb)
        assert torch.equal(ya, yb)
        ya.backward(g)
        yb.backward(g)
        torch.testing.assert_close(xb.grad, xa.grad, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(mine.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(mine.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-3)
        nb = NodeLinear(24, 10, bias=False)
        nb(x.requires_grad_(True)).sum().backward()
        assert nb.bias is None
    finally:
        L._ROWS_PER_CHUNK = old


@pytest.mark.parametrize("dims", [(24, 10), (10, 24), (16, 16)])
def test_sage_dense_matches_unfused(dims):
    """sage_dense (one GEMM + one accumulating GEMM per direction; the
    narrower side aggregated, its transpose taken inside the fused backward)
    equals fc_self(h) + fc_neigh(mean(h)) and its gradients within fp32
    summation tolerance, for a narrowing, a widening and a square layer."""
    import copy
    import dgl.function as fn
    from dgl.nn.pytorch import NodeLinear, sage_dense
    from dgl.nn.pytorch import linear as L
    fin, fout = dims
    rng = np.random.default_rng(fin * 100 + fout)
    n, m = 3000, 20000
    g = dgl.DGLGraph((torch.from_numpy(rng.integers(0, n, m)),
                      torch.from_numpy(rng.integers(0, n, m))))

    def aggregate(x):
        g.ndata["x"] = x
        g.update_all(fn.copy_src("x", "m"), fn.mean("m", "a"))
        g.ndata.pop("x")
        return g.ndata.pop("a")

    old = L._ROWS_PER_CHUNK
    L._ROWS_PER_CHUNK = 500
    try:
        torch.manual_seed(1)
        fs, fnb = NodeLinear(fin, fout), NodeLinear(fin, fout, bias=False)
        rs, rnb = copy.deepcopy(fs), copy.deepcopy(fnb)
        x = torch.randn(n, fin)
        dy = torch.randn(n, fout)
        xa = x.clone().requires_grad_(True)
        ref = rs(xa) + rnb(aggregate(xa))
        ref.backward(dy)
        xb = x.clone().requires_grad_(True)
        out = sage_dense(xb, aggregate, fs, fnb)
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
        out.backward(dy)
        torch.testing.assert_close(xb.grad, xa.grad, rtol=1e-4, atol=1e-4)
        for a, b in ((fs.weight, rs.weight), (fs.bias, rs.bias), (fnb.weight, rnb.weight)):
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-4, atol=1e-3)
        # a ReLU fused into the step (widening / square) or applied after it
        for p in (fs.weight, fs.bias, fnb.weight, rs.weight, rs.bias, rnb.weight):
            p.grad = None
        xc = x.clone().requires_grad_(True)
        xd = x.clone().requires_grad_(True)
        o1 = sage_dense(xc, aggregate, fs, fnb, torch.nn.functional.relu)
        o2 = torch.relu(rs(xd) + rnb(aggregate(xd)))
        torch.testing.assert_close(o1, o2, rtol=1e-5, atol=1e-5)
        o1.backward(dy)
        o2.backward(dy)
        torch.testing.assert_close(xc.grad, xd.grad, rtol=1e-4, atol=1e-4)
        for a, b in ((fs.weight, rs.weight), (fs.bias, rs.bias), (fnb.weight, rnb.weight)):
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-4, atol=1e-3)
        with torch.no_grad():  # inference path (no graph kept)
            torch.testing.assert_close(sage_dense(x, aggregate, fs, fnb), ref.detach(),
                                       rtol=1e-5, atol=1e-5)
    finally:
        L._ROWS_PER_CHUNK = old


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("n,k,m", [(232965, 41, 24), (20000, 64, 41), (3000, 16, 8), (100, 8, 4)])
def test_dense_mm_splitk_weight_gradient(device, n, k, m):
    """nn.pytorch.dense_mm: torch.mm's value; its weight gradient xᵀ·dy
    summed over 2K-row chunks (the split-K product) within 1e-5 of float64
    per element, relative to Σ|x·dy| (the chunking only reassociates)."""
    from dgl.nn.pytorch import dense_mm
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    gen = torch.Generator().manual_seed(n + k)
    x = torch.randn(n, k, generator=gen).to(device).requires_grad_(True)
    w = torch.randn(k, m, generator=gen).to(device).requires_grad_(True)
    dy = torch.randn(n, m, generator=gen).to(device)
    y = dense_mm(x, w)
    assert torch.equal(y.detach(), torch.mm(x.detach(), w.detach()))
    y.backward(dy)
    x64, dy64 = x.detach().double().cpu(), dy.double().cpu()
    want = x64.t() @ dy64
    bound = x64.abs().t() @ dy64.abs()
    err = (w.grad.double().cpu() - want).abs()
    assert bool((err <= 1e-5 * bound + 1e-30).all()), float((err / (bound + 1e-30)).max())
    wdx = dy64 @ w.detach().double().cpu().t()
    assert torch.allclose(x.grad.double().cpu(), wdx, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("F", [128, 41, 300])
@pytest.mark.parametrize("relu", [True, False])
def test_node_epilogue_bits_of_torch(F, relu):
    """nn.pytorch.node_epilogue on the device (one kernel each way) against
    torch's `x * norm`, `+ bias`, `relu` on the same device: the output and
    the input gradient bit for bit (zeros, -0.0, NaN and rows of scale 0
    included), the bias gradient within 1e-5 of Σ|d_pre|."""
    from dgl.nn.pytorch import node_epilogue
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda", 0)
    gen = torch.Generator().manual_seed(F)
    n = 5000
    x = torch.randn(n, F, generator=gen)
    x[0, :4] = torch.tensor([0.0, -0.0, float("nan"), 1e-30])
    norm = torch.rand(n, 1, generator=gen)
    norm[7] = 0.0
    bias = torch.randn(F, generator=gen)
    dout = torch.randn(n, F, generator=gen)
    act = torch.nn.functional.relu if relu else None
    res = []
    for fused in (True, False):
        x1 = x.to(dev).requires_grad_(True)
        b1 = bias.to(dev).requires_grad_(True)
        nd = norm.to(dev)
        if fused:
            out = node_epilogue(x1, nd, b1, act)
        else:
            out = x1 * nd + b1
            out = act(out) if act else out
        out.backward(dout.to(dev))
        res.append((out.detach().cpu(), x1.grad.cpu(), b1.grad.cpu()))
    (o1, g1, b1g), (o2, g2, b2g) = res
    assert torch.equal(o1.nan_to_num(7.0), o2.nan_to_num(7.0))
    assert torch.equal(torch.signbit(o1), torch.signbit(o2))
    assert torch.equal(g1.nan_to_num(7.0), g2.nan_to_num(7.0))
    d_pre = torch.where(o2 > 0, dout, torch.zeros(())) if relu else dout
    bound = d_pre.double().abs().sum(0)
    assert bool(((b1g.double() - b2g.double()).abs() <= 1e-5 * bound + 1e-30).all())
