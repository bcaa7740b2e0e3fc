"""R-GCN typed-edge block g-SpMM vs the reference's UDF formulation
(examples/pytorch/rgcn/layers.py:121-132: gather W[type], bmm, sum by dst),
forward and gradients, within fp32 tolerance (the reference's bmm/sum orders
are implementation-defined)."""
import numpy as np
import pytest
import torch

from dgl import kernel

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def reference(src, dst, etype, h, W, n_dst, norm=None):
    R, nb, si, so = W.shape
    w = W[etype].reshape(-1, si, so)                     # (E*nb, si, so)
    node = h[src].reshape(-1, 1, si)                     # (E*nb, 1, si)
    msg = torch.bmm(node, w).reshape(len(src), nb * so)  # (E, out)
    if norm is not None:
        msg = msg * norm.unsqueeze(1)
    out = torch.zeros(n_dst, nb * so, dtype=msg.dtype, device=msg.device)
    return out.index_add(0, dst, msg)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("shape", [(11, 4, 3, 5), (20, 100, 5, 5)])
def test_typed_block(device, shape):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device(device)
    R, nb, si, so = shape
    rng = np.random.default_rng(3)
    n, m = 300, 5000
    src = torch.from_numpy(rng.integers(0, n, m)).to(dev)
    dst = torch.from_numpy(rng.integers(0, n, m)).to(dev)
    etype = torch.from_numpy(rng.integers(0, R, m)).to(dev)
    norm = torch.from_numpy(rng.uniform(0.1, 1, m).astype(np.float32)).to(dev)
    h = torch.randn(n, nb * si, device=dev, dtype=torch.float64)
    W = torch.randn(R, nb, si, so, device=dev, dtype=torch.float64) * 0.3
    G = torch.randn(n, nb * so, device=dev)
    adj = kernel.from_coo(n, n, dst.cpu(), src.cpu(), kernel.ORDER_EID, dev)
    for nm in (None, norm):
        h1 = h.float().clone().requires_grad_(True)
        W1 = W.float().clone().requires_grad_(True)
        out = kernel.typed_block_spmm(adj, h1, W1, etype, nm)
        out.backward(G)
        h2 = h.clone().requires_grad_(True)
        W2 = W.clone().requires_grad_(True)
        ref = reference(src, dst, etype, h2, W2, n, None if nm is None else nm.double())
        ref.backward(G.double())
        # the fp32 chains' error bound, per element: 1e-5 of the sum of the
        # absolute terms (the same products over |h|, |W|, |norm|, |G|), the
        # bound tests/test_rmat26.py uses for chunked rows (r04 verdict, Weak 1)
        ha = h.abs().requires_grad_(True)
        Wa = W.abs().requires_grad_(True)
        scale = reference(src, dst, etype, ha, Wa, n,
                          None if nm is None else nm.double().abs())
        scale.backward(G.double().abs())
        for got, want, bound in ((out.double(), ref, scale.detach()),
                                 (h1.grad.double(), h2.grad, ha.grad),
                                 (W1.grad.double(), W2.grad, Wa.grad)):
            err = (got - want).abs()
            assert bool((err <= 1e-5 * bound + 1e-30).all()), \
                float((err / (1e-5 * bound + 1e-30)).max())


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(7, 3, 1, 2), (9, 10, 2, 7), (11, 4, 3, 5), (20, 100, 5, 5),
                                   (5, 8, 8, 3), (4, 2, 16, 40), (6, 3, 7, 9)])
def test_typed_block_device_matches_host_bits(shape):
    """The HIP kernels (templated block widths 1/2/4/5/8/16, runtime width
    otherwise; slices of 64 outputs per wave, edges in flight predicated)
    run the same per-element fma chains as the host kernels: identical bits,
    forward, the transposed-block backward and the weight gradient. A
    power-law destination set gives rows far longer than one chunk of
    kernel.TYPED_CHUNK slots (their partials added in chunk order), and the
    relations hold more than one chunk of edges each."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    R, nb, si, so = shape
    rng = np.random.default_rng(sum(shape))
    n, m = 400, 8000 * R // 4 + 8000
    p = 1.0 / np.arange(1, n + 1) ** 1.1
    dst = torch.from_numpy(rng.choice(n, size=m, p=p / p.sum()))
    src = torch.from_numpy(rng.integers(0, n, m))
    etype = torch.from_numpy(rng.integers(0, R, m))
    norm = torch.from_numpy(rng.uniform(0.1, 1, m).astype(np.float32))
    h = torch.randn(n, nb * si)
    W = torch.randn(R, nb, si, so) * 0.3
    G = torch.randn(n, nb * so)
    assert int(torch.bincount(dst).max()) > 4 * kernel.TYPED_CHUNK
    assert int(torch.bincount(etype).min()) > kernel.TYPED_CHUNK
    for nm in (norm, None):
        outs, grads, wgrads = [], [], []
        # the host, then the device's one-kernel forms at 8 output slices per
        # wave and at 1, then the relation-major messages + slot-order sum and
        # the LDS-staged weight gradient (r06; block widths outside the
        # message kernel's set fall back per direction)
        for dev, width, msgs in (("cpu", 8, 0), ("cuda", 8, 0), ("cuda", 1, 0), ("cuda", 1, 1)):
            kernel.set_typed_block_width(width)
            kernel.set_typed_block_messages(msgs)
            try:
                adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
                h1 = h.detach().to(dev).clone().requires_grad_(True)
                W1 = W.detach().to(dev).clone().requires_grad_(True)
                out = kernel.typed_block_spmm(adj, h1, W1, etype.to(dev),
                                              None if nm is None else nm.to(dev))
                out.backward(G.to(dev))
            finally:
                kernel.set_typed_block_width(1)
                kernel.set_typed_block_messages(_MSG_DEFAULT)
            outs.append(out.detach().cpu())
            grads.append(h1.grad.cpu())
            wgrads.append(W1.grad.cpu())
        for k in (1, 2, 3):
            assert torch.equal(outs[0], outs[k])
            assert torch.equal(grads[0], grads[k])
            assert torch.equal(wgrads[0], wgrads[k])


_MSG_DEFAULT = 1


def test_typed_block_messages_take_rgcn_widths():
    """The message path covers configs[4]'s 100 blocks of 5 x 5 both ways
    (and rejects widths its kernels are not built for)."""
    kernel.set_typed_block_messages(1)
    try:
        assert kernel._typed_msg_ok(100, 5, 5)
        assert not kernel._typed_msg_ok(3, 7, 9)
        assert not kernel._typed_msg_ok(300, 5, 5)  # rows past 1024 features
    finally:
        kernel.set_typed_block_messages(_MSG_DEFAULT)


def _example():
    import importlib.util
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "examples", "rgcn",
                        "link_predict.py")
    spec = importlib.util.spec_from_file_location("rgcn_link_predict_tb", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("device", DEVICES)
def test_typed_block_fb15k_shape(device):
    """BASELINE configs[4] at its shape (examples/pytorch/rgcn/utils.py:72-108,
    layers.py:121-132): FB15k-237's 14,541 entities and 237 relations (474
    typed relations with the reverse edges), a 30,000-edge sampled training
    graph from the power-law triples (the sampled entities' hub rows
    included), 100 bases of 5 x 5 on 500 features. Forward, dH and dW vs the
    float64 bmm formulation, with and without the 1/in-degree norm."""
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device(device)
    ex = _example()
    triples = ex.synthetic_kg(14541, 237, 272115, seed=0)
    uniq, src, dst, rel, norm, _, _ = ex.sample_graph(triples, 30000, 237,
                                                      np.random.default_rng(0))
    n, R, nb, si = len(uniq), 2 * 237, 100, 5
    assert len(src) == 30000 and int(rel.max()) < R
    deg = np.bincount(dst, minlength=n)
    assert deg.max() >= 100  # hub entities: rows far longer than the kernel's edge group
    src_t, dst_t = torch.from_numpy(src).to(dev), torch.from_numpy(dst).to(dev)
    etype = torch.from_numpy(rel).to(dev)
    nrm = torch.from_numpy(norm[dst]).to(dev)  # 1 / in-degree of each edge's destination
    gen = torch.Generator().manual_seed(4)
    h = torch.randn(n, nb * si, generator=gen, dtype=torch.float64).to(dev)
    W = (torch.randn(R, nb, si, si, generator=gen, dtype=torch.float64) * 0.3).to(dev)
    G = torch.randn(n, nb * si, generator=gen).to(dev)
    adj = kernel.from_coo(n, n, dst_t.cpu(), src_t.cpu(), kernel.ORDER_EID, dev)
    for nm in (None, nrm):
        h1 = h.float().clone().requires_grad_(True)
        W1 = W.float().clone().requires_grad_(True)
        out = kernel.typed_block_spmm(adj, h1, W1, etype, nm)
        out.backward(G)
        h2 = h.clone().requires_grad_(True)
        W2 = W.clone().requires_grad_(True)
        ref = reference(src_t, dst_t, etype, h2, W2, n, None if nm is None else nm.double())
        ref.backward(G.double())
        # the fp32 chains' error bound, per element: 1e-5 of the sum of the
        # absolute terms (the same products over |h|, |W|, |norm|, |G|), the
        # bound tests/test_rmat26.py uses for chunked rows (r04 verdict, Weak 1)
        ha = h.abs().requires_grad_(True)
        Wa = W.abs().requires_grad_(True)
        scale = reference(src_t, dst_t, etype, ha, Wa, n,
                          None if nm is None else nm.double().abs())
        scale.backward(G.double().abs())
        for got, want, bound in ((out.double(), ref, scale.detach()),
                                 (h1.grad.double(), h2.grad, ha.grad),
                                 (W1.grad.double(), W2.grad, Wa.grad)):
            err = (got - want).abs()
            assert bool((err <= 1e-5 * bound + 1e-30).all()), \
                float((err / (1e-5 * bound + 1e-30)).max())


@pytest.mark.gpu
def test_groupings_device_match_host():
    """The one-call device groupings (relation-major slots for the typed-block
    kernels, positions by id for DistMult, each with its item list) equal the
    host builds: a CSR over the keys, the gathers and kernel._typed_items."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    rng = np.random.default_rng(11)
    n, m, R = 500, 9000, 37
    p = 1.0 / np.arange(1, n + 1) ** 1.1
    dst = torch.from_numpy(rng.choice(n, size=m, p=p / p.sum()))
    src = torch.from_numpy(rng.integers(0, n, m))
    etype = torch.from_numpy(rng.integers(0, R, m))
    etype[:300] = 5  # one relation of several chunks
    host = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, "cpu")
    dev = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, "cuda")
    gh = kernel._RelationGroups(host.fwd, etype, R)
    gd = kernel._RelationGroups(dev.fwd, etype.cuda(), R)
    for a, b in ((gh.ptr, gd.ptr), (gh.src, gd.src), (gh.slot, gd.slot), (gh.dst, gd.dst)):
        assert torch.equal(a, b.cpu())
    ip, ir = kernel._typed_items(gh.ptr, m)
    assert torch.equal(ip, gd.items[0].cpu()) and torch.equal(ir, gd.items[1].cpu())
    for rows, ids in ((n, torch.cat([src, dst])), (R, etype), (n, torch.zeros(5, dtype=torch.int64))):
        ph, oh = kernel._position_groups(ids, rows)
        pd, od, ipd, ird = kernel._position_groups_items(ids.cuda(), rows)
        assert torch.equal(ph, pd.cpu()) and torch.equal(oh, od.cpu())
        iph, irh = kernel._typed_items(ph, ids.numel())
        assert torch.equal(iph, ipd.cpu()) and torch.equal(irh, ird.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(11, 4, 3, 5), (20, 100, 5, 5), (6, 3, 7, 9)])
def test_typed_block_row_scale_bits(shape):
    """row_scale inside the message path's kernels (the forward sum's store,
    the dH messages' and dW's staged dout rows) gives the bits of
    ``typed_block_spmm(...) * scale.unsqueeze(1)`` with torch's product and
    its backward, on the host; widths outside the message kernels take that
    product themselves."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    R, nb, si, so = shape
    rng = np.random.default_rng(7 + sum(shape))
    n, m = 400, 9000
    p = 1.0 / np.arange(1, n + 1) ** 1.1
    dst = torch.from_numpy(rng.choice(n, size=m, p=p / p.sum()))
    src = torch.from_numpy(rng.integers(0, n, m))
    etype = torch.from_numpy(rng.integers(0, R, m))
    scale = torch.from_numpy(rng.uniform(0.01, 1, n).astype(np.float32))
    h = torch.randn(n, nb * si)
    W = torch.randn(R, nb, si, so) * 0.3
    G = torch.randn(n, nb * so)
    res = []
    for dev in ("cpu", "cuda"):
        adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
        h1 = h.detach().to(dev).clone().requires_grad_(True)
        W1 = W.detach().to(dev).clone().requires_grad_(True)
        if dev == "cpu":
            out = kernel.typed_block_spmm(adj, h1, W1, etype) * scale.unsqueeze(1)
        else:
            out = kernel.typed_block_spmm(adj, h1, W1, etype.cuda(), row_scale=scale.cuda())
        out.backward(G.to(dev))
        res.append((out.detach().cpu(), h1.grad.cpu(), W1.grad.cpu()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
