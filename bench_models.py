"""bench.py's model legs (BASELINE.json configs[2]-[4] at N = 1): each a
training step of one §8(f) model through the engine, timed like the headline
(warm-up, then K steps between two synchronises), with

* ``kernel_ms``: the library's own launches per step (hipEvent pairs around
  every g-SpMM / g-SDDMM / GAT / typed-block launch on its stream);
* ``roofline``: the step's dominant engine kernel alone (its algorithmic
  bytes per call over its mean duration, events on the launch stream)
  against the ceiling of its regime (bench.gather_peak);
* ``cpu_baseline``: the reference's formulation of the same step on the host
  cores (this engine's host path, kind "port", core count stated), on the
  same model or a bounded sample of the same graph.

The reference times these loops itself: gat/train.py:216-235 (epoch),
rgcn/link_predict.py:163-174 (forward + backward + Adam), and (the mean
reducer as a UDF: the reference has no builtin mean) degree_bucketing.py.
"""
from __future__ import absolute_import

import contextlib
import gc
import importlib.util
import os
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))

_EXAMPLES = {}


def example(relpath):
    """An example script imported by path (once)."""
    if relpath not in _EXAMPLES:
        name = "bench_ex_" + relpath.replace("/", "_").replace(".py", "")
        spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "examples",
                                                                         relpath))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _EXAMPLES[relpath] = mod
    return _EXAMPLES[relpath]


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


@contextlib.contextmanager
def _no_gc():
    """Setup garbage collected first, no collection inside the timed region
    (bench.timed_steps does the same)."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def wall_steps(step, steps, warmup, dev, kernel):
    """(wall ms per step, library kernel ms per step) over ``steps`` steps
    after ``warmup``; kernel ms from the library's per-launch events, taken
    over ``steps`` further steps: the event pairs and their lock cost host
    time on every launch (≈0.5 ms of an R-GCN step, r06), so the wall-clock
    steps run without them."""
    for _ in range(warmup):
        step()
    _sync(dev)
    with _no_gc():
        _marker(dev)  # tools/window_stats.py: this region's kernels
        _sync(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        _sync(dev)
        el = time.perf_counter() - t0
        _marker(dev)
        kernel.timing_enable(True)
        try:
            for _ in range(steps):
                step()
            _sync(dev)
            kms, launches = kernel.timing_read()
        finally:
            kernel.timing_enable(False)
    return el / steps * 1e3, kms / steps, launches // max(steps, 1)


def _marker(dev):
    """A one-wave spin kernel outside the timed region (bench._window_marker)."""
    if dev.type == "cuda":
        torch.cuda._sleep(1)


def call_ms(fn, iters, dev):
    """Mean GPU span of ``fn`` (events on the current stream, which the
    library launches on), after one untimed call."""
    fn()
    _sync(dev)
    if dev.type != "cuda":  # host kernels: wall time
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        return (time.perf_counter() - t0) / iters * 1e3
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with _no_gc():
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
    return s.elapsed_time(e) / iters


def _threads():
    return torch.get_num_threads()


def roof(bytes_, ms, peak, source, kernel_name, **extra):
    ach = bytes_ / (ms * 1e-3) / 1e9 if ms > 0 else None
    r = {"bound": "hbm", "achieved": ach, "peak": peak, "unit": "GB/s",
         "frac": None if ach is None else ach / peak, "kernel": kernel_name,
         "kernel_ms": ms, "bytes_per_call": bytes_, "peak_source": source}
    r.update(extra)
    return r


# -- GCN on the Reddit-shaped graph (configs[1]) -------------------------------
GCN_IN, GCN_HIDDEN, GCN_CLASSES = 602, 128, 41


def gcn_reddit_data(n, dev, seed=7):
    """configs[1]'s synthetic node data at the graph's size: 602-wide
    features (Reddit's embedding width), 41 classes, 66 % training nodes."""
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    feats = 0.1 * torch.randn(n, GCN_IN, generator=gen, device=dev)
    labels = torch.randint(0, GCN_CLASSES, (n,), generator=gen, device=dev)
    mask = (torch.rand(n, generator=gen, device=dev) < 0.66).nonzero(as_tuple=True)[0]
    return feats, labels, mask


def gcn_norm(g, dev):
    """gcn_spmv.py:138-143: in-degree^-1/2 (self-loops already in the graph)."""
    norm = torch.pow(g.in_degrees().float(), -0.5)
    norm[torch.isinf(norm)] = 0
    return norm.unsqueeze(1).to(dev)


def gcn_reddit_leg(g, dev, kernel, gather_peak, algorithmic_bytes, sample, epochs=10, warmup=3,
                   cpu=True, dropout=0.5):
    """configs[1]: the example's 2-layer GCN (602 -> 128 -> 41, dropout 0.5 ahead
    of the second layer, Adam; examples/gcn/gcn_spmv.py, the reference's
    examples/pytorch/gcn/gcn_spmv.py:45-62,136-143,168-182) for full-graph
    epochs on the headline graph (self-loops included): forward, cross-entropy
    over the training nodes, backward, Adam. Eager, and one replayed HIP graph
    per epoch (the example's --hip-graph)."""
    from dgl.nn.pytorch import weighted_cross_entropy
    gcn = example("gcn/gcn_spmv.py")
    n, E = g.number_of_nodes(), g.number_of_edges()
    feats, labels, mask = gcn_reddit_data(n, dev)
    # the mean cross-entropy over the training nodes as the library's fused
    # node-row loss with 0/1 row weights (as the sage leg): torch's NLL over
    # the gathered rows took 0.37 ms of the epoch
    train_w = torch.zeros(n, device=dev)
    train_w[mask] = 1.0
    inv_ntrain = 1.0 / float(mask.numel())

    def loss_of(logits):
        return weighted_cross_entropy(logits, labels, train_w) * inv_ntrain
    saved = {k: g.ndata[k] for k in ("h",) if k in g.ndata}
    g.ndata["norm"] = gcn_norm(g, dev)
    try:
        def build(capturable=False):
            torch.manual_seed(0)
            m = gcn.GCN(g, GCN_IN, GCN_HIDDEN, GCN_CLASSES, 1, F.relu, dropout).to(dev)
            return m, torch.optim.Adam(m.parameters(), lr=1e-2, weight_decay=5e-4,
                                       capturable=capturable, fused=True)
        model, opt = build()
        model.train()

        def epoch():
            loss = loss_of(model(feats))
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
        ms, kms, launches = wall_steps(epoch, epochs, warmup, dev, kernel)
        # the same epoch captured once and replayed
        gmodel, gopt = build(capturable=True)
        gmodel.train()

        def gepoch():
            gopt.zero_grad(set_to_none=True)
            loss_of(gmodel(feats)).backward()
            gopt.step()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                gepoch()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        gopt.zero_grad(set_to_none=True)
        with torch.cuda.graph(graph, stream=side):
            gepoch()
        gms = call_ms(graph.replay, epochs, dev)
        del graph, gmodel, gopt
        # the aggregations alone: layer 1 (F = 128, the headline product) and
        # layer 2 (F = 41, rows padded to 48 floats by the plan)
        adj = g.sparse_adjacency(dev)
        h128 = torch.rand(n, GCN_HIDDEN, device=dev)
        h41 = torch.rand(n, GCN_CLASSES, device=dev)
        a128 = call_ms(lambda: kernel.gspmm(adj, "copy_u", "sum", h128), epochs, dev)
        a41 = call_ms(lambda: kernel.gspmm(adj, "copy_u", "sum", h41), epochs, dev)
        blocks = kernel.blocked_schedule(adj, h128)
        peak, src_ = gather_peak(n * GCN_HIDDEN * 4, blocks)
        del h128, h41
    finally:
        g.ndata.pop("norm", None)
        for k in ("h",):
            g.ndata.pop(k, None)
        g.ndata.update(saved)
    res = {"value": E / (gms * 1e-3), "unit": "edges/s per epoch (HIP graph)",
           "ms_per_epoch": ms, "ms_per_epoch_hip_graph": gms, "kernel_ms": kms,
           "launches_per_epoch": launches, "epochs": epochs, "warmup": warmup,
           "aggregation_ms": {"layer1_f128": a128, "layer2_f41": a41},
           "config": "configs[1]: 2-layer GCN %d-%d-%d (examples/gcn/gcn_spmv.py: dense Linear, "
                     "norm, update_all(copy_src, sum), norm, bias, ReLU; dropout %.1f ahead of "
                     "layer 2), full graph = the headline graph (%d nodes, %d edges incl. "
                     "self-loops), random features, 41 classes, 66 %% training nodes, "
                     "mean cross-entropy over them (the library's fused node-row loss, 0/1 "
                     "row weights) + backward + Adam per epoch; bias gradients as chunked "
                     "column sums (nn.bias_add); eager and one replayed HIP graph"
                     % (GCN_IN, GCN_HIDDEN, GCN_CLASSES, dropout, n, E),
           "roofline": roof(algorithmic_bytes(E, n, GCN_HIDDEN), a128, peak, src_,
                            "layer 1's aggregation: g-SpMM copy_u + sum, F = 128 (%d launches "
                            "per call); per epoch 4 aggregations run (F = 128 and 41, forward "
                            "and transposed)" % max(blocks, 1)),
           "cpu_baseline": None}
    if cpu and sample is not None:
        res["cpu_baseline"] = gcn_reddit_cpu(sample, n, dropout)
    return res


def gcn_reddit_cpu(sample, n, dropout, target_edges=2_000_000, epochs=2):
    """The reference's epoch on the host: gcn_spmv.py:45-62,168-182 with its
    backend's products (torch.sparse.mm on the uncoalesced COO adjacency,
    python/dgl/backend/pytorch/tensor.py:45-51,145-146) written out in torch,
    over the in-edges of the first rows of the headline's CPU sample (about
    ``target_edges``, sources over all ``n`` nodes; every node keeps its
    Linear and its loss term)."""
    rows, d, s = sample
    cum = torch.cumsum(torch.bincount(d, minlength=rows), 0)
    r1 = min(int(torch.searchsorted(cum, torch.tensor(target_edges))) + 1, rows)
    sel = d < r1
    d, s = d[sel], s[sel]
    e = int(s.numel())
    A = torch.sparse_coo_tensor(torch.stack([d, s]), torch.ones(e), (n, n))
    deg = torch.bincount(d, minlength=n).float()
    norm = torch.pow(deg, -0.5)
    norm[torch.isinf(norm)] = 0
    norm = norm.unsqueeze(1)
    feats, labels, mask = gcn_reddit_data(n, torch.device("cpu"))
    torch.manual_seed(0)
    w1 = torch.nn.Parameter(torch.empty(GCN_IN, GCN_HIDDEN).uniform_(-0.088, 0.088))
    b1 = torch.nn.Parameter(torch.zeros(GCN_HIDDEN))
    w2 = torch.nn.Parameter(torch.empty(GCN_HIDDEN, GCN_CLASSES).uniform_(-0.156, 0.156))
    b2 = torch.nn.Parameter(torch.zeros(GCN_CLASSES))
    opt = torch.optim.Adam([w1, b1, w2, b2], lr=1e-2, weight_decay=5e-4)

    def layer(h, w, b, act, p):
        if p:
            h = F.dropout(h, p)
        h = torch.mm(h, w) * norm
        h = torch.sparse.mm(A, h) * norm + b
        return F.relu(h) if act else h

    def once():
        logits = layer(layer(feats, w1, b1, True, 0.0), w2, b2, False, dropout)
        loss = F.cross_entropy(logits[mask], labels[mask])
        opt.zero_grad()
        loss.backward()
        opt.step()
    once()
    t = 0.0
    for _ in range(epochs):
        t0 = time.perf_counter()
        once()
        t += time.perf_counter() - t0
    ms = t / epochs * 1e3
    return {"value": e / (ms * 1e-3), "unit": "edges/s per epoch", "ms_per_epoch": ms,
            "cores": _threads(), "kind": "reference",
            "sample": "the reference's GCN epoch (gcn_spmv.py:45-62,168-182: torch.mm, norm, "
                      "torch.sparse.mm on the uncoalesced COO adjacency, norm, bias, ReLU; "
                      "dropout %.1f; cross-entropy, backward, Adam) on the in-edges of the first "
                      "%d rows of the headline graph (%d edges, sources over all %d nodes; the "
                      "dense layers over all %d nodes), %d epochs after one warm-up, torch %d "
                      "threads" % (dropout, r1, e, n, n, epochs, _threads())}


# -- GAT layer on the Reddit-shaped graph: 8 heads x 16 ------------------------
def gat_fwd_bytes(E, n, H, D, stored, logits_read=True):
    """Fused GAT forward (kernel.gat_aggregate): per edge the gathered feature
    row, its column id, the source's H logits (unless recomputed from the
    row: ``logits_read`` False) and (training) the H stored attention values;
    per row the output row, its H normalisers, H logits and its indptr
    entry."""
    F_ = H * D
    return (E * (4 * F_ + 4 + (4 * H if logits_read else 0) + (4 * H if stored else 0)) +
            n * (4 * F_ + 8 * H + 8))


def gat_layer_leg(g, dev, kernel, gather_peak, sample, steps=10, warmup=3, H=8, D=16,
                  cpu=True):
    """One GAT layer's aggregation, forward + backward, on the bench graph
    (attention, its per-head weighted sum and the copy_edge normaliser: the
    message passing of gat/train.py:61-96) with random features."""
    adj = g.sparse_adjacency(dev)
    n, E = g.number_of_nodes(), g.number_of_edges()
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    ft = (torch.rand(n, H, D, generator=gen, device=dev) * 2 - 1).requires_grad_(True)
    el = (torch.rand(n, H, generator=gen, device=dev) - 0.5).requires_grad_(True)
    er = (torch.rand(n, H, generator=gen, device=dev) - 0.5).requires_grad_(True)
    gout = torch.rand(n, H, D, generator=gen, device=dev)
    gz = torch.rand(n, H, 1, generator=gen, device=dev)

    def step():
        fs, z = kernel.gat_aggregate(adj, ft, el, er)
        torch.autograd.backward([fs, z], [gout, gz])
        ft.grad = el.grad = er.grad = None
    ms, kms, launches = wall_steps(step, steps, warmup, dev, kernel)

    def fwd():
        kernel.gat_aggregate(adj, ft, el, er)  # training forward
    fms = call_ms(fwd, steps, dev)
    # study: the forward with el from gat_logits(ft, attn_l, attn_r) and the
    # sources' logits recomputed from their gathered rows (off by default:
    # slower)
    al = ((torch.rand(H, D, 1, generator=gen, device=dev) - 0.5) * 0.25).requires_grad_(True)
    ar = ((torch.rand(H, D, 1, generator=gen, device=dev) - 0.5) * 0.25).requires_grad_(True)
    el_t, er_t = kernel.gat_logits(ft, al, ar)
    kernel.check_call(kernel.LIB.dglhip_set_gat_logit_recompute(1))
    try:
        fms_recomputed = call_ms(lambda: kernel.gat_aggregate(adj, ft, el_t, er_t), steps, dev)
    finally:
        kernel.check_call(kernel.LIB.dglhip_set_gat_logit_recompute(0))
    del el_t, er_t
    # the one-pass transposed backward recomputes the attention: nothing stored
    stored = kernel.LIB.dglhip_gat_backward_t_ok(H, D) != 1
    # the forward's row ranges as gat_aggregate cuts them (nothing stored:
    # _GAT_BLOCK_BYTES_NOGRAD), the backward's plan over the transpose
    cuts = kernel._block_cuts(adj.fwd, (H * D + H) * 4,
                              None if stored else kernel._GAT_BLOCK_BYTES_NOGRAD)
    peak, src = gather_peak(n * H * D * 4, 0 if cuts is None else len(cuts) - 1)
    bplan = kernel._block_plan(adj.bwd, gout.view(n, H * D), H * D,
                               kernel._GAT_BWD_BLOCK_BYTES)
    bpeak, bsrc = gather_peak(n * H * D * 4, 0 if bplan is None else len(bplan))
    res = {"value": E / (ms * 1e-3), "unit": "edges/s (fwd+bwd)", "ms_per_step": ms,
           "kernel_ms": kms, "launches_per_step": launches, "steps": steps, "warmup": warmup,
           "config": "GAT layer aggregation, %d heads x %d, on the headline graph (%d nodes, "
                     "%d edges): kernel.gat_aggregate forward + backward, dropout 0"
                     % (H, D, n, E),
           "forward_ms_logits_recomputed": fms_recomputed,
           "roofline": roof(gat_fwd_bytes(E, n, H, D, stored), fms, peak, src,
                            "fused GAT forward (dglhip_gat_aggregate_device%s)"
                            % (", attention stored for the backward" if stored else
                               "; the backward recomputes the attention")),
           "cpu_baseline": None}
    if not stored:
        # the backward's kernels (the transposed pass and d_er's row sums): the
        # step's library launches less the forward's
        bms = max(kms - fms, 1e-6)
        F_ = H * D
        bbytes = (E * (4 * F_ + 12 + 12 * H) + n * (8 * F_ + 8 * H + 8) +
                  E * 4 * H + n * 4 * H)
        res["roofline_backward"] = roof(
            bbytes, bms, bpeak, bsrc,
            "GAT backward: dglhip_gat_backward_t_device (per edge the gathered dout row, "
            "column id, forward slot, er and dz values, the stored gradient; per source row "
            "ft, el, d_ft, d_el) + dglhip_rowsum_heads8_device (d_er)",
            timing="library launches per step less the forward call")
    if cpu and sample is not None:
        res["cpu_baseline"] = gat_layer_cpu(sample, n, H, D)
    return res


def _edge_attention(edges):
    # gat/train.py:90-96 (the reference's edge UDF), dropout 0
    a = F.leaky_relu(edges.src["a1"] + edges.dst["a2"], 0.2)
    a = torch.exp(a).clamp(-10, 10)
    return {"a": a, "a_drop": a}


def gat_layer_cpu(sample, n, H, D, target_edges=1_000_000):
    """The reference's layer on the host: the edge UDF for the attention,
    then update_all([src_mul_edge, copy_edge], [sum, sum]) and the division
    (gat/train.py:74-96), forward + backward, on the in-edges of the first
    rows of the headline's CPU sample (about ``target_edges``)."""
    import dgl
    import dgl.function as fn
    rows, d, s = sample
    cum = torch.cumsum(torch.bincount(d, minlength=rows), 0)
    r1 = min(int(torch.searchsorted(cum, torch.tensor(target_edges))) + 1, rows)
    sel = d < r1
    d, s = d[sel], s[sel]
    # sources keep their ids in the full table; rows are the first r1 nodes
    g = dgl.DGLGraph((s, d))
    if g.number_of_nodes() < n:
        g.add_nodes(n - g.number_of_nodes())
    gen = torch.Generator().manual_seed(6)
    ft = (torch.rand(n, H, D, generator=gen) * 2 - 1).requires_grad_(True)
    a1 = (torch.rand(n, H, 1, generator=gen) - 0.5).requires_grad_(True)
    a2 = (torch.rand(n, H, 1, generator=gen) - 0.5).requires_grad_(True)

    def once():
        g.ndata.update({"ft": ft, "a1": a1, "a2": a2})
        g.apply_edges(_edge_attention)
        g.update_all([fn.src_mul_edge("ft", "a_drop", "ft"), fn.copy_edge("a", "a")],
                     [fn.sum("ft", "ft"), fn.sum("a", "z")])
        out = g.ndata["ft"] / g.ndata["z"].clamp(min=1e-30)
        out[:r1].sum().backward()
    once()  # builds the host CSRs
    reps, t = 0, 0.0
    while reps < 2:
        t0 = time.perf_counter()
        once()
        t += time.perf_counter() - t0
        reps += 1
    e = int(s.numel())
    return {"value": e * reps / t, "unit": "edges/s (fwd+bwd)", "cores": _threads(),
            "kind": "port",
            "sample": "the reference's GAT layer (edge UDF attention + src_mul_edge/copy_edge "
                      "sums, gat/train.py:74-96) through this engine's host path, forward + "
                      "backward, on the in-edges of the first %d rows of the headline graph "
                      "(%d edges, sources over all %d nodes), %d heads x %d, %d reps, "
                      "torch %d threads" % (r1, e, n, H, D, reps, _threads())}


# -- GAT on Pubmed (configs[2]) ----------------------------------------------
def gat_pubmed_leg(dev, kernel, gather_peak, epochs=20, warmup=3, cpu=True):
    """configs[2]: the example's GAT (8 heads x 8 hidden, 8 output heads,
    fused layer aggregation) on the Pubmed-shaped dataset, one epoch =
    forward + cross-entropy + backward + Adam; eager and as one replayed HIP
    graph (gat/train.py --hip-graph)."""
    from dgl import DGLGraph
    from dgl.data import load_data
    gat = example("gat/train.py")
    data = load_data("pubmed", seed=0, device=dev)
    src, dst = data.graph
    g = DGLGraph((src.cpu(), dst.cpu()))
    g.add_edges(g.nodes(), g.nodes())
    E, n = g.number_of_edges(), g.number_of_nodes()

    def build(device, udf=False, capturable=False):
        torch.manual_seed(0)
        m = gat.GAT(g, 1, data.features.shape[1], 8, data.num_labels, [8, 8], F.elu, 0.6, 0.6,
                    0.2, False, udf).to(device)
        return m, torch.optim.Adam(m.parameters(), lr=0.005, weight_decay=5e-4,
                                   capturable=capturable, fused=device.type == "cuda")
    model, opt = build(dev)
    model.train()
    feats, labels = data.features, data.labels
    mask = data.train_mask.nonzero(as_tuple=True)[0]
    lab = labels[mask]

    def epoch():
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(model(feats).index_select(0, mask), lab)
        loss.backward()
        opt.step()
    ms, kms, launches = wall_steps(epoch, epochs, warmup, dev, kernel)
    # the same epoch captured once and replayed (the example's --hip-graph)
    gmodel, gopt = build(dev, capturable=True)
    gmodel.train()

    def gepoch():
        gopt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(gmodel(feats).index_select(0, mask), lab)
        loss.backward()
        gopt.step()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            gepoch()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    gopt.zero_grad(set_to_none=True)
    with torch.cuda.graph(graph, stream=side):
        gepoch()
    gms = call_ms(graph.replay, epochs, dev)
    # the dominant engine kernel: the first layer's fused aggregation forward
    layer = model.layers[0]
    with torch.no_grad():
        ft = layer.fc(feats).reshape(n, 8, -1)
        hf = ft.transpose(0, 1)
        a1 = torch.bmm(hf, layer.attn_l).transpose(0, 1).contiguous()
        a2 = torch.bmm(hf, layer.attn_r).transpose(0, 1).contiguous()
    ft, a1, a2 = ft.requires_grad_(True), a1.requires_grad_(True), a2.requires_grad_(True)
    adj = g.sparse_adjacency(dev)
    fms = call_ms(lambda: kernel.gat_aggregate(adj, ft, a1, a2, attn_drop=0.6), epochs, dev)
    D = ft.shape[2]
    peak, src_ = gather_peak(n * 8 * D * 4, 0)
    res = {"value": 1e3 / gms, "unit": "epochs/s (HIP graph)", "ms_per_epoch": ms,
           "ms_per_epoch_hip_graph": gms, "kernel_ms": kms, "launches_per_epoch": launches,
           "epochs": epochs, "warmup": warmup,
           "config": "configs[2]: GAT 8 heads x 8 hidden + 8 output heads on the Pubmed-shaped "
                     "dataset (%d nodes, %d edges incl. self-loops, 500 features, 3 classes), "
                     "dropout 0.6, Adam; eager and one replayed HIP graph per epoch" % (n, E),
           "roofline": roof(gat_fwd_bytes(E, n, 8, D, True) + E * 4 * 8, fms, peak, src_,
                            "fused GAT forward of layer 1 (attention dropout 0.6: the "
                            "attention and its dropped copy stored)",
                            regime="launch-bound: %.1f MB per call" %
                                   ((gat_fwd_bytes(E, n, 8, D, True) + E * 32) / 1e6)),
           "reference_v100_ms_per_epoch": 30.2,
           "cpu_baseline": None}
    if cpu:
        res["cpu_baseline"] = gat_pubmed_cpu(build, feats.cpu(), labels.cpu(), mask.cpu())
    return res


def gat_pubmed_cpu(build, feats, labels, mask, epochs=3):
    model, opt = build(torch.device("cpu"), udf=True)
    model.train()
    lab = labels[mask]

    def epoch():
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(model(feats).index_select(0, mask), lab)
        loss.backward()
        opt.step()
    epoch()
    t0 = time.perf_counter()
    for _ in range(epochs):
        epoch()
    ms = (time.perf_counter() - t0) / epochs * 1e3
    return {"value": 1e3 / ms, "unit": "epochs/s", "ms_per_epoch": ms, "cores": _threads(),
            "kind": "port",
            "sample": "the whole configs[2] epoch with the reference's edge UDF attention "
                      "(examples/gat/train.py --udf, gat/train.py:74-96) through this engine's "
                      "host path, %d epochs, torch %d threads" % (epochs, _threads())}


# -- R-GCN link prediction (configs[4]) ----------------------------------------
def rgcn_leg(dev, kernel, gather_peak, steps=20, warmup=3, cpu=True):
    """configs[4]: the example's R-GCN link-prediction step (2 block layers,
    500 hidden, 100 bases of 5 x 5, DistMult, Adam) on 30,000-edge samples of
    the FB15k-237-shaped KG; timed as the reference times it (forward +
    backward + clip + Adam, link_predict.py:163-171), sampled graphs built
    outside the timer."""
    import tools.rgcn_step as rs
    args = rs.lp.parser().parse_args([])
    prev_blas = rs.lp.select_blas(args.blas) if dev.type == "cuda" else None
    try:
        return _rgcn_leg(rs, args, dev, kernel, gather_peak, steps, warmup, cpu)
    finally:
        if prev_blas is not None:
            rs.lp.select_blas(prev_blas)


def _rgcn_leg(rs, args, dev, kernel, gather_peak, steps, warmup, cpu):
    raw = rs.make_samples(args, warmup + steps)
    samples = [rs.to_dev(s, dev) for s in raw]
    model, opt = rs.build_model(args, dev)
    model.train()
    graphs = []
    for s in samples:
        uniq, src, dst = s[0], s[1], s[2]
        from dgl import DGLGraph
        gg = DGLGraph((src, dst), multigraph=True)
        if gg.number_of_nodes() < len(uniq):
            gg.add_nodes(len(uniq) - gg.number_of_nodes())
        graphs.append(gg)
    it = iter(range(1 << 30))

    def step():  # the samples in turn (wall_steps' kernel-time pass reuses them)
        i = next(it) % len(samples)
        uniq, _, _, rel, norm, smp, lab = samples[i]
        h = model(graphs[i], uniq, rel, norm)
        loss = model.loss(h, smp, lab)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), args.grad_norm)
        opt.step()
    ms, kms, launches = wall_steps(step, steps, warmup, dev, kernel)
    kt = rs.kernel_times(model, samples[-1], dev)
    E = int(samples[0][1].numel())
    peak, src_ = gather_peak(len(raw[0][0]) * 500 * 4, 0)
    res = {"value": 1e3 / ms, "unit": "steps/s", "ms_per_step": ms, "kernel_ms": kms,
           "launches_per_step": launches, "steps": steps, "warmup": warmup,
           "config": "configs[4]: R-GCN link prediction, FB15k-237-shaped synthetic KG (14,541 "
                     "entities, 237 relations x 2 directions, 272,115 triples), %d-edge sampled "
                     "graph per step, 2 block layers of 100 bases 5x5 (500 hidden), DistMult, "
                     "Adam; graph sampling and DGLGraph build outside the timer (the "
                     "reference's); dense products on %s" % (E, args.blas),
           "typed_block_kernels": kt,
           "roofline": roof(kt["forward"]["bytes"], kt["forward"]["ms"], peak, src_,
                            "typed_block_spmm forward (chunked items + combine)",
                            regime="latency-bound: %.0f MB per call over %d rows"
                                   % (kt["forward"]["bytes"] / 1e6, kt["rows"])),
           "reference_v100_ms_per_step": 633.0,
           "cpu_baseline": None}
    if cpu:
        res["cpu_baseline"] = rgcn_cpu(rs, raw[:3])
    return res


def rgcn_cpu(rs, raw):
    args = rs.lp.parser().parse_args(["--udf"])
    dev = torch.device("cpu")
    model, opt = rs.build_model(args, dev)
    model.train()
    samples = [rs.to_dev(s, dev) for s in raw]
    rs.one_step(model, opt, samples[0], args)
    t0 = time.perf_counter()
    for s in samples[1:]:
        rs.one_step(model, opt, s, args)
    ms = (time.perf_counter() - t0) / (len(samples) - 1) * 1e3
    return {"value": 1e3 / ms, "unit": "steps/s", "ms_per_step": ms, "cores": _threads(),
            "kind": "port",
            "sample": "the same step with the reference's formulation (edge UDF gather + bmm "
                      "into an E x 500 message tensor, builtin sum, rgcn/layers.py:121-132; "
                      "link_predict.py --udf) through this engine's host path, %d steps on the "
                      "same samples, torch %d threads" % (len(samples) - 1, _threads())}


# -- GraphSAGE-mean epoch on the Reddit-shaped graph ---------------------------
def sage_leg(g, dev, kernel, gather_peak, algorithmic_bytes, sample, epochs=10, warmup=3,
             cpu=True):
    """configs[3]'s model (GraphSAGE-mean, 602 -> 128 -> 41, examples/
    graphsage/train.py) for one full-graph epoch (forward + loss + backward +
    Adam) on the bench's Reddit-shaped graph, random 602-wide features, 41
    classes, 66 % training nodes."""
    import dgl.function as fn
    from dgl.nn.pytorch import weighted_cross_entropy
    sage = example("graphsage/train.py")
    n, E = g.number_of_nodes(), g.number_of_edges()
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    feats = 0.1 * torch.randn(n, 602, generator=gen, device=dev)
    labels = torch.randint(0, 41, (n,), generator=gen, device=dev)
    train_w = (torch.rand(n, generator=gen, device=dev) < 0.66).float()
    ntrain = float(train_w.sum())

    def aggregate(h):
        g.ndata["h"] = h
        g.update_all(fn.copy_src("h", "m"), fn.mean("m", "neigh"))
        return g.ndata.pop("neigh")
    aggregate.add_into = lambda h, out: kernel.gspmm_mean_add(g.sparse_adjacency(h.device),
                                                              h, out)
    torch.manual_seed(0)
    model = sage.SAGE(602, 128, 41, 1, 0.0).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    model.train()

    def epoch():
        logits = model(feats, aggregate)
        loss = weighted_cross_entropy(logits, labels, train_w) * (1.0 / ntrain)
        opt.zero_grad()
        loss.backward()
        opt.step()
    ms, kms, launches = wall_steps(epoch, epochs, warmup, dev, kernel)
    h = torch.rand(n, 128, generator=gen, device=dev)
    adj = g.sparse_adjacency(dev)
    ams = call_ms(lambda: kernel.gspmm(adj, "copy_u", "mean", h), epochs, dev)
    blocks = kernel.blocked_schedule(adj, h)
    peak, src_ = gather_peak(n * 128 * 4, blocks)
    res = {"value": 1e3 / ms, "unit": "epochs/s", "ms_per_epoch": ms, "kernel_ms": kms,
           "launches_per_epoch": launches, "epochs": epochs, "warmup": warmup,
           "config": "configs[3]'s model (GraphSAGE-mean 602-128-41, fc_neigh ahead of the "
                     "mean, NodeLinear, fused loss; examples/graphsage/train.py) for one "
                     "full-graph epoch on the headline graph (%d nodes, %d edges), 66 %% "
                     "training nodes, Adam" % (n, E),
           "roofline": roof(algorithmic_bytes(E, n, 128), ams, peak, src_,
                            "g-SpMM copy_u + mean, F = 128 (one layer's aggregation; %d "
                            "launches per call)" % max(blocks, 1)),
           "cpu_baseline": None}
    if cpu and sample is not None:
        res["cpu_baseline"] = mean_bucketing_cpu(sample, n)
    return res


def sage_rmat_leg(st, dev, kernel, gather_peak, algorithmic_bytes, epochs=2, warmup=1, cpu=True):
    """configs[3] at its own size: GraphSAGE-mean 128-128-41 (examples/
    graphsage/train.py: fc_neigh ahead of the mean, NodeLinear, the fused
    loss) for full-graph epochs (forward + loss + backward + Adam) on the
    rmat leg's RMAT-26 graph (67.1M nodes, 1.07B edges), one GPU, heavy rows
    chunked, edge ids offloaded (copy_u + mean never reads them), random
    128-wide features, 41 classes, 66 % training nodes. The reference has no
    GraphSAGE example; its timing loop is gcn_spmv.py:168-182's."""
    from dgl.nn.pytorch import weighted_cross_entropy
    sage = example("graphsage/train.py")
    adj, n, sample = st["adj"], st["n"], st.get("sample")
    st.clear()
    E = adj.fwd.nnz
    old = kernel.set_row_split("auto")
    try:
        t0 = time.time()
        adj.bwd  # the transposed CSR (the backward's), built ahead of the epochs
        adj.offload_edge_ids()
        _sync(dev)
        build_s = time.time() - t0
        if dev.type == "cuda":
            # the rmat leg's freed 34-GB blocks go back to the device: the
            # epochs' differently sized tensors would otherwise make the
            # caching allocator free and retry mid-epoch
            torch.cuda.empty_cache()
            retries0 = torch.cuda.memory_stats(dev).get("num_alloc_retries", 0)
        gen = torch.Generator(device=dev)
        gen.manual_seed(9)
        feats = 0.1 * torch.randn(n, 128, generator=gen, device=dev)
        labels = torch.randint(0, 41, (n,), generator=gen, device=dev)
        train_w = (torch.rand(n, generator=gen, device=dev) < 0.66).float()
        ntrain = float(train_w.sum())

        def aggregate(h):
            return kernel.gspmm(adj, "copy_u", "mean", h)
        aggregate.add_into = lambda h, out: kernel.gspmm_mean_add(adj, h, out)
        torch.manual_seed(0)
        model = sage.SAGE(128, 128, 41, 1, 0.0).to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=1e-2)
        model.train()

        def epoch():
            logits = model(feats, aggregate)
            loss = weighted_cross_entropy(logits, labels, train_w) * (1.0 / ntrain)
            opt.zero_grad()
            loss.backward()
            opt.step()
        ms, kms, launches = wall_steps(epoch, epochs, warmup, dev, kernel)
        peak_mem = torch.cuda.max_memory_allocated(dev) / 1e9 if dev.type == "cuda" else None
        retries = (torch.cuda.memory_stats(dev).get("num_alloc_retries", 0) - retries0
                   if dev.type == "cuda" else None)
        del model, opt
        h = feats  # the first layer's aggregation alone, for the roofline
        ams = call_ms(lambda: kernel.gspmm(adj, "copy_u", "mean", h), 2, dev)
    finally:
        kernel.set_row_split(old)
    peak, src_ = gather_peak(n * 128 * 4, 0)
    res = {"value": 1e3 / ms, "unit": "epochs/s", "ms_per_epoch": ms, "kernel_ms": kms,
           "launches_per_epoch": launches, "epochs": epochs, "warmup": warmup,
           "transposed_csr_build_s": build_s, "peak_hbm_gb": peak_mem,
           "alloc_retries": retries,
           "config": "configs[3] (GraphSAGE-mean 128-128-41, examples/graphsage/train.py) for "
                     "full-graph epochs on the rmat leg's graph (RMAT-%d: %d nodes, %d edges), "
                     "one GPU, heavy rows chunked, 66 %% training nodes, Adam"
                     % (int(round(np.log2(max(n, 1)))), n, E),
           "roofline": roof(algorithmic_bytes(E, n, 128), ams, peak, src_,
                            "g-SpMM copy_u + mean, F = 128 (the first layer's aggregation "
                            "over the whole graph; heavy-row chunks and short-row tiers)"),
           "cpu_baseline": None}
    if cpu and sample is not None:
        res["cpu_baseline"] = mean_bucketing_cpu(sample, n, sparse_table=True)
    return res


def mean_bucketing_cpu(sample, n, F_=128, target_edges=2_000_000, sparse_table=False):
    """The reference's mean aggregation on the host: no builtin mean exists
    (function/reducer.py: sum, max), so ``lambda nodes: mailbox.mean(1)``
    runs under degree bucketing (runtime/degree_bucketing.py:13-84: rows
    grouped by in-degree, each bucket's messages gathered into (rows, deg,
    F) and reduced, the buckets merged by row id) — restated here with torch
    on a sample of the headline graph (the in-edges of its first rows)."""
    rows, d, s = sample
    cum = torch.cumsum(torch.bincount(d, minlength=rows), 0)
    r1 = min(int(torch.searchsorted(cum, torch.tensor(target_edges))) + 1, rows)
    sel = d < r1
    d, s = d[sel], s[sel]
    e = int(s.numel())
    if sparse_table:
        # a full-size (n, F) table whose pages are touched only for the
        # sample's source rows (RMAT-26: 34 GB of address space, the sample's
        # rows resident), as bench.cpu_baseline does
        h = torch.empty(n, F_)
        uniq = torch.unique(s)
        h[uniq] = torch.rand(uniq.numel(), F_, generator=torch.Generator().manual_seed(8))
    else:
        h = torch.rand(n, F_, generator=torch.Generator().manual_seed(8))
    order = torch.sort(d, stable=True)[1]  # mailbox order: edge order within a row
    d, s = d[order], s[order]

    def once():
        deg = torch.bincount(d, minlength=r1)
        starts = torch.zeros(r1 + 1, dtype=torch.int64)
        torch.cumsum(deg, 0, out=starts[1:])
        out = torch.zeros(r1, F_)
        for k in torch.unique(deg[deg > 0]).tolist():
            vb = torch.nonzero(deg == k).squeeze(1)
            mids = (starts[vb].unsqueeze(1) + torch.arange(k)).reshape(-1)
            mail = h.index_select(0, s.index_select(0, mids)).view(-1, k, F_)
            out[vb] = mail.mean(1)
        return out
    once()
    reps, t = 0, 0.0
    while reps < 2:
        t0 = time.perf_counter()
        once()
        t += time.perf_counter() - t0
        reps += 1
    return {"value": e * reps / t, "unit": "edges/s (mean aggregation)", "cores": _threads(),
            "kind": "port",
            "sample": "degree-bucketing mean (the reference's UDF route for mean, "
                      "degree_bucketing.py:13-84) restated with torch, on the in-edges of the "
                      "first %d rows of the graph (%d edges, F = %d), %d reps, torch "
                      "%d threads; GPU comparison: roofline.kernel_ms is one such aggregation "
                      "over the whole graph" % (r1, e, F_, reps, _threads())}
