"""R-GCN link-prediction training step at configs[4]'s shape, phase by phase.

The reference times forward (model.get_loss) and backward + clip + Adam
(/root/reference/examples/pytorch/rgcn/link_predict.py:163-171); the sampled
graph is built before its timer. Here, per step on pre-drawn samples:

  graph     DGLGraph from the sample's (src, dst) (the reference's sampler output)
  forward   embedding -> 2 R-GCN block layers -> DistMult loss (the device
            CSR, its transpose and the relation groups are built inside, on
            first use, as in the reference's lazy adjacency)
  backward  loss.backward + clip_grad_norm_ + Adam

with a synchronize after each phase, and the same steps unsynchronised
(``step_ms``: graph + forward + backward as one region). ``--kernels`` adds
each typed-block kernel alone, timed with events on the launch stream, with
its algorithmic bytes.

  python tools/rgcn_step.py [--steps 20] [--udf] [--kernels]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import DGLGraph, kernel  # noqa: E402


def _load_example(relpath, name):
    import importlib.util
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "examples", relpath))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


lp = _load_example("rgcn/link_predict.py", "rgcn_step_lp")


def make_samples(args, steps):
    triplets = lp.synthetic_kg(args.num_entities, args.num_rels, args.num_triples, args.seed)
    rng = np.random.default_rng(args.seed)
    return [lp.sample_graph(triplets, args.graph_batch_size, args.num_rels, rng)
            for _ in range(steps)]


def to_dev(sample, dev):
    uniq, src, dst, rel, norm, samples, labels = sample
    return (torch.from_numpy(uniq).to(dev), torch.from_numpy(src), torch.from_numpy(dst),
            torch.from_numpy(rel).to(dev), torch.from_numpy(norm).to(dev),
            torch.from_numpy(samples).to(dev), torch.from_numpy(labels).to(dev))


def build_model(args, dev):
    torch.manual_seed(args.seed)
    model = lp.LinkPredict(args.num_entities, args.n_hidden, args.num_rels, args.n_bases,
                           args.dropout, args.regularization, args.udf).to(dev)
    return model, torch.optim.Adam(model.parameters(), lr=args.lr, fused=dev.type == "cuda")


def one_step(model, opt, s, args, sync=None):
    uniq, src, dst, rel, norm, samples, labels = s
    t = [time.perf_counter()]
    g = DGLGraph((src, dst), multigraph=True)
    if g.number_of_nodes() < len(uniq):
        g.add_nodes(len(uniq) - g.number_of_nodes())
    if sync:
        sync()
        t.append(time.perf_counter())
    h = model(g, uniq, rel, norm)
    loss = model.loss(h, samples, labels)
    if sync:
        sync()
        t.append(time.perf_counter())
    opt.zero_grad()
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), args.grad_norm)
    opt.step()
    if sync:
        sync()
        t.append(time.perf_counter())
    return loss, t


def kernel_times(model, s, dev, iters=20):
    """Each typed-block kernel of layer 0 alone: (ms per call, algorithmic
    bytes) for the forward g-SpMM, the transposed dH g-SpMM and dW."""
    uniq, src, dst, rel, norm, _, _ = s
    norm = norm.index_select(0, dst.to(norm.device))  # per edge: 1 / in-degree of its dst
    g = DGLGraph((src, dst), multigraph=True)
    if g.number_of_nodes() < len(uniq):
        g.add_nodes(len(uniq) - g.number_of_nodes())
    adj = g.sparse_adjacency(dev)
    layer = model.layers[0]
    w = layer.weight.detach().clone().requires_grad_(True)
    R, nb, si, so = w.shape
    h = (torch.rand(len(uniq), nb * si, device=dev) - 0.5).requires_grad_(True)
    E, N = int(src.numel()), len(uniq)
    res = {}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        kernel.timing_enable(True)
        for _ in range(iters):
            fn()
        ms, n = kernel.timing_read()
        kernel.timing_enable(False)
        return ms / iters, n // iters

    out = kernel.typed_block_spmm(adj, h, w, rel, norm)
    dout = torch.rand_like(out)
    # per edge: col id, eid, etype, norm, the source row (Fi floats) and the
    # weight block column it reads (L2-resident: counted once per call);
    # per row: indptr, output row
    Fi, Fo = nb * si, nb * so
    wbytes = R * nb * si * so * 4
    fwd_b = E * (4 + 8 + 8 + 4 + 4 * Fi) + N * (8 + 4 * Fo) + wbytes
    ms, n = timed(lambda: kernel.typed_block_spmm(adj, h.detach(), w.detach(), rel, norm))
    res["forward"] = {"ms": ms, "launches": n, "bytes": fwd_b}
    with torch.no_grad():
        pass
    du_b = E * (4 + 8 + 8 + 4 + 4 * Fo) + N * (8 + 4 * Fi) + wbytes

    def bwd_du():
        o = kernel.typed_block_spmm(adj, h, w.detach(), rel, norm)
        torch.autograd.grad(o, h, dout)
    ms_all, n_all = timed(bwd_du)
    res["forward+dH"] = {"ms": ms_all, "launches": n_all, "bytes": fwd_b + du_b}

    def bwd_dw():
        o = kernel.typed_block_spmm(adj, h.detach(), w, rel, norm)
        torch.autograd.grad(o, w, dout)
    ms_w, n_w = timed(bwd_dw)
    # dW: per edge the source row and the destination's gradient row once
    dw_b = E * (4 + 8 + 8 + 4 + 4 * Fi + 4 * Fo) + wbytes
    res["forward+dW"] = {"ms": ms_w, "launches": n_w, "bytes": fwd_b + dw_b}
    res["dH_ms"] = ms_all - ms
    res["dW_ms"] = ms_w - ms
    for key, b in (("dH", du_b), ("dW", dw_b)):
        t = res[key + "_ms"]
        res[key + "_GBs"] = b / (t * 1e-3) / 1e9 if t > 0 else None
    res["forward_GBs"] = fwd_b / (ms * 1e-3) / 1e9
    res["edges"], res["rows"] = E, N
    return res


def main():
    ap = lp.parser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--kernels", action="store_true")
    ap.add_argument("--typed-width", type=int, default=1,
                    help="output slices of 64 per typed-block wave (study knob)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    kernel.set_typed_block_width(args.typed_width)
    if dev.type == "cuda":
        lp.select_blas(args.blas)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    raw = make_samples(args, args.warmup + args.steps)
    samples = [to_dev(s, dev) for s in raw]
    model, opt = build_model(args, dev)
    model.train()
    for s in samples[:args.warmup]:
        one_step(model, opt, s, args)
    sync()
    phases = []
    for s in samples[args.warmup:]:
        _, t = one_step(model, opt, s, args, sync)
        phases.append(np.diff(t) * 1e3)
    ph = np.mean(phases, 0)
    sync()
    t0 = time.perf_counter()
    for s in samples[args.warmup:]:
        loss, _ = one_step(model, opt, s, args)
    sync()
    step = (time.perf_counter() - t0) / args.steps * 1e3
    res = {"udf": args.udf, "steps": args.steps, "graph_edges": int(samples[0][1].numel()),
           "rows": int(samples[0][0].numel()),
           "phase_ms": {"graph": ph[0], "forward": ph[1], "backward": ph[2]},
           "step_ms": step, "loss": float(loss.item())}
    if args.kernels and dev.type == "cuda" and not args.udf:
        res["kernels"] = kernel_times(model, samples[-1], dev)
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
