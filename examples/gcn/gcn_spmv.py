"""GCN with the builtin SPMV path (counterpart of the reference's
examples/pytorch/gcn/gcn_spmv.py): Linear -> * norm -> update_all(copy_src,
sum) -> * norm -> bias/activation, trained full-graph with Adam.

BASELINE.json configs[0] (Cora, CPU) and configs[1] (Reddit, hidden 128,
1 x MI355X). Datasets are shape-matched synthetic graphs (dgl.data).

  python examples/gcn/gcn_spmv.py --dataset cora --gpu -1
  python examples/gcn/gcn_spmv.py --dataset reddit --gpu 0 --n-hidden 128
"""
import argparse
import math
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "dgl-1_amd"))
import dgl  # noqa: E402
import dgl.function as fn  # noqa: E402
from dgl import DGLGraph  # noqa: E402
from dgl.data import load_data  # noqa: E402
from dgl.nn.pytorch import dense_mm, node_epilogue  # noqa: E402


class GCNLayer(nn.Module):
    def __init__(self, g, in_feats, out_feats, activation, dropout, bias=True):
        super(GCNLayer, self).__init__()
        self.g = g
        self.weight = nn.Parameter(torch.Tensor(in_feats, out_feats))
        self.bias = nn.Parameter(torch.Tensor(out_feats)) if bias else None
        self.activation = activation
        self.dropout = nn.Dropout(p=dropout) if dropout else None
        stdv = 1. / math.sqrt(self.weight.size(1))
        self.weight.data.uniform_(-stdv, stdv)
        if self.bias is not None:
            self.bias.data.uniform_(-stdv, stdv)

    def forward(self, h):
        if self.dropout is not None:
            h = self.dropout(h)
        # dense Linear: MFMA via torch/hipBLASLt; its weight gradient split
        # over row chunks (one GEMM with K = 232,965 filled 20 of 256 CUs)
        h = dense_mm(h, self.weight)
        h = h * self.g.ndata["norm"]          # source-degree normalisation
        self.g.ndata["h"] = h
        self.g.update_all(fn.copy_src(src="h", out="m"), fn.sum(msg="m", out="h"))  # g-SpMM
        h = self.g.ndata.pop("h")
        # destination-degree normalisation, + bias, activation: one pass each
        # way on the device (the bits of `h * norm`, `+ bias`, `relu`)
        return node_epilogue(h, self.g.ndata["norm"], self.bias, self.activation)


class GCN(nn.Module):
    def __init__(self, g, in_feats, n_hidden, n_classes, n_layers, activation, dropout):
        super(GCN, self).__init__()
        self.layers = nn.ModuleList([GCNLayer(g, in_feats, n_hidden, activation, 0.)])
        for _ in range(n_layers - 1):
            self.layers.append(GCNLayer(g, n_hidden, n_hidden, activation, dropout))
        self.layers.append(GCNLayer(g, n_hidden, n_classes, None, dropout))

    def forward(self, features):
        h = features
        for layer in self.layers:
            h = layer(h)
        return h


def build_graph(data, device):
    """Graph + self-loops + symmetric normalisation, as gcn_spmv.py:131-143."""
    src, dst = data.graph
    g = DGLGraph((src.cpu(), dst.cpu()))
    g.add_edges(g.nodes(), g.nodes())
    degs = g.in_degrees().float()
    norm = torch.pow(degs, -0.5)
    norm[torch.isinf(norm)] = 0
    g.ndata["norm"] = norm.unsqueeze(1).to(device)
    return g


def evaluate(model, features, labels, mask):
    model.eval()
    with torch.no_grad():
        logits = model(features)[mask]
        return (logits.argmax(1) == labels[mask]).float().mean().item()


def run(args):
    device = torch.device("cpu") if args.gpu < 0 else torch.device("cuda", args.gpu)
    data = load_data(args.dataset, seed=args.seed, device=device)
    g = build_graph(data, device)
    n_edges = g.number_of_edges()
    torch.manual_seed(args.seed)
    model = GCN(g, data.features.shape[1], args.n_hidden, data.num_labels, args.n_layers,
                F.relu, args.dropout).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr, weight_decay=args.weight_decay,
                           capturable=args.hip_graph, fused=device.type == "cuda")
    loss_fcn = nn.CrossEntropyLoss()
    dur = []
    if args.hip_graph:
        return run_captured(args, model, opt, loss_fcn, data, g, n_edges)
    for epoch in range(args.n_epochs):
        model.train()
        if device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.time()
        logits = model(data.features)
        loss = loss_fcn(logits[data.train_mask], data.labels[data.train_mask])
        opt.zero_grad()
        loss.backward()
        opt.step()
        if device.type == "cuda":
            torch.cuda.synchronize()
        if epoch >= 3:
            dur.append(time.time() - t0)
        if args.verbose:
            acc = evaluate(model, data.features, data.labels, data.val_mask)
            mean = sum(dur) / len(dur) if dur else float("nan")
            print("Epoch {:05d} | Time(s) {:.4f} | Loss {:.4f} | Accuracy {:.4f} | "
                  "ETputs(KTEPS) {:.2f}".format(epoch, mean, loss.item(), acc,
                                                n_edges / mean / 1000 if dur else 0.0))
    mean = sum(dur) / len(dur) if dur else float("nan")
    return {"dataset": args.dataset, "epoch_s": mean, "edges": n_edges,
            "loss": float(loss.item()),
            "test_acc": evaluate(model, data.features, data.labels, data.test_mask)}


def run_captured(args, model, opt, loss_fcn, data, g, n_edges):
    """Whole training step (forward, backward, Adam) captured once in a HIP
    graph and replayed: removes the per-launch host cost that dominates small
    graphs. The g-SpMM launches go to torch's current (capturing) stream."""
    feats, labels = data.features, data.labels
    mask = data.train_mask.nonzero(as_tuple=True)[0]  # index form: no host sync in capture
    labels_train = labels[mask]
    model.train()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):  # warm-up builds the cached CSRs (fwd + transposed)
            opt.zero_grad(set_to_none=True)
            loss = loss_fcn(model(feats).index_select(0, mask), labels_train)
            loss.backward()
            opt.step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=True)
    # capture on the warm-up stream: the parameters' AccumulateGrad nodes were
    # created there, so the captured backward accumulates on the same stream
    with torch.cuda.graph(graph, stream=side):
        static_loss = loss_fcn(model(feats).index_select(0, mask), labels_train)
        static_loss.backward()
        opt.step()
    dur = []
    for epoch in range(3, args.n_epochs):  # the 3 warm-up steps count as epochs 0-2
        torch.cuda.synchronize()
        t0 = time.time()
        graph.replay()
        torch.cuda.synchronize()
        dur.append(time.time() - t0)
    mean = sum(dur) / len(dur) if dur else float("nan")
    return {"dataset": args.dataset, "epoch_s": mean, "edges": n_edges,
            "loss": float(static_loss.item()), "hip_graph": True,
            "test_acc": evaluate(model, feats, labels, data.test_mask)}


def parser():
    p = argparse.ArgumentParser(description="GCN (SPMV path) on the MI355X engine")
    p.add_argument("--dataset", default="cora")
    p.add_argument("--gpu", type=int, default=-1)
    p.add_argument("--dropout", type=float, default=0.5)
    p.add_argument("--lr", type=float, default=1e-2)
    p.add_argument("--n-epochs", type=int, default=200)
    p.add_argument("--n-hidden", type=int, default=16)
    p.add_argument("--n-layers", type=int, default=1)
    p.add_argument("--weight-decay", type=float, default=5e-4)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--hip-graph", action="store_true",
                   help="capture the training step in a HIP graph and replay it (GPU)")
    return p


if __name__ == "__main__":
    print(run(parser().parse_args()))
