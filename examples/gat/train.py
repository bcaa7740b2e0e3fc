"""Graph Attention Network on the engine (counterpart of the reference's
examples/pytorch/gat/train.py; BASELINE.json configs[2]: 8 heads on Pubmed).

Per layer, by default ONE kernel (dgl.kernel.gat_aggregate): the
unnormalised attention exp(leaky_relu(a_l[src] + a_r[dst])), its dropout, the
per-head weighted sum of the source features and the copy_edge normaliser, in
one pass over each destination row's in-edges (the attention kept in CSR slot
order only for the backward). ``--unfused`` runs the same arithmetic as three
kernels (attention g-SDDMM, then ONE
``update_all([src_mul_edge('ft','a_drop','ft'), copy_edge('a','a')],
[sum('ft','ft'), sum('a','z')])`` whose pairs are fused g-SpMMs) with torch's
dropout; ``--udf`` runs the reference's edge UDF for the attention. The
reference materialises E x H x D messages and reduces them with an
incidence-matrix SPMV.

  python examples/gat/train.py --dataset pubmed --gpu 0 [--hip-graph]

``--hip-graph`` captures the whole training step (forward, backward, Adam) in
one HIP graph after three warm-up steps and replays it: Pubmed is small
enough that per-launch host cost dominates an eager epoch.
"""
import argparse
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "dgl-1_amd"))
import dgl.function as fn  # noqa: E402
from dgl import DGLGraph, kernel  # noqa: E402
from dgl.nn.pytorch.linear import NodeLinear  # noqa: E402
from dgl.data import load_data  # noqa: E402


class GraphAttention(nn.Module):
    def __init__(self, g, in_dim, out_dim, num_heads, feat_drop, attn_drop, alpha, residual,
                 udf=False, unfused=False):
        super(GraphAttention, self).__init__()
        self.g = g
        self.udf = udf
        self.unfused = unfused
        self.alpha = alpha
        self.num_heads = num_heads
        # the engine's per-node Linear (nn.Linear's parameters, initialisation
        # and forward; its weight gradient split over the node dimension: torch's
        # GEMM ran Pubmed's 19,717-deep reductions on one to 33 workgroups)
        self.fc = NodeLinear(in_dim, num_heads * out_dim, bias=False)
        self.feat_drop = nn.Dropout(feat_drop) if feat_drop else None
        self.attn_drop = nn.Dropout(attn_drop) if attn_drop else None
        self.attn_l = nn.Parameter(torch.Tensor(size=(num_heads, out_dim, 1)))
        self.attn_r = nn.Parameter(torch.Tensor(size=(num_heads, out_dim, 1)))
        for p in (self.fc.weight, self.attn_l, self.attn_r):
            nn.init.xavier_normal_(p.data, gain=1.414)
        self.leaky_relu = nn.LeakyReLU(alpha)
        self.residual = residual
        self.res_fc = None
        if residual and in_dim != num_heads * out_dim:
            self.res_fc = NodeLinear(in_dim, num_heads * out_dim, bias=False)
            nn.init.xavier_normal_(self.res_fc.weight.data, gain=1.414)

    def forward(self, h):
        if self.feat_drop is not None:
            h = self.feat_drop(h)
        ft = self.fc(h).reshape((h.shape[0], self.num_heads, -1))     # N x H x D
        # the reference's bmm(head_ft, attn_l) (gat/train.py:66-67) in the
        # library (kernel.gat_logits: a fixed association; its backward
        # reduces attn's gradient over the nodes in torch's column reduction
        # instead of a GEMM with an H x D x 1 output and a 19,717-deep K, 0.1 ms
        # per call on one workgroup per head). Given the same ft (no feature
        # dropout in between), the fused aggregation recomputes el from the
        # rows it gathers
        a1, a2 = kernel.gat_logits(ft, self.attn_l, self.attn_r)      # N x H x 1
        if self.feat_drop is not None:
            ft = self.feat_drop(ft)
        if self.udf:  # the reference's edge UDF (gat/train.py:90-96)
            self.g.ndata.update({"ft": ft, "a1": a1.contiguous(), "a2": a2.contiguous()})
            self.g.apply_edges(self.edge_attention)
            self.g.update_all([fn.src_mul_edge("ft", "a_drop", "ft"), fn.copy_edge("a", "a")],
                              [fn.sum("ft", "ft"), fn.sum("a", "z")])
            ret = self.g.ndata["ft"] / self.g.ndata["z"]
        elif self.unfused:  # three kernels: attention g-SDDMM, u_mul_e and copy_e g-SpMMs
            self.g.ndata["ft"] = ft
            a = kernel.edge_attention(self.g.sparse_adjacency(h.device), a1, a2,
                                      self.g.number_of_edges(), self.alpha)
            a = a.unsqueeze(-1)  # E x H x 1
            a_drop = self.attn_drop(a) if self.attn_drop is not None else a
            self.g.edata.update({"a": a, "a_drop": a_drop})
            self.g.update_all([fn.src_mul_edge("ft", "a_drop", "ft"), fn.copy_edge("a", "a")],
                              [fn.sum("ft", "ft"), fn.sum("a", "z")])
            ret = self.g.ndata["ft"] / self.g.ndata["z"]
        else:  # one kernel: attention, dropout, weighted sum and normaliser
            ft_sum, z = kernel.gat_aggregate(
                self.g.sparse_adjacency(h.device), ft, a1, a2, self.alpha,
                attn_drop=self.attn_drop.p if self.attn_drop is not None else 0.0,
                training=self.training)
            ret = ft_sum / z
        if self.residual:
            res = self.res_fc(h).reshape(ret.shape) if self.res_fc is not None \
                else h.reshape(ret.shape)
            ret = res + ret
        return ret

    def edge_attention(self, edges):
        a = self.leaky_relu(edges.src["a1"] + edges.dst["a2"])
        a = torch.exp(a).clamp(-10, 10)
        a_drop = self.attn_drop(a) if self.attn_drop is not None else a
        return {"a": a, "a_drop": a_drop}


class GAT(nn.Module):
    def __init__(self, g, num_layers, in_dim, num_hidden, num_classes, heads, activation,
                 feat_drop, attn_drop, alpha, residual, udf=False, unfused=False):
        super(GAT, self).__init__()
        self.activation = activation
        kw = {"udf": udf, "unfused": unfused}
        self.layers = nn.ModuleList([GraphAttention(g, in_dim, num_hidden, heads[0], feat_drop,
                                                    attn_drop, alpha, False, **kw)])
        for i in range(1, num_layers):
            self.layers.append(GraphAttention(g, num_hidden * heads[i - 1], num_hidden, heads[i],
                                              feat_drop, attn_drop, alpha, residual, **kw))
        self.layers.append(GraphAttention(g, num_hidden * heads[-2], num_classes, heads[-1],
                                          feat_drop, attn_drop, alpha, residual, **kw))

    def forward(self, h):
        for layer in self.layers[:-1]:
            h = self.activation(layer(h).flatten(1))
        return self.layers[-1](h).mean(1)


def run(args):
    device = torch.device("cpu") if args.gpu < 0 else torch.device("cuda", args.gpu)
    data = load_data(args.dataset, seed=args.seed, device=device)
    src, dst = data.graph
    g = DGLGraph((src.cpu(), dst.cpu()))
    g.add_edges(g.nodes(), g.nodes())  # self-loops (gat/train.py:189)
    torch.manual_seed(args.seed)
    heads = [args.num_heads] * args.num_layers + [args.num_out_heads]
    model = GAT(g, args.num_layers, data.features.shape[1], args.num_hidden, data.num_labels,
                heads, F.elu, args.in_drop, args.attn_drop, args.alpha, args.residual, args.udf,
                args.unfused)
    model = model.to(device)
    # one fused kernel per step on the device (torch's multi-tensor Adam: 20
    # launches per epoch)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr, weight_decay=args.weight_decay,
                           capturable=args.hip_graph, fused=device.type == "cuda")
    if args.hip_graph:
        return run_captured(args, model, opt, data, g)
    dur = []
    for epoch in range(args.epochs):
        model.train()
        if device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.time()
        logits = model(data.features)
        loss = F.cross_entropy(logits[data.train_mask], data.labels[data.train_mask])
        opt.zero_grad()
        loss.backward()
        opt.step()
        if device.type == "cuda":
            torch.cuda.synchronize()
        if epoch >= 3:
            dur.append(time.time() - t0)
    mean = sum(dur) / len(dur) if dur else float("nan")
    return {"dataset": args.dataset, "epoch_s": mean, "edges": g.number_of_edges(),
            "loss": float(loss.item())}


def run_captured(args, model, opt, data, g):
    """Training step captured once in a HIP graph, then replayed. The mask is
    an index tensor (boolean indexing would sync with the host during capture);
    dropout draws from torch's graph-safe generator state."""
    feats, labels = data.features, data.labels
    mask = data.train_mask.nonzero(as_tuple=True)[0]
    labels_train = labels[mask]
    model.train()

    def step():
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(model(feats).index_select(0, mask), labels_train)
        loss.backward()
        opt.step()
        return loss
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):  # warm-up: cached CSRs (fwd + transposed), allocator pools
            step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=True)
    # same stream as the warm-up (where the AccumulateGrad nodes were made)
    with torch.cuda.graph(graph, stream=side):
        static_loss = step()
    dur = []
    for _ in range(3, args.epochs):  # the warm-up steps count as epochs 0-2
        torch.cuda.synchronize()
        t0 = time.time()
        graph.replay()
        torch.cuda.synchronize()
        dur.append(time.time() - t0)
    mean = sum(dur) / len(dur) if dur else float("nan")
    return {"dataset": args.dataset, "epoch_s": mean, "edges": g.number_of_edges(),
            "loss": float(static_loss.item()), "hip_graph": True}


def parser():
    p = argparse.ArgumentParser(description="GAT on the MI355X engine")
    p.add_argument("--dataset", default="pubmed")
    p.add_argument("--gpu", type=int, default=-1)
    p.add_argument("--epochs", type=int, default=200)
    p.add_argument("--num-heads", type=int, default=8)
    p.add_argument("--num-out-heads", type=int, default=8)
    p.add_argument("--num-layers", type=int, default=1)
    p.add_argument("--num-hidden", type=int, default=8)
    p.add_argument("--residual", action="store_true")
    p.add_argument("--in-drop", type=float, default=0.6)
    p.add_argument("--attn-drop", type=float, default=0.6)
    p.add_argument("--lr", type=float, default=0.005)
    p.add_argument("--weight-decay", type=float, default=5e-4)
    p.add_argument("--alpha", type=float, default=0.2)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--udf", action="store_true", help="reference edge UDF for the attention")
    p.add_argument("--unfused", action="store_true",
                   help="attention g-SDDMM + u_mul_e and copy_e g-SpMMs as three kernels "
                        "(torch dropout) instead of the one fused kernel")
    p.add_argument("--hip-graph", action="store_true",
                   help="capture the training step in a HIP graph and replay it (GPU)")
    return p


if __name__ == "__main__":
    print(run(parser().parse_args()))
