"""R-GCN link prediction (counterpart of the reference's
examples/pytorch/rgcn/link_predict.py; BASELINE.json configs[4]).

Model as the reference: entity embedding -> 2 block-diagonal R-GCN layers
(hidden 500, 100 bases of 5 x 5, self-loop, dropout) -> DistMult scores with
negative sampling, on a sampled 30,000-edge training graph per step (edges in
both directions, reverse relations, norm = 1 / in-degree).

The message passing of each layer is ONE fused kernel
(dgl.kernel.typed_block_spmm: gather h[src], block-diagonal transform with
W[type], sum at dst) instead of the reference's edge UDF (gather + bmm into
an E x 500 message tensor) + builtin sum. ``--udf`` runs the reference's
formulation on the same engine for comparison.

FB15k-237 cannot be downloaded here: the triples are synthetic with its
shape (14,541 entities, 237 relations, 272,115 training triples, power-law
entity frequency).

  python examples/rgcn/link_predict.py --gpu 0
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "dgl-1_amd"))
import dgl.function as fn  # noqa: E402
from dgl import DGLGraph, kernel  # noqa: E402


def synthetic_kg(num_entities=14541, num_rels=237, num_triples=272115, seed=0):
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, num_entities + 1) ** 0.8
    p /= p.sum()
    perm = rng.permutation(num_entities)
    s = perm[rng.choice(num_entities, num_triples, p=p)]
    o = perm[rng.choice(num_entities, num_triples, p=p)]
    r = rng.integers(0, num_rels, num_triples)
    return np.stack([s, r, o], 1).astype(np.int64)


def sample_graph(triplets, sample_size, num_rels, rng):
    """Uniform edge sample -> relabelled bidirectional graph + norm + samples."""
    idx = rng.choice(len(triplets), sample_size, replace=False)
    s, r, o = triplets[idx].T
    uniq, inv = np.unique(np.concatenate([s, o]), return_inverse=True)
    s, o = inv[:sample_size], inv[sample_size:]
    n = len(uniq)
    # half of the sampled edges form the graph, all are positive samples
    g_idx = rng.choice(sample_size, sample_size // 2, replace=False)
    src = np.concatenate([s[g_idx], o[g_idx]])
    dst = np.concatenate([o[g_idx], s[g_idx]])
    rel = np.concatenate([r[g_idx], r[g_idx] + num_rels])
    order = np.lexsort((rel, src, dst))  # sorted(zip(dst, src, rel)) as utils.py:116-132
    src, dst, rel = src[order], dst[order], rel[order]
    deg = np.bincount(dst, minlength=n).astype(np.float32)
    norm = np.where(deg > 0, 1.0 / np.maximum(deg, 1), 0).astype(np.float32)
    pos = np.stack([s, r, o], 1)
    neg = pos.copy()
    flip = rng.random(len(neg)) < 0.5
    neg[flip, 0] = rng.integers(0, n, flip.sum())
    neg[~flip, 2] = rng.integers(0, n, (~flip).sum())
    samples = np.concatenate([pos, neg])
    labels = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))]).astype(np.float32)
    return uniq, src, dst, rel, norm, samples, labels


class RGCNBlockLayer(nn.Module):
    def __init__(self, feat, num_rels, num_bases, activation, dropout, udf):
        super(RGCNBlockLayer, self).__init__()
        self.nb, self.si = num_bases, feat // num_bases
        self.weight = nn.Parameter(torch.Tensor(num_rels, num_bases, self.si, self.si))
        nn.init.xavier_uniform_(self.weight, gain=nn.init.calculate_gain("relu"))
        self.loop_weight = nn.Parameter(torch.Tensor(feat, feat))
        nn.init.xavier_uniform_(self.loop_weight, gain=nn.init.calculate_gain("relu"))
        self.activation = activation
        self.dropout = nn.Dropout(dropout) if dropout else None
        self.udf = udf

    def forward(self, g, h, etype, norm):
        loop = h @ self.loop_weight
        if self.dropout is not None:
            loop = self.dropout(loop)
        if self.udf:  # the reference's formulation (layers.py:121-132)
            g.ndata["h"] = h
            g.edata["type"] = etype
            w_all = self.weight

            def msg(edges):
                w = w_all[edges.data["type"]].view(-1, self.si, self.si)
                node = edges.src["h"].view(-1, 1, self.si)
                return {"msg": torch.bmm(node, w).view(-1, self.nb * self.si)}
            g.update_all(msg, fn.sum(msg="msg", out="h"))
            agg = g.ndata.pop("h") * norm.unsqueeze(1)
        else:  # fused typed-edge g-SpMM
            adj = g if isinstance(g, kernel.SparseAdj) else g.sparse_adjacency(h.device)
            # (the 1 / in-degree scale rides in the kernels: the bits of
            # `typed_block_spmm(...) * norm.unsqueeze(1)`)
            agg = kernel.typed_block_spmm(adj, h, self.weight, etype, row_scale=norm)
        out = agg + loop
        return self.activation(out) if self.activation else out


class LinkPredict(nn.Module):
    def __init__(self, num_entities, h_dim, num_rels, num_bases, dropout, reg, udf):
        super(LinkPredict, self).__init__()
        self.emb = nn.Embedding(num_entities, h_dim)
        self.layers = nn.ModuleList([
            RGCNBlockLayer(h_dim, 2 * num_rels, num_bases, F.relu, dropout, udf),
            RGCNBlockLayer(h_dim, 2 * num_rels, num_bases, None, dropout, udf)])
        self.w_relation = nn.Parameter(torch.Tensor(num_rels, h_dim))
        nn.init.xavier_uniform_(self.w_relation, gain=nn.init.calculate_gain("relu"))
        self.reg = reg
        self.udf = udf

    def forward(self, g, node_ids, etype, norm):
        if self.udf:
            h = self.emb(node_ids)
        else:
            # the sample's entities are unique (np.unique), so the lookup's
            # gradient is one row per entity: index_select's backward (a zero
            # fill and a collision-free index_add) gives the bits of
            # nn.Embedding's sort-based backward in 2 launches instead of ~8
            h = self.emb.weight.index_select(0, node_ids)
        for layer in self.layers:
            h = layer(g, h, etype, norm)
        return h

    def loss(self, h, samples, labels):
        # DistMult (the reference's calc_score); the fused model scores the
        # triples in one kernel with deterministic chained gradients
        # (kernel.distmult_score: no [samples, 500] gathers or products)
        if self.udf:
            s = h[samples[:, 0]] * self.w_relation[samples[:, 1]] * h[samples[:, 2]]
            score = s.sum(1)
            reg = h.pow(2).mean() + self.w_relation.pow(2).mean()
            return F.binary_cross_entropy_with_logits(score, labels) + self.reg * reg
        # the same loss as one engine op: scores, BCE and the regulariser in
        # two launches forward, their gradients inside the decoder's
        return kernel.distmult_link_loss(h, self.w_relation, samples[:, 0], samples[:, 1],
                                         samples[:, 2], labels, self.reg)


def select_blas(name):
    """The dense products' BLAS library on ROCm ("rocblas" or "hipblaslt";
    returns the previous one). The step's Linear GEMMs are small (11,816 x
    500 x 500) and the step is host-bound: rocBLAS enqueues one in ≈7 µs
    against hipBLASLt's ≈18 (profiles/r05/host_costs.txt), 0.3 ms per step
    here (tools/rgcn_host_study.py, r06)."""
    old = torch.backends.cuda.preferred_blas_library()
    torch.backends.cuda.preferred_blas_library({"rocblas": "cublas",
                                                "hipblaslt": "cublaslt"}[name])
    return "rocblas" if old == torch._C._BlasBackend.Cublas else "hipblaslt"


def run(args):
    device = torch.device("cpu") if args.gpu < 0 else torch.device("cuda", args.gpu)
    if device.type == "cuda":
        select_blas(args.blas)
    triplets = synthetic_kg(args.num_entities, args.num_rels, args.num_triples, args.seed)
    rng = np.random.default_rng(args.seed)
    torch.manual_seed(args.seed)
    model = LinkPredict(args.num_entities, args.n_hidden, args.num_rels, args.n_bases,
                        args.dropout, args.regularization, args.udf).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr, fused=device.type == "cuda")
    dur, edges = [], 0
    for epoch in range(args.n_epochs):
        uniq, src, dst, rel, norm, samples, labels = sample_graph(
            triplets, args.graph_batch_size, args.num_rels, rng)
        if device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.time()
        g = DGLGraph((torch.from_numpy(src), torch.from_numpy(dst)), multigraph=True)
        if g.number_of_nodes() < len(uniq):
            g.add_nodes(len(uniq) - g.number_of_nodes())
        etype = torch.from_numpy(rel).to(device)
        nrm = torch.from_numpy(norm).to(device)
        h = model(g, torch.from_numpy(uniq).to(device), etype, nrm)
        loss = model.loss(h, torch.from_numpy(samples).to(device),
                          torch.from_numpy(labels).to(device))
        opt.zero_grad()
        loss.backward()
        nn.utils.clip_grad_norm_(model.parameters(), args.grad_norm)
        opt.step()
        if device.type == "cuda":
            torch.cuda.synchronize()
        if epoch >= 2:
            dur.append(time.time() - t0)
        edges = len(src)
    return {"epoch_s": sum(dur) / max(len(dur), 1), "graph_edges": edges,
            "loss": float(loss.item()), "fused": not args.udf}


def parser():
    p = argparse.ArgumentParser(description="R-GCN link prediction on the MI355X engine")
    p.add_argument("--gpu", type=int, default=-1)
    p.add_argument("--udf", action="store_true", help="reference formulation (edge UDF + sum)")
    p.add_argument("--n-hidden", type=int, default=500)
    p.add_argument("--n-bases", type=int, default=100)
    p.add_argument("--dropout", type=float, default=0.2)
    p.add_argument("--lr", type=float, default=1e-2)
    p.add_argument("--regularization", type=float, default=0.01)
    p.add_argument("--grad-norm", type=float, default=1.0)
    p.add_argument("--graph-batch-size", type=int, default=30000)
    p.add_argument("--n-epochs", type=int, default=20)
    p.add_argument("--num-entities", type=int, default=14541)
    p.add_argument("--num-rels", type=int, default=237)
    p.add_argument("--num-triples", type=int, default=272115)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--blas", choices=["rocblas", "hipblaslt"], default="rocblas",
                   help="BLAS library of the dense products (select_blas)")
    return p


if __name__ == "__main__":
    print(run(parser().parse_args()))
