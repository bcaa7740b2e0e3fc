"""GraphSAGE (mean aggregator), full-graph, single GPU or node-partitioned over
the GPUs of one node (BASELINE.json configs[3]).

The reference has no GraphSAGE example; this driver exercises the engine's
``mean`` reducer (g-SpMM copy_u + mean) and the multi-GPU path of
dgl.distributed:

* single device: ``g.update_all(fn.copy_src('h','m'), fn.mean('m','neigh'))``;
* ``--dist``: one process per GPU (torchrun), dst rows 1-D partitioned;
  each layer exchanges the feature halo over RCCL (all-gather or
  all-to-allv, dgl.distributed) in ``--pipeline-chunks`` chunks overlapped
  with the local g-SpMM segments, forward and backward (the reverse exchange
  of each chunk's gradient rows runs while the next chunk's transposed
  product does); dense-layer gradients are all-reduced by DDP.

Layer: h' = act(fc_self(h) + fc_neigh(mean_{u->v} h_u)). fc_neigh has no bias,
so it commutes with the mean: when it narrows the features (602 -> 128 on
Reddit) it is applied before the aggregation, which then moves 4.7x fewer
bytes through the g-SpMM (same result up to fp32 rounding).

  python examples/graphsage/train.py --dataset reddit --gpu 0
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/graphsage/train.py --dist \\
      --graph rmat --rmat-scale 24
"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "dgl-1_amd"))
import dgl.function as fn  # noqa: E402
from dgl import DGLGraph, data, kernel  # noqa: E402
from dgl.distributed import PartitionedGraph, balanced_bounds  # noqa: E402
from dgl.nn.pytorch import NodeLinear, sage_dense, weighted_cross_entropy  # noqa: E402


class SAGELayer(nn.Module):
    def __init__(self, in_feats, out_feats, activation):
        super(SAGELayer, self).__init__()
        # NodeLinear: nn.Linear with MFMA-shaped backward reductions over the
        # node dimension (dgl/nn/pytorch/linear.py)
        self.fc_self = NodeLinear(in_feats, out_feats)
        self.fc_neigh = NodeLinear(in_feats, out_feats, bias=False)
        self.activation = activation

    def forward(self, h, aggregate):
        # fc_self(h) + fc_neigh(aggregate(h)), the narrower side aggregated,
        # both products and their sum fused (dgl.nn.pytorch.sage_dense)
        # the activation fused into the dense step where it can be (ReLU)
        return sage_dense(h, aggregate, self.fc_self, self.fc_neigh, self.activation)


class SAGE(nn.Module):
    def __init__(self, in_feats, n_hidden, n_classes, n_layers, dropout):
        super(SAGE, self).__init__()
        dims = [in_feats] + [n_hidden] * n_layers + [n_classes]
        self.layers = nn.ModuleList([
            SAGELayer(dims[i], dims[i + 1], F.relu if i < n_layers else None)
            for i in range(len(dims) - 1)])
        self.dropout = nn.Dropout(dropout) if dropout else None

    def forward(self, h, aggregate):
        for i, layer in enumerate(self.layers):
            if self.dropout is not None and i > 0:
                h = self.dropout(h)
            h = layer(h, aggregate)
        return h


def graph_and_data(args, device):
    if args.graph == "rmat":
        src, dst, n = data.rmat(args.rmat_scale, 16, seed=args.seed, device=device)
        gen = torch.Generator(device=device)
        gen.manual_seed(args.seed + 1)
        feats = 0.1 * torch.randn(n, args.in_feats, generator=gen, device=device)
        labels = torch.randint(0, args.n_classes, (n,), generator=gen, device=device)
        train = torch.rand(n, generator=gen, device=device) < 0.5
        return src, dst, n, feats, labels, train, args.n_classes
    ds = data.load_data(args.dataset, seed=args.seed, device=device)
    src, dst = ds.graph
    return src, dst, ds.num_nodes, ds.features, ds.labels, ds.train_mask, ds.num_labels


def run(args):
    distributed = args.dist
    if distributed:
        if not dist.is_initialized():
            backend = args.dist_backend or ("nccl" if torch.cuda.is_available() else "gloo")
            dist.init_process_group(backend)
        rank, world = dist.get_rank(), dist.get_world_size()
        if torch.cuda.is_available() and args.gpu >= 0:
            local = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
            device = torch.device("cuda", local)
            torch.cuda.set_device(device)
        else:
            device = torch.device("cpu")
    else:
        rank, world = 0, 1
        device = torch.device("cpu") if args.gpu < 0 else torch.device("cuda", args.gpu)

    src, dst, n, feats, labels, train, ncls = graph_and_data(args, device)
    n_train_global = int(train.sum())
    if distributed:
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        sel = (dst >= lo) & (dst < hi)
        pg = PartitionedGraph(n, src[sel], dst[sel], bounds, device,
                              pipeline_chunks=args.pipeline_chunks)
        feats, labels, train = feats[lo:hi], labels[lo:hi], train[lo:hi]

        def aggregate(h):
            return pg.update_all(h, "copy_u", "mean")
        aggregate.add_into = pg.mean_add  # out + mean(h) without a sum pass
        num_edges = int(src.numel())
    else:
        g = DGLGraph((src.cpu(), dst.cpu()))
        num_edges = g.number_of_edges()

        def aggregate(h):
            g.ndata["h"] = h
            g.update_all(fn.copy_src("h", "m"), fn.mean("m", "neigh"))
            return g.ndata.pop("neigh")
        # out + mean(h) in the aggregation's store (sage_dense's narrowing
        # layer adds fc_self(h) there; the same bits as the sum of the two)
        aggregate.add_into = lambda h, out: kernel.gspmm_mean_add(
            g.sparse_adjacency(h.device), h, out)
    del src, dst
    if args.row_split is not None:
        kernel.set_row_split(args.row_split)

    torch.manual_seed(args.seed)
    model = SAGE(feats.shape[1], args.n_hidden, ncls, args.n_layers, args.dropout).to(device)
    if distributed:
        model = nn.parallel.DistributedDataParallel(
            model, device_ids=[device.index] if device.type == "cuda" else None)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    train_w = train.to(torch.float32)
    dur, losses = [], []
    for epoch in range(args.n_epochs):
        model.train()
        if device.type == "cuda":
            torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        t0 = time.time()
        logits = model(feats, aggregate)
        # sum over local training nodes / global count: DDP's gradient average
        # times world size equals the single-process mean-loss gradient. The
        # per-row losses of every node, masked: at 10^7-10^8 nodes the
        # reducing nll_loss kernel runs as one workgroup (RMAT-26: 118 ms of a
        # 616 ms epoch), and logits[train] adds a gather and its scatter
        # backward. weighted_cross_entropy is
        # (F.cross_entropy(logits, labels, reduction="none") * train_w).sum()
        # as one pass over the logits forward and one backward
        loss = weighted_cross_entropy(logits, labels, train_w) * (world / max(n_train_global, 1))
        opt.zero_grad()
        loss.backward()
        opt.step()
        if device.type == "cuda":
            torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        if epoch >= min(3, args.n_epochs - 1):
            dur.append(time.time() - t0)
        losses.append(float(loss.item()))
    mean = sum(dur) / len(dur)
    state = {k: v.detach().cpu() for k, v in
             (model.module if distributed else model).state_dict().items()}
    return {"graph": args.graph if args.graph == "rmat" else args.dataset, "world": world,
            "epoch_s": mean, "edges": num_edges, "row_split": kernel.get_row_split(),
            "edges_per_s": num_edges * (args.n_layers + 1) / mean, "loss": losses[-1],
            "state": state}


def parser():
    p = argparse.ArgumentParser(description="GraphSAGE-mean on the MI355X engine")
    p.add_argument("--graph", default="dataset", choices=["dataset", "rmat"])
    p.add_argument("--dataset", default="reddit")
    p.add_argument("--rmat-scale", type=int, default=20)
    p.add_argument("--in-feats", type=int, default=128)
    p.add_argument("--n-classes", type=int, default=41)
    p.add_argument("--gpu", type=int, default=0)
    p.add_argument("--dist", action="store_true")
    p.add_argument("--dist-backend", default=None)
    p.add_argument("--pipeline-chunks", type=int, default=4,
                   help="--dist: halo exchange cut into this many chunks, overlapped with "
                        "the local g-SpMM segments in the forward and backward (0: one "
                        "exchange, then the kernel; bit-identical rows)")
    p.add_argument("--n-hidden", type=int, default=128)
    p.add_argument("--n-layers", type=int, default=1)
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--lr", type=float, default=1e-2)
    p.add_argument("--n-epochs", type=int, default=10)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--row-split", default=None,
                   help="heavy-row policy of the g-SpMM (off / auto / a chunk length; "
                        "default: the library's, dgl.kernel.set_row_split)")
    return p


if __name__ == "__main__":
    res = run(parser().parse_args())
    res.pop("state")
    if res["world"] == 1 or dist.get_rank() == 0:
        print(res)
    if dist.is_initialized():
        dist.destroy_process_group()
