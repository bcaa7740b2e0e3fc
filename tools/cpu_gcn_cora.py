"""configs[0] on the host: the 2-layer GCN on Cora (2,708 nodes, 13,264 edges
with self-loops, hidden 16), one training epoch (forward + backward + Adam),
through the engine's host g-SpMM (examples/gcn/gcn_spmv.py's model on
DGLGraph.update_all) and through the reference's CPU arithmetic
(torch.sparse.mm on the uncoalesced COO, python/dgl/backend/pytorch/
tensor.py:145-146), same data, same threads.

  python tools/cpu_gcn_cora.py [--epochs 200]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dgl-1_amd"))
import dgl  # noqa: E402
import dgl.function as fn  # noqa: E402
from dgl import data  # noqa: E402


class GCN(nn.Module):
    def __init__(self, fin, hid, ncls, spmm):
        super().__init__()
        self.l1, self.l2 = nn.Linear(fin, hid), nn.Linear(hid, ncls)
        self.spmm = spmm

    def forward(self, x, norm):
        h = F.relu(self.spmm(self.l1(x) * norm) * norm)
        return self.spmm(self.l2(h) * norm) * norm


def run(spmm, ds, norm, epochs):
    torch.manual_seed(0)
    model = GCN(ds.features.shape[1], 16, ds.num_labels, spmm)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    mask = ds.train_mask
    times = []
    for e in range(epochs):
        t0 = time.perf_counter()
        loss = F.cross_entropy(model(ds.features, norm)[mask], ds.labels[mask])
        opt.zero_grad()
        loss.backward()
        opt.step()
        if e >= 10:
            times.append(time.perf_counter() - t0)
    return sum(times) / len(times), float(loss.detach())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=200)
    a = ap.parse_args()
    ds = data.load_data("cora", seed=0, device="cpu")
    src, dst = ds.graph
    n = ds.num_nodes
    loops = torch.arange(n)
    src, dst = torch.cat([src, loops]), torch.cat([dst, loops])
    g = dgl.DGLGraph((src, dst))
    deg = torch.bincount(dst, minlength=n).float().clamp(min=1)
    norm = deg.pow(-0.5).unsqueeze(1)

    def engine(h):
        g.ndata["h"] = h
        g.update_all(fn.copy_src("h", "m"), fn.sum("m", "h"))
        return g.ndata.pop("h")

    A = torch.sparse_coo_tensor(torch.stack([dst, src]), torch.ones(src.numel()), (n, n))

    def reference(h):
        return torch.sparse.mm(A, h)

    res = {"graph": "cora-shaped", "nodes": n, "edges": int(src.numel()),
           "threads": torch.get_num_threads(), "cpus": os.cpu_count()}
    for name, fn_ in (("engine_host_gspmm", engine), ("reference_torch_sparse_mm", reference)):
        t, loss = run(fn_, ds, norm, a.epochs)
        res[name] = {"epoch_ms": t * 1e3, "final_loss": loss}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
