"""Host-side audit of a GraphSAGE training epoch on one GPU (RMAT graph,
SCALE env, default 20): after warm-up, one epoch runs under
torch.cuda.set_sync_debug_mode("warn") and prints every distinct call stack
that synchronises with the device; three more epochs run under cProfile with
the forward's host time printed. A forward that issues its kernels without
blocking shows well under a millisecond of host time.

    SCALE=26 python tools/sync_hunt.py
"""
import os, sys, time, runpy, traceback, warnings, cProfile, pstats
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dgl-1_amd"))
sys.argv = ["x"]
mod = runpy.run_path(os.path.join(ROOT, "examples", "graphsage", "train.py"), run_name="sage")
import torch.nn.functional as F
from dgl import DGLGraph, data
import dgl.function as fn
dev = torch.device("cuda", 0)
src, dst, n = data.rmat(int(os.environ.get("SCALE", "20")), 16, seed=0, device=dev)
g = DGLGraph((src.cpu(), dst.cpu()))
if g.number_of_nodes() < n:
    g.add_nodes(n - g.number_of_nodes())
del src, dst
gen = torch.Generator(device=dev); gen.manual_seed(1)
feats = 0.1 * torch.randn(n, 128, generator=gen, device=dev)
labels = torch.randint(0, 41, (n,), generator=gen, device=dev)
train_w = (torch.rand(n, generator=gen, device=dev) < 0.5).float()
def aggregate(h):
    g.ndata["h"] = h
    g.update_all(fn.copy_src("h", "m"), fn.mean("m", "neigh"))
    return g.ndata.pop("neigh")
model = mod["SAGE"](128, 128, 41, 1, 0.0).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-2)
def epoch():
    logits = model(feats, aggregate)
    loss = (F.cross_entropy(logits, labels, reduction="none") * train_w).sum()
    opt.zero_grad(); loss.backward(); opt.step()
for _ in range(3):
    epoch()
torch.cuda.synchronize()
seen = set()
def show(message, category, filename, lineno, file=None, line=None):
    st = "".join(traceback.format_stack()[:-2][-8:])
    if st not in seen:
        seen.add(st)
        print("SYNC:", message, "\n", st, flush=True)
warnings.showwarning = show
warnings.simplefilter("always")
torch.cuda.set_sync_debug_mode("warn")
epoch()
torch.cuda.set_sync_debug_mode(0)
torch.cuda.synchronize()
print("distinct sync stacks:", len(seen), flush=True)
pr = cProfile.Profile()
torch.cuda.synchronize(); t0 = time.perf_counter()
pr.enable()
for _ in range(3):
    t1 = time.perf_counter(); logits = model(feats, aggregate); t2 = time.perf_counter()
    print("fwd host %.1f ms" % ((t2 - t1) * 1e3), flush=True)
    loss = (F.cross_entropy(logits, labels, reduction="none") * train_w).sum()
    opt.zero_grad(); loss.backward(); opt.step()
pr.disable()
torch.cuda.synchronize()
print("3 epochs %.1f ms" % ((time.perf_counter() - t0) * 1e3))
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
