"""Operator-level profile of one GraphSAGE training epoch on one GPU (RMAT
graph, SCALE env, default 22): torch.profiler with shapes and Python stacks,
so that every PyTorch-side pass (copies, element-wise kernels, reductions)
is traced back to the line of the engine or the model that issued it.

    SCALE=22 python tools/sage_op_profile.py
"""
import os
import runpy
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dgl-1_amd"))
sys.argv = ["x"]
mod = runpy.run_path(os.path.join(ROOT, "examples", "graphsage", "train.py"), run_name="sage")
from dgl import DGLGraph, data  # noqa: E402
import dgl.function as fn  # noqa: E402

dev = torch.device("cuda", 0)
src, dst, n = data.rmat(int(os.environ.get("SCALE", "22")), 16, seed=0, device=dev)
g = DGLGraph((src.cpu(), dst.cpu()))
if g.number_of_nodes() < n:
    g.add_nodes(n - g.number_of_nodes())
del src, dst
gen = torch.Generator(device=dev)
gen.manual_seed(1)
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
    loss = (F.cross_entropy(logits, labels, reduction="none") * train_w).sum() / n
    opt.zero_grad()
    loss.backward()
    opt.step()


for _ in range(3):
    epoch()
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
    epoch()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(
    sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=40,
    max_shapes_column_width=60))
# every large PyTorch-side op with the model / engine line that issued it
for e in prof.events():
    if not e.name.startswith("aten::") or e.device_type != torch.autograd.DeviceType.CPU:
        continue
    big = [sh for sh in e.input_shapes if sh and len(sh) >= 2 and sh[0] * sh[-1] >= (1 << 22)]
    if not big or e.name in ("aten::empty", "aten::view", "aten::slice", "aten::as_strided",
                             "aten::detach", "aten::reshape", "aten::t", "aten::transpose",
                             "aten::expand", "aten::select", "aten::alias", "aten::_unsafe_view",
                             "aten::empty_strided", "aten::resize_"):
        continue
    where = [f for f in e.stack if "dgl-1_amd" in f or "examples" in f or "tools" in f][:3]
    print("%-34s %-44s %s" % (e.name, e.input_shapes[:2], " <- ".join(where)))
