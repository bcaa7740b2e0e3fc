"""u_mul_e + sum with a scalar edge weight on the Reddit-shaped graph, for
three edge-id orders of the same graph: "src" (the generator's (src, dst)
order: a row's edge ids increase but are far apart), "shuffled" (arbitrary ids,
as after add_edges in random order) and "dst" (ids already in CSR slot order,
eid == arange: the CSR's slot_eid is None and the kernel skips the
indirection). copy_u + sum on the same CSR is the no-edge-feature floor.

  python tools/eid_study.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def time_ms(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda", 0)
    src0, dst0, n = data.reddit_like(device=dev)
    E = int(src0.numel())
    F = 128
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    h = torch.rand(n, F, generator=gen, device=dev) * 2 - 1
    w0 = torch.rand(E, generator=gen, device=dev)
    res = {}
    for order in ("src", "shuffled", "dst"):
        if order == "src":
            perm = torch.arange(E, device=dev)
        elif order == "shuffled":
            perm = torch.randperm(E, generator=gen, device=dev)
        else:
            perm = torch.argsort(dst0 * n + src0, stable=True)
        src, dst, w = src0[perm], dst0[perm], w0[perm]
        adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
        del src, dst, perm
        row = {"eid_is_identity": adj.fwd.slot_eid is None}
        row["u_mul_e_sum"] = time_ms(lambda: kernel.gspmm(adj, "u_mul_e", "sum", h, w))
        row["copy_u_sum"] = time_ms(lambda: kernel.gspmm(adj, "copy_u", "sum", h))
        res[order] = row
        del adj
    print(json.dumps({"edges": E, "feat": F, "ms": res}, indent=1))


if __name__ == "__main__":
    main()
