"""The one-pass GAT backward with er and dz packed into one [rows, 2H] table
(one cache line per slot for the pair's destination operands) against two
tables: Reddit-shaped graph, 8 heads x 16, forward + backward wall ms per
call, interleaved rounds, every gradient compared bit for bit.

  python tools/gat_pack_ab.py [--rounds 3] [--iters 10] [--out file.json]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(scale=1, seed=0, device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    ft = (torch.rand(n, 8, 16, generator=gen, device=dev) * 2 - 1).requires_grad_(True)
    el = (torch.rand(n, 8, generator=gen, device=dev) - 0.5).requires_grad_(True)
    er = (torch.rand(n, 8, generator=gen, device=dev) - 0.5).requires_grad_(True)
    gout = torch.rand(n, 8, 16, generator=gen, device=dev)
    gz = torch.rand(n, 8, 1, generator=gen, device=dev)

    def fb():
        fs, z = kernel.gat_aggregate(adj, ft, el, er, seed=7)
        torch.autograd.backward([fs, z], [gout, gz])
        r = (ft.grad, el.grad, er.grad)
        ft.grad = el.grad = er.grad = None
        return r

    def wall():
        fb()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            fb()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / args.iters

    kernel.set_gat_bwd_pack(False)
    ref = fb()
    res = {"packed": [], "two_tables": []}
    same = True
    for _ in range(args.rounds):
        for name, on in (("two_tables", False), ("packed", True)):
            kernel.set_gat_bwd_pack(on)
            got = fb()
            same = same and all(bool(torch.equal(a, b)) for a, b in zip(got, ref))
            res[name].append(wall())
    kernel.set_gat_bwd_pack(True)
    out = {"fwd_bwd_ms": res, "min": {k: min(v) for k, v in res.items()},
           "bit_identical": same, "graph": "reddit_like", "heads": 8, "head_dim": 16}
    print(json.dumps(out))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
