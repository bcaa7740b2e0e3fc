"""Source-block size of the one-pass GAT backward over the transpose
(kernel._GAT_BWD_BLOCK_BYTES), Reddit-shaped graph, 8 heads x 16: forward +
backward wall ms per size, interleaved over rounds, gradients vs the default.

  python tools/gat_bwd_sweep.py [--rounds 3] [--out file.json]
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
    ap.add_argument("--mib", type=int, nargs="+", default=[4, 6, 8, 11, 14, 18])
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
        fs, z = kernel.gat_aggregate(adj, ft, el, er)
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
    default = kernel._GAT_BWD_BLOCK_BYTES
    ref = fb()
    res, same, launches = {}, {}, {}
    try:
        for _ in range(args.rounds):
            for mib in args.mib:
                kernel._GAT_BWD_BLOCK_BYTES = mib << 20
                got = fb()
                same[mib] = all(bool(torch.equal(a, b)) for a, b in zip(got, ref))
                plan = kernel._block_plan(adj.bwd, gout.view(n, 128), 128, mib << 20)
                launches[mib] = 0 if plan is None else len(plan)
                res.setdefault(mib, []).append(wall())
    finally:
        kernel._GAT_BWD_BLOCK_BYTES = default
    line = json.dumps({"fwd_bwd_ms": res, "min": {k: min(v) for k, v in res.items()},
                       "launches": launches, "bit_identical": same})
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
