"""A/B of the running-row cache policy of the headline's blocked launches
(dglhip_set_row_policy): per policy, the mean GPU span of a
copy_u + sum call on the Reddit-shaped graph (events around the call on the
launch stream), interleaved over rounds, and the output bits against policy
0.

  python tools/rowpol_ab.py [--calls 20 --rounds 3] [--out file.json]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def block_sweep(adj, h, ref, args):
    """ms per call at 5 / 6 / 7 / 8 / 9 MiB source blocks under row policies 0, 2 and
    4 (interleaved), and whether each keeps the bits."""
    old_bytes = kernel.schedule_policy()["block_bytes"]
    res, same = {}, {}
    try:
        for _ in range(args.rounds):
            for mib in (5, 6, 7, 8, 9):
                kernel.set_schedule_policy(block_bytes=mib << 20)
                for p in (0, 2, 4):
                    kernel.check_call(kernel.LIB.dglhip_set_row_policy(p))
                    o = kernel.gspmm(adj, "copy_u", "sum", h)
                    torch.cuda.synchronize()
                    key = "%d MiB / policy %d (%d launches)" % (
                        mib, p, kernel.blocked_schedule(adj, h))
                    same[key] = bool(torch.equal(o, ref))
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
                        enable_timing=True)
                    s.record()
                    for _ in range(args.calls):
                        kernel.gspmm(adj, "copy_u", "sum", h)
                    e.record()
                    e.synchronize()
                    res.setdefault(key, []).append(s.elapsed_time(e) / args.calls)
    finally:
        kernel.set_schedule_policy(block_bytes=old_bytes)
        kernel.check_call(kernel.LIB.dglhip_set_row_policy(0))
    return {"ms_per_call": res, "min": {k: min(v) for k, v in res.items()},
            "bit_identical": same}


def gat_ab(adj, n, dev, args):
    """The GAT layer 8 x 16 on the same graph: forward (training) and forward +
    backward wall ms per policy 0 / 2 / 4, outputs and gradients vs policy 0."""
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
        r = (fs.detach(), z.detach(), ft.grad, el.grad, er.grad)
        ft.grad = el.grad = er.grad = None
        return r

    def wall(fn, iters):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / iters
    ref = fb()
    res = {"fwd": {}, "fwd_bwd": {}, "same": {}}
    for _ in range(args.rounds):
        for p in (0, 2, 4):
            kernel.check_call(kernel.LIB.dglhip_set_row_policy(p))
            got = fb()
            res["same"][p] = all(bool(torch.equal(a, b)) for a, b in zip(got, ref))
            res["fwd"].setdefault(p, []).append(
                wall(lambda: kernel.gat_aggregate(adj, ft, el, er), 10))
            res["fwd_bwd"].setdefault(p, []).append(wall(fb, 10))
    kernel.check_call(kernel.LIB.dglhip_set_row_policy(0))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--gat", action="store_true")
    ap.add_argument("--sweep", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(scale=1, seed=0, device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev) * 2 - 1
    ref = kernel.gspmm(adj, "copy_u", "sum", h)
    res = {p: [] for p in range(5)}
    same = {}
    for _ in range(args.rounds):
        for p in range(5):
            kernel.check_call(kernel.LIB.dglhip_set_row_policy(p))
            out = kernel.gspmm(adj, "copy_u", "sum", h)
            torch.cuda.synchronize()
            same[p] = bool(torch.equal(out, ref))
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.calls):
                kernel.gspmm(adj, "copy_u", "sum", h)
            e.record()
            e.synchronize()
            res[p].append(s.elapsed_time(e) / args.calls)
    kernel.check_call(kernel.LIB.dglhip_set_row_policy(0))
    out = {"ms_per_call": res, "min": {p: min(v) for p, v in res.items()},
           "bit_identical": same, "launches": kernel.blocked_schedule(adj, h)}
    if args.sweep:
        out["block_sweep"] = block_sweep(adj, h, ref, args)
    if args.gat:
        out["gat"] = gat_ab(adj, n, dev, args)
    line = json.dumps(out)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
