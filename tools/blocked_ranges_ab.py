"""Interleaved A/B of the source-blocked schedule (items) against one launch
on the bench graph: copy_u + sum, u_mul_e + sum with weights by edge id and
in slot order; bits checked. (The r03 record's earlier columns, segment CSRs
and row ranges, came from the forms this replaced.)

  python tools/blocked_ranges_ab.py [--rounds 7] [--iters 5]
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev) * 2 - 1
    w = torch.rand(adj.fwd.nnz, device=dev)
    cases = [("copy_u", None, "eid"), ("u_mul_e", w, "eid"), ("u_mul_e", w, "slot")]
    pols = ["off", "auto"]
    refs = {}
    times = {(c, p): [] for c in range(len(cases)) for p in pols}
    for _ in range(args.rounds):
        for ci, (msg, e, order) in enumerate(cases):
            for p in pols:
                old = kernel.set_blocked(p)
                out = kernel.gspmm(adj, msg, "sum", h, e, edge_order=order)
                if ci not in refs:
                    refs[ci] = out
                assert torch.equal(out, refs[ci]), (msg, order, p)
                kernel.timing_enable(True)
                for _ in range(args.iters):
                    kernel.gspmm(adj, msg, "sum", h, e, edge_order=order)
                ms, cnt = kernel.timing_read()
                kernel.timing_enable(False)
                # wall time too: the blocked u_mul_e's edge-value gather is a torch op
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                for _ in range(args.iters):
                    kernel.gspmm(adj, msg, "sum", h, e, edge_order=order)
                t1.record()
                torch.cuda.synchronize()
                kernel.set_blocked(old)
                times[(ci, p)].append((ms / args.iters, cnt // args.iters,
                                       t0.elapsed_time(t1) / args.iters))
    res = []
    for (ci, p), t in times.items():
        if not t:
            continue
        ms = sorted(x[0] for x in t)
        wall = sorted(x[2] for x in t)
        res.append({"msg": cases[ci][0], "edge_order": cases[ci][2], "policy": p,
                    "launches": t[0][1], "median_ms": round(ms[len(ms) // 2], 3),
                    "median_wall_ms": round(wall[len(wall) // 2], 3)})
    print(json.dumps({"graph": "reddit_like", "feat": 128, "cases": res}, indent=1))


if __name__ == "__main__":
    main()
