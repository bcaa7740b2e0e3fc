"""copy_u + sum across feature widths on the Reddit-shaped graph: one launch
vs the source-blocked schedule (default gate, and with the table floor at
4 MiB so narrow tables block too), interleaved in rounds, bits checked.

  python tools/blocked_width_sweep.py [--feats 16 32 41 64 128 256] [--rounds 5]
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
    ap.add_argument("--feats", type=int, nargs="+", default=[16, 32, 41, 64, 128, 256])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    default_min = kernel.schedule_policy()["block_table_min"]
    configs = [("one launch", "off", default_min), ("blocked", "auto", default_min),
               ("blocked, 4 MiB floor", "auto", 4 << 20)]
    res = []
    for F in args.feats:
        h = torch.rand(n, F, device=dev) * 2 - 1
        old = kernel.set_blocked("off")
        ref = kernel.gspmm(adj, "copy_u", "sum", h)
        kernel.set_blocked(old)
        times = {c[0]: [] for c in configs}
        launches = {}
        for _ in range(args.rounds):
            for name, pol, tmin in configs:
                old = kernel.set_blocked(pol)
                kernel.set_schedule_policy(block_table_min=tmin)
                out = kernel.gspmm(adj, "copy_u", "sum", h)
                assert torch.equal(out, ref), (F, name)
                kernel.timing_enable(True)
                for _ in range(args.iters):
                    kernel.gspmm(adj, "copy_u", "sum", h)
                ms, cnt = kernel.timing_read()
                kernel.timing_enable(False)
                kernel.set_blocked(old)
                kernel.set_schedule_policy(block_table_min=default_min)
                times[name].append(ms / args.iters)
                launches[name] = cnt // args.iters
        e = {"feat": F, "table_MB": n * F * 4 / 1e6}
        for name, t in times.items():
            t = sorted(t)
            e[name] = {"ms": round(t[len(t) // 2], 3), "launches": launches[name]}
        res.append(e)
        print(json.dumps(e), flush=True)
        del h, ref
    print(json.dumps({"graph": "reddit_like", "widths": res}))


if __name__ == "__main__":
    main()
