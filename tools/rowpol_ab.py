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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
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
    line = json.dumps({"ms_per_call": res, "min": {p: min(v) for p, v in res.items()},
                       "bit_identical": same, "launches": kernel.blocked_schedule(adj, h)})
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
