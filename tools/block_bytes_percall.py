"""Source-block size of the blocked schedule re-swept with per-call timing
(kernel.timing_enable(per_call=True): two events per call, none between the
launches), on the Reddit-shaped graph (copy_u + sum, F = 128): the earlier
sweeps bracketed every launch, which charged schedules with more launches
for their markers. Bits compared with the one-launch kernel.

  python tools/block_bytes_percall.py [--mib 3 4 5 6 8] [--rounds 3] [--iters 20]
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
    ap.add_argument("--mib", type=float, nargs="+", default=[3, 4, 5, 6, 8])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    csr = adj.fwd
    h = torch.rand(n, 128, device=dev) * 2 - 1
    out = torch.empty(n, 128, device=dev)
    old = kernel.set_blocked("off")
    kernel.gspmm_into(csr, out, h)
    ref = out.clone()
    kernel.set_blocked(old)
    res = {"graph": "reddit_like", "rounds": []}
    for _ in range(args.rounds):
        row = {}
        for mib in args.mib:
            kernel.set_schedule_policy(block_bytes=int(mib * (1 << 20)))
            kernel.gspmm_into(csr, out, h)
            torch.cuda.synchronize()
            same = bool(torch.equal(out, ref))
            kernel.timing_enable(True, per_call=True)
            for _ in range(args.iters):
                kernel.gspmm_into(csr, out, h)
            ms, calls = kernel.timing_read()
            kernel.timing_enable(False)
            row["%g" % mib] = {"ms": ms / calls, "blocks": kernel.blocked_schedule(adj, h),
                               "bits_equal": same}
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
