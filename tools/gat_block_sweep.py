"""Interleaved block-size sweep of the source-blocked fused GAT layer on the
Reddit-shaped graph (8 heads x 16): forward (no grad, and with dropout 0.6)
and forward + backward, per block size; outputs checked against the
one-launch kernels bit for bit.

  python tools/gat_block_sweep.py [--block-mb 6 7.5 9 11] [--rounds 5]
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
    ap.add_argument("--block-mb", type=float, nargs="+", default=[6, 7.5, 9, 11, 14])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    ft = torch.rand(n, 8, 16, device=dev) * 2 - 1
    el = torch.rand(n, 8, device=dev) - 0.5
    er = torch.rand(n, 8, device=dev) - 0.5
    old = kernel.set_blocked("off")
    with torch.no_grad():
        ref = kernel.gat_aggregate(adj, ft, el, er)
    kernel.set_blocked(old)
    sizes = [0] + [int(mb * (1 << 20)) for mb in args.block_mb]
    times = {s: {"fwd": [], "fwd_drop": []} for s in sizes}
    for _ in range(args.rounds):
        for s in sizes:
            pol = kernel.set_blocked("off" if s == 0 else "auto")
            if s:
                kernel._GAT_BLOCK_BYTES = s
            with torch.no_grad():
                out = kernel.gat_aggregate(adj, ft, el, er)
                assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]), s
                for key, p in (("fwd", 0.0), ("fwd_drop", 0.6)):
                    kernel.gat_aggregate(adj, ft, el, er, attn_drop=p)
                    torch.cuda.synchronize()
                    kernel.timing_enable(True)
                    for _ in range(args.iters):
                        kernel.gat_aggregate(adj, ft, el, er, attn_drop=p)
                    ms, cnt = kernel.timing_read()
                    kernel.timing_enable(False)
                    times[s][key].append(ms / args.iters)
            kernel.set_blocked(pol)
    res = []
    for s, t in times.items():
        e = {"block_mb": s / (1 << 20) if s else "one launch"}
        for k, v in t.items():
            v = sorted(v)
            e[k + "_ms"] = round(v[len(v) // 2], 3)
        res.append(e)
    print(json.dumps({"graph": "reddit_like", "heads": 8, "head_dim": 16, "sizes": res},
                     indent=1))


if __name__ == "__main__":
    main()
