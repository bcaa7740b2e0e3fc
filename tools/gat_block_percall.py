"""The fused GAT layer's source-block size (kernel._GAT_BLOCK_BYTES) re-swept
by wall time between two events per call (no marker between the launches), on
the Reddit-shaped graph at 8 heads x 16: forward without and with the
attention stored, forward + backward; bits compared with the 11 MiB default.

  python tools/gat_block_percall.py [--mib 7 9 11 13] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def wall(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, nargs="+", default=[7, 9, 11, 13])
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    H, D = 8, 16
    g = torch.Generator(device=dev).manual_seed(3)
    ft = (torch.rand(n, H, D, device=dev, generator=g) * 2 - 1).requires_grad_(True)
    el = (torch.rand(n, H, device=dev, generator=g) - 0.5).requires_grad_(True)
    er = (torch.rand(n, H, device=dev, generator=g) - 0.5).requires_grad_(True)
    gout = torch.rand(n, H, D, device=dev, generator=g)
    gz = torch.rand(n, H, 1, device=dev, generator=g)

    def fwd_ng():
        with torch.no_grad():
            return kernel.gat_aggregate(adj, ft, el, er)

    def fwd_g():
        return kernel.gat_aggregate(adj, ft, el, er)

    def fb():
        fs, z = kernel.gat_aggregate(adj, ft, el, er)
        torch.autograd.backward([fs, z], [gout, gz])

    kernel._GAT_BLOCK_BYTES = kernel._GAT_BLOCK_BYTES_NOGRAD = 11 << 20
    ref = [t.detach().clone() for t in fwd_ng()]
    res = {"graph": "reddit_like", "rows": []}
    for mib in args.mib:
        kernel._GAT_BLOCK_BYTES = kernel._GAT_BLOCK_BYTES_NOGRAD = int(mib * (1 << 20))
        same = all(torch.equal(a, b) for a, b in zip(fwd_ng(), ref))
        row = {"block_MiB": mib, "fwd_ms": wall(fwd_ng, args.iters),
               "fwd_stored_ms": wall(fwd_g, args.iters), "fwd_bwd_ms": wall(fb, args.iters),
               "bits_equal": same}
        res["rows"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
