"""Interleaved sweep of the source-blocked g-SpMM's launch knobs on the bench
graph (copy_u + sum, F = 128): kernel variant (vec, lanes per row, gathers
per batch, pipelined) x gather mode (64-bit addresses / buffer descriptors)
x short-row tiers (on / off) x block bytes. Every configuration is checked
bit-identical to the one-launch result.

  python tools/blocked_kernel_sweep.py [--rounds 3] [--iters 5] [--block-mb 7.5 5 3]
                                      [--default-variant-only]
"""
import argparse
import itertools
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402

VARIANTS = [(0, 0, 0, 0), (2, 64, 8, 0), (2, 64, 32, 0), (2, 64, 16, 1), (4, 32, 16, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--block-mb", type=float, nargs="+", default=[7.5, 5.0, 3.0],
                    help="block bytes (MiB) to sweep")
    ap.add_argument("--default-variant-only", action="store_true",
                    help="default kernel variant, gather mode and tiers: block bytes only")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev) * 2 - 1
    old = kernel.set_blocked("off")
    ref = kernel.gspmm(adj, "copy_u", "sum", h)
    kernel.set_blocked(old)
    sizes = [int(mb * (1 << 20)) for mb in args.block_mb]
    if args.default_variant_only:
        configs = [(VARIANTS[0], 0, True, bb) for bb in sizes]
    else:
        configs = list(itertools.product(VARIANTS, (0, 1), (True, False), sizes))
    times = {c: [] for c in configs}
    for _ in range(args.rounds):
        for c in configs:
            v, gm, short, bb = c
            _ffi.check_call(_ffi.LIB.dglhip_set_spmm_variant(*v))
            kernel.set_gather_mode(gm)
            kernel.set_short_rows(short)
            kernel.set_schedule_policy(block_bytes=bb)
            out = kernel.gspmm(adj, "copy_u", "sum", h)
            assert torch.equal(out, ref), c
            kernel.timing_enable(True)
            for _ in range(args.iters):
                kernel.gspmm(adj, "copy_u", "sum", h)
            ms, cnt = kernel.timing_read()
            kernel.timing_enable(False)
            times[c].append((ms / args.iters, cnt // args.iters))
    res = []
    for c, t in times.items():
        ms = sorted(x[0] for x in t)
        res.append({"variant": "%d,%d,%d,%d" % c[0], "gather_mode": c[1], "short_rows": c[2],
                    "block_bytes": c[3], "launches": t[0][1], "median_ms": ms[len(ms) // 2],
                    "min_ms": ms[0]})
    res.sort(key=lambda r: r["median_ms"])
    print(json.dumps({"graph": "reddit_like", "configs": res}, indent=1))


if __name__ == "__main__":
    main()
