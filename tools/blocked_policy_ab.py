"""Interleaved A/B of cache policies under the source-blocked copy_u + sum
(bench graph, F = 128): default, non-temporal output stores (the block's
out rows streamed past L2), every access non-temporal. Bits checked.

  python tools/blocked_policy_ab.py [--rounds 7]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import _ffi, data, kernel  # noqa: E402

POLICIES = {"auto": -1, "nt_out": 3, "nt_all": 1}


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
    ref = kernel.gspmm(adj, "copy_u", "sum", h)
    times = {p: [] for p in POLICIES}
    for _ in range(args.rounds):
        for name, pol in POLICIES.items():
            _ffi.check_call(_ffi.LIB.dglhip_set_cache_policy(pol))
            out = kernel.gspmm(adj, "copy_u", "sum", h)
            assert torch.equal(out, ref), name
            kernel.timing_enable(True)
            for _ in range(args.iters):
                kernel.gspmm(adj, "copy_u", "sum", h)
            ms, _ = kernel.timing_read()
            kernel.timing_enable(False)
            times[name].append(ms / args.iters)
    _ffi.check_call(_ffi.LIB.dglhip_set_cache_policy(-1))
    print(json.dumps({k: sorted(v)[len(v) // 2] for k, v in times.items()}))


if __name__ == "__main__":
    main()
