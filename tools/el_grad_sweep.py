"""Sweep of the GAT el-gradient's destination blocks (kernel._gat_el_grad,
_EL_GRAD_BLOCK_BYTES) on the Reddit-shaped graph at 8 heads: kernel ms per
call of the copy_edge sum of an E x H attention gradient along the transpose,
one launch vs blocks of 32-512 MiB of forward-slot values; bits compared with
the one launch.

  python tools/el_grad_sweep.py [--iters 10]
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
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    H = 8
    g = torch.rand(adj.fwd.nnz, H, device=dev) * 2 - 1
    res = {"graph": "reddit_like", "heads": H, "rows": []}
    old = kernel.set_blocked("off")
    ref = kernel._gat_el_grad(adj, g, H)
    kernel.set_blocked(old)
    for mib in (0, 32, 64, 128, 256, 512):
        if mib == 0:
            old = kernel.set_blocked("off")
        else:
            kernel._EL_GRAD_BLOCK_BYTES = mib << 20
        out = kernel._gat_el_grad(adj, g, H)
        same = bool(torch.equal(out, ref))
        torch.cuda.synchronize()
        kernel.timing_enable(True)
        for _ in range(args.iters):
            kernel._gat_el_grad(adj, g, H)
        ms, launches = kernel.timing_read()
        kernel.timing_enable(False)
        if mib == 0:
            kernel.set_blocked(old)
        row = {"block_MiB": mib, "kernel_ms": ms / args.iters,
               "launches": launches // args.iters, "bits_equal_one_launch": same}
        res["rows"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
