"""A/B of the copy_u + sum kernel's row gathers: global loads (a 64-bit
address per gather in flight, 72 VGPRs, 7 waves per SIMD) vs buffer
descriptors built from the wave-uniform row address (one 32-bit offset, 42
VGPRs, 8 waves per SIMD). Interleaved rounds in one process on the
Reddit-shaped graph and RMAT (heavy rows chunked); outputs compared bit for
bit.

  python tools/gather_mode_ab.py [--rmat-scale 26] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def ab(name, adj, h, rounds, iters=10):
    res = {0: [], 1: []}
    outs = {}
    for _ in range(rounds):
        for mode in (0, 1):
            kernel.set_gather_mode(mode)
            outs[mode] = kernel.gspmm(adj, "copy_u", "sum", h)
            torch.cuda.synchronize()
            kernel.timing_enable(True)
            for _ in range(iters):
                kernel.gspmm(adj, "copy_u", "sum", h)
            ms, n = kernel.timing_read()
            kernel.timing_enable(False)
            res[mode].append(ms / iters)
    kernel.set_gather_mode(0)
    same = bool(torch.equal(outs[0], outs[1]))
    return {"graph": name, "global_loads_ms": res[0], "buffer_descriptors_ms": res[1],
            "best_global": min(res[0]), "best_buffer": min(res[1]), "bit_identical": same}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rmat-scale", type=int, default=26)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = []
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev) * 2 - 1
    out.append(ab("reddit_like", adj, h, args.rounds))
    print(json.dumps(out[-1]), flush=True)
    del adj, h
    torch.cuda.empty_cache()
    kernel.set_row_split("auto")
    src, dst, n = data.rmat(args.rmat_scale, 16, seed=0, device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    h = torch.rand(n, 128, device=dev) * 2 - 1
    out.append(ab("rmat-%d" % args.rmat_scale, adj, h, args.rounds, iters=3))
    print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
