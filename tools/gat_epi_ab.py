"""A/B of the GAT backward's attention-gradient g-SDDMM (sliced dot with the
GAT epilogue): the epilogue's per-slot operands (attention, dropped copy)
loaded with the slot's gathers (default) or after the dot product
(dglhip_set_sddmm_variant(2), the earlier form), on the Reddit-shaped graph at
8 heads x 16, source-blocked: forward + backward wall ms and kernel ms per
step interleaved over rounds, gradients compared bit for bit (no dropout and
dropout 0.6 at a fixed seed).

  python tools/gat_epi_ab.py [--rounds 3] [--iters 10]
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
    ap.add_argument("--rounds", type=int, default=3)
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

    def step(p):
        for t in (ft, el, er):
            t.grad = None
        fs, z = kernel.gat_aggregate(adj, ft, el, er, attn_drop=p, seed=99)
        torch.autograd.backward([fs, z], [gout, gz])
        return [t.grad.clone() for t in (ft, el, er)]

    res = {"graph": "reddit_like", "heads": H, "head_dim": D, "bits_equal": {}, "rounds": []}
    for p in (0.0, 0.6):
        grads = []
        for v in (0, 2):
            kernel.set_sddmm_variant(v)
            grads.append(step(p))
        kernel.set_sddmm_variant(0)
        res["bits_equal"]["drop%.1f" % p] = all(torch.equal(a, b) for a, b in zip(*grads))
    print(json.dumps(res["bits_equal"]), flush=True)
    for _ in range(args.rounds):
        row = {}
        for p in (0.0, 0.6):
            for v in (0, 2):
                kernel.set_sddmm_variant(v)
                step(p)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    step(p)
                e.record()
                torch.cuda.synchronize()
                row["drop%.1f_v%d_wall_ms" % (p, v)] = s.elapsed_time(e) / args.iters
                kernel.timing_enable(True)
                for _ in range(args.iters):
                    step(p)
                ms, _ = kernel.timing_read()
                kernel.timing_enable(False)
                row["drop%.1f_v%d_kernel_ms" % (p, v)] = ms / args.iters
            kernel.set_sddmm_variant(0)
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
