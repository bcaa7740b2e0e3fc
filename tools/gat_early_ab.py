"""A/B of the fused GAT aggregation's automatic kernel choice (variant 0)
against the same choice with the LDS kernel's feature-row gathers issued
before each batch's attention (variant 3): the Reddit-shaped graph at 8 heads
x 16 (source-blocked) and a Pubmed-shaped graph at 8 x 8 and 8 x 3 (one
launch); kernel ms per call interleaved over rounds, outputs compared bit for
bit (no dropout, dropout 0.6 at a fixed seed, attention stored).

  python tools/gat_early_ab.py [--rounds 3] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
from dgl import data, kernel  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    kernel.timing_enable(True)
    for _ in range(iters):
        fn()
    ms, cnt = kernel.timing_read()
    kernel.timing_enable(False)
    return ms / iters


def cases_for(adj, n, H, D, dev):
    g = torch.Generator(device=dev).manual_seed(3)
    ft = torch.rand(n, H, D, device=dev, generator=g) * 2 - 1
    el = torch.rand(n, H, device=dev, generator=g) - 0.5
    er = torch.rand(n, H, device=dev, generator=g) - 0.5
    ftg = ft.clone().requires_grad_(True)
    return {
        "plain": (True, lambda: kernel.gat_aggregate(adj, ft, el, er)),
        "drop": (True, lambda: kernel.gat_aggregate(adj, ft, el, er, attn_drop=0.6, seed=1234)),
        "stored": (False, lambda: kernel.gat_aggregate(adj, ftg, el, er)),
    }


def run_graph(name, adj, n, H, D, dev, rounds, iters):
    cases = cases_for(adj, n, H, D, dev)
    res = {"graph": name, "heads": H, "head_dim": D, "rounds": [], "bits_equal": {}}
    for cname, (ng, fn) in cases.items():
        outs = []
        for v in (0, 3):
            kernel.set_gat_variant(v)
            with torch.no_grad() if ng else torch.enable_grad():
                outs.append([t.detach().clone() for t in fn()])
        kernel.set_gat_variant(0)
        res["bits_equal"][cname] = all(torch.equal(a, b) for a, b in zip(*outs))
    for _ in range(rounds):
        row = {}
        for cname, (ng, fn) in cases.items():
            for v in (0, 3):
                kernel.set_gat_variant(v)
                with torch.no_grad() if ng else torch.enable_grad():
                    row["%s_v%d_ms" % (cname, v)] = timed(fn, iters)
            kernel.set_gat_variant(0)
        res["rounds"].append(row)
    print(json.dumps(res), flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = []
    src, dst, n = data.reddit_like(device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    del src, dst
    out.append(run_graph("reddit_like", adj, n, 8, 16, dev, args.rounds, args.iters))
    del adj
    torch.cuda.empty_cache()
    src, dst, n = data.chung_lu(19717, 88651, 10.0, seed=0, device=dev)
    adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
    for D in (8, 3):
        out.append(run_graph("pubmed_shape", adj, n, 8, D, dev, args.rounds, args.iters * 10))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
